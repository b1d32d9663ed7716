import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import pkgload  # noqa: E402

pkgload.load()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def amd():
    # torch's HIP runtime must initialise before the library's first HIP call in this process (after
    # it, torch reports "No HIP GPUs are available"); device_count() does not initialise the GPU
    import torch
    if torch.cuda.device_count() > 0:
        torch.cuda.init()
    return sys.modules["orb_slam2_amd"]
