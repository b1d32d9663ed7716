"""Import helper: the package directory is named `orb-slam2-_amd` (not a valid
Python identifier), so it is registered under the module name `orb_slam2_amd`."""
import importlib.util
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent
PKG_DIR = ROOT / "orb-slam2-_amd"


def load():
    if "orb_slam2_amd" in sys.modules:
        return sys.modules["orb_slam2_amd"]
    spec = importlib.util.spec_from_file_location(
        "orb_slam2_amd", PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["orb_slam2_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
