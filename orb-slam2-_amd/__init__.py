"""MI355X-native ORB-SLAM2 hot path: ORBextractor / ORBmatcher /
Optimizer::LocalBundleAdjustment / Optimizer::PoseOptimization over hand-written gfx950 HIP kernels.
Import as `orb_slam2_amd` (see pkgload.py)."""
from . import _abi  # noqa: F401
from .extractor import ORBextractor  # noqa: F401
from .matcher import ORBmatcher, Frame, LocalMapPoints, ComputeDistinctiveDescriptors, Fuse, FuseSim3, SearchBySim3, \
    SearchForTriangulation  # noqa: F401
from .optimizer import Optimizer, LocalBA, LocalBAGroup, PoseOptimization  # noqa: F401
from .stereo import ComputeStereoMatches  # noqa: F401
from .vocabulary import ORBVocabulary  # noqa: F401
