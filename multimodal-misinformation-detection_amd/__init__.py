"""mmfd — MI355X-native (gfx950) hot path of sakdag/multimodal-misinformation-detection.

Drop-in mirror of the reference's fusion model / encoder / dataset / training-step API, computed by
hand-written HIP kernels (libmmfd_hip.so, C ABI in include/mmfd.h) launched through ctypes on the
current PyTorch HIP stream.
"""
__version__ = "0.1.0"

from . import kernels  # noqa: F401  (ctypes binding; loads lazily on first op)
