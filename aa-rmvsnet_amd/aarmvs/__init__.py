"""aarmvs — MI355X-native (gfx950) depth sweep of AA-RMVSNet.

The hot path (homography warp, inter-view aggregation, ConvLSTM U-Net sweep,
online WTA) runs in libaarmvs.so (HIP, C ABI: include/aarmvs.h).  The
reference-compatible Python API lives in the sibling ``models`` package.
"""
from ._lib import AarmvsError, LIB_PATH, lib  # noqa: F401

__version__ = "0.1.0"
