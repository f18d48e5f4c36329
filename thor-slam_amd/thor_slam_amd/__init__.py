"""MI355X-native visual-SLAM back end for the thor-slam ``SlamEngine`` interface.

Host side: this Python package (boundary types, calibration, synthetic sources, the engine).
Device side: ``libtslam_hip.so`` built from ``../csrc`` (hand-written HIP for gfx950), bound
through the C-ABI declared in ``include/tslam.h``.
"""

__version__ = "0.1.0"
