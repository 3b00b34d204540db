"""MI355X-native ``optical_flow`` (drop-in for awaelchli/torch-optical-flow's ``optical_flow`` package).

Re-exports the operator API of the reference (`optical_flow/__init__.py:2`). ``warp`` runs on a hand-written
gfx950 HIP kernel through the C ABI of ``liboflow_hip.so`` (include/oflow.h). The inference I/O of the reference
 is here too: ``flow2rgb``/``colorwheel`` on a fused colour-map kernel and ``read``/``write``
(Middlebury, PFM, KITTI) with the file payload laid out on the device.
"""
from .io.read_write import read, write
from .operator.operator import denormalize, integrate, normalize, resize, scale, warp, warp_grid
from .visualization.flow2rgb import colorwheel, flow2rgb

__all__ = ["colorwheel", "denormalize", "flow2rgb", "integrate", "normalize", "read", "resize", "scale", "warp",
           "warp_grid", "write"]
