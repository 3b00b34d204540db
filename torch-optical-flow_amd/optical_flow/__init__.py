"""MI355X-native ``optical_flow`` (drop-in for awaelchli/torch-optical-flow's ``optical_flow`` package).

Re-exports the operator API of the reference (`optical_flow/__init__.py:2`). ``warp`` runs on a hand-written
gfx950 HIP kernel through the C ABI of ``liboflow_hip.so`` (include/oflow.h). File I/O (``read``/``write``) and
visualisation (``flow2rgb``/``colorwheel``) of the reference are outside this build's hot-path scope
(DESIGN.md "Out of scope").
"""
from .operator.operator import denormalize, integrate, normalize, resize, scale, warp, warp_grid

__all__ = ["denormalize", "integrate", "normalize", "resize", "scale", "warp", "warp_grid"]
