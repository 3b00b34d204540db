"""MI355X-native ``model`` package (drop-in for the reference's methods/raft/model).

Use exactly like the reference: put ``methods/raft`` on ``sys.path`` and ``from model import RAFT``. The
sibling ``optical_flow`` package (two directories up) is added to ``sys.path`` when it is not importable yet,
as an installed ``optical_flow`` would be for the reference.
"""
import os as _os
import sys as _sys

try:
    import optical_flow as _of  # noqa: F401
except ImportError:  # pragma: no cover - path bootstrap
    _sys.path.insert(0, _os.path.abspath(_os.path.join(_os.path.dirname(__file__), "..", "..", "..")))

from .corr import AlternateCorrBlock, CorrBlock  # noqa: E402
from .raft import RAFT  # noqa: E402
from .utils import InputPadder, bilinear_sampler, coords_grid, upflow8  # noqa: E402

__all__ = ["RAFT", "AlternateCorrBlock", "CorrBlock", "InputPadder", "bilinear_sampler", "coords_grid", "upflow8"]
