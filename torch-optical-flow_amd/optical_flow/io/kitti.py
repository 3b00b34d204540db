"""KITTI 16-bit PNG flow files (drop-in for optical_flow/io/kitti.py of the reference).

Like the reference these need opencv-python (kitti.py:8-19): without it both functions raise the reference's
ModuleNotFoundError. Encoding: channel values 64 * flow + 2^15 as uint16, third channel = valid mask, BGR order
(kitti.py:52-75)."""
from __future__ import annotations

from pathlib import Path
from typing import Tuple, Union

import numpy as np
import torch
from torch import Tensor

try:
    import cv2
except ModuleNotFoundError:
    cv2 = None


def _check_cv2_available():
    if not cv2:
        raise ModuleNotFoundError(
            "Reading and writing optical flow in KITTI format requires the opencv-python package."
            " To install it, run: pip install opencv-python-headless"
        )


def read_kitti(file: Union[str, Path], mask: bool = False) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    """KITTI PNG -> (2, H, W) flow [and (H, W) valid mask] CPU tensors (kitti.py:22-49)."""
    _check_cv2_available()
    raw = cv2.imread(str(file), cv2.IMREAD_ANYDEPTH | cv2.IMREAD_COLOR)
    raw = raw[:, :, ::-1].astype(np.float32)
    flow = (raw[:, :, :2] - 2 ** 15) / 64.0
    valid = raw[:, :, 2]
    flow_t = torch.tensor(np.ascontiguousarray(flow)).permute(2, 0, 1)
    valid_t = torch.tensor(np.ascontiguousarray(valid))
    return (flow_t, valid_t) if mask else flow_t


def write_kitti(file: Union[str, Path], flow: Union[Tensor, np.ndarray]) -> None:
    """(2, H, W) flow -> KITTI PNG (kitti.py:52-75)."""
    _check_cv2_available()
    if isinstance(flow, Tensor):
        flow = flow.detach().cpu().numpy()
    enc = 64.0 * flow.transpose((1, 2, 0)) + 2 ** 15
    enc = np.concatenate([enc, np.ones(enc.shape[:2] + (1,))], axis=-1).astype(np.uint16)
    cv2.imwrite(str(file), enc[..., ::-1])
