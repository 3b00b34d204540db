"""Flow -> file payload (H, W, C) fp32 for the writers. A ROCm tensor is re-laid out by the flow_pack kernel
(csrc/flow_io.hip) and copied to the host once, so the D2H copy moves exactly the file's bytes; a host array is
already where the file is written from and is only re-laid out (no arithmetic on either path)."""
from __future__ import annotations

from typing import Union

import numpy as np
import torch
from torch import Tensor

from .. import _native


def check_flow(flow: Union[Tensor, np.ndarray]) -> None:
    # the reference's asserts (read_write.py:69-70, middlebury.py:64-65)
    assert flow.ndim == 3
    assert flow.shape[0] == 2


def payload(flow: Union[Tensor, np.ndarray], channels: int, flip_rows: bool) -> np.ndarray:
    check_flow(flow)
    if isinstance(flow, Tensor) and flow.device.type == "cuda":
        packed = _native.flow_pack(flow.detach().unsqueeze(0), channels, flip_rows)[0]
        return packed.cpu().numpy()
    arr = flow.detach().numpy() if isinstance(flow, Tensor) else np.asarray(flow)
    arr = arr.astype(np.float32, copy=False).transpose(1, 2, 0)
    if channels == 3:
        arr = np.concatenate((arr, np.zeros_like(arr[..., :1])), -1)
    if flip_rows:
        arr = arr[::-1]
    return np.ascontiguousarray(arr)
