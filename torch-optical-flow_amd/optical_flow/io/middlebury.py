"""Middlebury .flo files (drop-in for optical_flow/io/middlebury.py of the reference).

Format: float32 magic 202021.25, int32 width, int32 height, then H rows of W interleaved (u, v) float32, little
endian (middlebury.py:60-71). ``write_middlebury`` writes the same bytes as the reference; the (H, W, 2) payload
of a ROCm tensor is built on the device (flow_pack kernel)."""
from __future__ import annotations

from pathlib import Path
from typing import Union

import numpy as np
import torch
from torch import Tensor

from ._payload import payload

MAGIC_NUMBER = 202021.25


def read_middleburry(file: Union[str, Path]) -> Tensor:
    """.flo file -> (2, H, W) fp32 CPU tensor (middlebury.py:11-40; the reference's spelling is kept).
    Raises RuntimeError on a wrong magic number."""
    with open(file, "rb") as f:
        magic = np.fromfile(f, np.float32, count=1)
        if magic.size != 1 or magic[0] != MAGIC_NUMBER:
            raise RuntimeError("Magic number incorrect. Invalid .flo file.")
        w = int(np.fromfile(f, np.int32, count=1)[0])
        h = int(np.fromfile(f, np.int32, count=1)[0])
        data = np.fromfile(f, np.float32, count=2 * w * h)
    # np.resize repeats a short payload cyclically, like the reference
    data = np.resize(data, (h, w, 2)).transpose((2, 0, 1))
    return torch.tensor(data)


read_middlebury = read_middleburry


def write_middlebury(file: Union[str, Path], flow: Union[Tensor, np.ndarray]) -> None:
    """(2, H, W) flow -> .flo file (middlebury.py:43-71)."""
    data = payload(flow, 2, False)
    h, w = data.shape[:2]
    with open(file, "wb") as f:
        f.write(np.array([MAGIC_NUMBER], np.float32).tobytes())
        f.write(np.array([w, h], np.int32).tobytes())
        f.write(data.tobytes())
