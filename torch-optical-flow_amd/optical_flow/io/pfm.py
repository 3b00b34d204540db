"""PFM flow files of the Freiburg datasets (drop-in for optical_flow/io/pfm.py of the reference).

Header "PF\\n", "<w> <h>\\n", "<scale>\\n" (negative = little endian), then H rows of W (u, v, 0) float32, bottom
row first (pfm.py:79-104). The (H, W, 3) flipped payload of a ROCm tensor is built on the device (flow_pack)."""
from __future__ import annotations

import re
import sys
from pathlib import Path
from typing import Union

import numpy as np
import torch
from torch import Tensor

from ._payload import check_flow, payload


def read_pfm(file: Union[str, Path]) -> Tensor:
    """PFM file -> (2, H, W) fp32 CPU tensor (pfm.py:33-76). Raises RuntimeError for single-channel data, a non-PFM
    file or a malformed header, like the reference."""
    with open(file, "rb") as f:
        header = f.readline().rstrip()
        if header == b"Pf":
            raise RuntimeError("PFM file contains single-channel data. Cannot decode flow data.")
        if header != b"PF":
            raise RuntimeError("Not a PFM file.")
        dim_match = re.match(rb"^(\d+)\s(\d+)\s$", f.readline())
        if not dim_match:
            raise RuntimeError("Malformed PFM header. Cannot read spatial dimensions.")
        width, height = map(int, dim_match.groups())
        scale = float(f.readline().rstrip())
        endian = "<" if scale < 0 else ">"
        data = np.fromfile(f, endian + "f")
    data = np.reshape(data, (height, width, 3))[:, :, :2]
    data = np.flipud(data).transpose((2, 0, 1))
    return torch.tensor(data.astype(np.float32))


def write_pfm(file: Union[str, Path], flow: Union[Tensor, np.ndarray]) -> None:
    """(2, H, W) float32 flow -> PFM file (pfm.py:79-104)."""
    check_flow(flow)
    assert flow.dtype in (np.float32, torch.float32)
    _, h, w = flow.shape
    data = payload(flow, 3, True)
    scale = -1 if sys.byteorder == "little" else 1  # native-order float32 payload
    with open(file, "wb") as f:
        f.write("PF\n".encode())
        f.write(f"{w:d} {h:d}\n".encode())
        f.write(f"{scale:f}\n".encode())
        f.write(data.tobytes())
