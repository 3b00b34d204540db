"""``optical_flow.read`` / ``optical_flow.write`` (drop-in for optical_flow/io/read_write.py of the reference):
same formats, dispatch, asserts and ValueError. Writers take the flow where it is: a ROCm tensor's file payload is
laid out on the device (csrc/flow_io.hip) and copied to the host once; readers return CPU tensors, like the
reference."""
from __future__ import annotations

from pathlib import Path
from typing import Any, Union

from torch import Tensor

from .kitti import read_kitti, write_kitti
from .middlebury import read_middleburry, write_middlebury
from .pfm import read_pfm, write_pfm

FORMATS = ["kitti", "middlebury", "pfm"]


def read(file: Union[str, Path], fmt="middlebury", **kwargs: Any) -> Union[Tensor, Any]:
    """Read a (2, H, W) flow from ``file`` in format ``fmt`` (read_write.py:13-40)."""
    if fmt == "kitti":
        return read_kitti(file, **kwargs)
    if fmt == "middlebury":
        return read_middleburry(file)
    if fmt == "pfm":
        return read_pfm(file)
    raise ValueError(f"Unknown format: {fmt}.")


def write(file: Union[str, Path], flow: Tensor, fmt="middlebury") -> None:
    """Write a (2, H, W) flow to ``file`` in format ``fmt`` (read_write.py:43-78)."""
    assert flow.ndim == 3
    assert flow.shape[0] == 2
    if fmt == "kitti":
        write_kitti(file, flow)
    elif fmt == "middlebury":
        write_middlebury(file, flow)
    elif fmt == "pfm":
        write_pfm(file, flow)
    else:
        raise ValueError(f"Unknown format: {fmt}")
