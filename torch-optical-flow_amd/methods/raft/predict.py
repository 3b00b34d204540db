"""Folder-to-folder RAFT inference (drop-in for methods/raft/predict.py of the reference).

Same arguments and outputs as the reference's ``main`` (predict.py:39-95): flow between consecutive images of
``source`` (sorted by name), written to ``destination`` as ``{i:06d}.flo`` (Middlebury) and, with ``visualize``,
``{i:06d}.png`` = [image0 | image1 | flow2rgb(flow)] in torchvision's ``save_image`` grid layout (2-px black
padding).

The output side is built for the GPU: padding, unpadding, the .flo payload (flow_pack kernel) and the colour map
(flow2rgb kernels) run on the device on the model's stream; one non-blocking copy per file moves exactly the
bytes that are written into pinned host memory, and a writer thread waits on that copy's event and writes the
files while the GPU already runs the next pair. Differences from the reference: no jsonargparse/torchvision
(argparse and a 20-line grid writer instead), ``ext`` results are sorted like the unfiltered listing (the
reference keeps an un-indexable glob there), and ``checkpoint=None`` uses the deterministic synthetic weights.
"""
from __future__ import annotations

import argparse
import os
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import List, Optional, Tuple, Union

import numpy as np
import torch
from torch import Tensor
from torch.utils.data import DataLoader, Dataset

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from model import RAFT, synthetic  # noqa: E402
from model.utils import InputPadder  # noqa: E402

import optical_flow  # noqa: E402
from optical_flow import _native  # noqa: E402
from optical_flow.io.middlebury import MAGIC_NUMBER  # noqa: E402


class FlowInferenceDataset(Dataset):
    """Consecutive image pairs of a folder as (3, H, W) fp32 tensors in [0, 255] (predict.py:20-36)."""

    def __init__(self, folder: Union[Path, str], ext: Optional[str] = None) -> None:
        if ext is None:
            self.files = sorted(Path(folder, p) for p in os.listdir(folder))
        else:
            self.files = sorted(Path(folder).glob(f"*.{ext}"))

    def __getitem__(self, item: int) -> Tuple[Tensor, Tensor]:
        from PIL import Image

        img0 = torch.tensor(np.array(Image.open(self.files[item]))).permute(2, 0, 1)[:3].float()
        img1 = torch.tensor(np.array(Image.open(self.files[item + 1]))).permute(2, 0, 1)[:3].float()
        return img0, img1

    def __len__(self) -> int:
        return max(len(self.files) - 1, 0)


def image_grid(images: List[Tensor], padding: int = 2) -> Tensor:
    """torchvision.utils.make_grid(images, nrow=8, padding=2, pad_value=0) followed by save_image's conversion
    (x * 255 + 0.5, clamped, uint8), for up to 8 (3, H, W) images of one size -> (H', W', 3) uint8, on their
    device."""
    n = len(images)
    _, h, w = images[0].shape
    grid = torch.zeros((3, h + 2 * padding, n * (w + padding) + padding), device=images[0].device)
    for i, im in enumerate(images):
        x0 = padding + i * (w + padding)
        grid[:, padding:padding + h, x0:x0 + w] = im
    return grid.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8)


def _write_outputs(event: torch.cuda.Event, flo_path: Path, payload: Tensor, png_path: Optional[Path],
                   grid: Optional[Tensor], range_snapshot=None) -> None:
    event.synchronize()
    if range_snapshot is not None and range_snapshot.overflowed():
        # this pair's forward overflowed a split-fp16 operand: its flow is not valid, so nothing is written for it
        raise RuntimeError(f"predict: pair {flo_path.stem}: {_native.RANGE_ERROR}")
    h, w = payload.shape[:2]
    with open(flo_path, "wb") as f:
        f.write(np.array([MAGIC_NUMBER], np.float32).tobytes())
        f.write(np.array([w, h], np.int32).tobytes())
        f.write(payload.numpy().tobytes())
    if png_path is not None:
        from PIL import Image

        Image.fromarray(grid.numpy(), "RGB").save(png_path)


def main(
    source: str,
    destination: str,
    checkpoint: Optional[str] = None,
    ext: Optional[str] = None,
    overwrite: bool = False,
    iters: int = 24,
    visualize: bool = True,
    eval_mode: bool = False,
    num_workers: int = 4,
) -> int:
    """Predict flow for every consecutive pair in ``source`` and write it to ``destination`` (predict.py:39-95).
    ``eval_mode`` puts the model in eval mode; the reference never calls ``.eval()`` (cnet's batch norm then uses
    batch statistics), which stays the default. ``num_workers`` image-decoding processes (the reference's 4).
    Returns the number of pairs written."""
    if iters <= 0:
        raise ValueError("iters must be a positive integer")
    destination = Path(destination)
    destination.mkdir(parents=True, exist_ok=overwrite)
    dataset = FlowInferenceDataset(source, ext=ext)
    loader = DataLoader(dataset, batch_size=1, num_workers=num_workers, pin_memory=True)
    if not torch.cuda.is_available():
        raise RuntimeError("predict: this MI355X build runs RAFT on a ROCm GPU only (no CPU fallback)")
    device = torch.device("cuda", 0)
    if checkpoint is not None:
        model = RAFT.load_from_checkpoint(checkpoint)
    else:
        model = RAFT()
        model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model.to(device)
    if eval_mode:
        model.eval()

    # writes overlap the next pairs' inference on one writer thread, at most WRITES_IN_FLIGHT behind: each slot owns
    # its pinned host buffers (reused while the shape holds) and is waited on before reuse, which bounds host memory
    # and re-raises a failed write at the next pair instead of after the whole folder
    slots = [None] * WRITES_IN_FLIGHT
    count = 0
    with torch.inference_mode(), ThreadPoolExecutor(max_workers=1) as writer:
        for i, (img0, img1) in enumerate(loader):
            img0 = img0.to(device, non_blocking=True)
            img1 = img1.to(device, non_blocking=True)
            padder = InputPadder(img0.shape)
            padded0, padded1 = padder.pad(img0, img1)
            _, flow = model(padded0, padded1, iters=iters, test_mode=True)
            snap = model.last_range_snapshot  # this pair's own range status, checked by the writer before writing
            assert flow.shape[0] == 1
            flow = padder.unpad(flow)[0]

            slot = slots[i % WRITES_IN_FLIGHT]
            if slot is not None:
                slot["future"].result()
            else:
                slot = slots[i % WRITES_IN_FLIGHT] = {"payload": None, "grid": None, "future": None}
            payload_dev = _native.flow_pack(flow.unsqueeze(0), 2, False)[0]
            payload = _pinned(slot, "payload", payload_dev)
            grid = png = None
            if visualize:
                rgb = optical_flow.flow2rgb(flow)
                grid = _pinned(slot, "grid", image_grid([img0[0] / 255.0, img1[0] / 255.0, rgb]))
                png = destination / f"{i:06d}.png"
            done = torch.cuda.Event()
            done.record()
            slot["future"] = writer.submit(_write_outputs, done, destination / f"{i:06d}.flo", payload, png, grid, snap)
            count += 1
        for slot in slots:
            if slot is not None:
                slot["future"].result()
        model.check_range(device)  # the split-fp16 range guard of the last pairs' forwards (earlier ones: checked as
        # the loop went on, RAFT.range_guard "deferred")
    return count


WRITES_IN_FLIGHT = 3


def _pinned(slot: dict, key: str, src: torch.Tensor) -> torch.Tensor:
    """Copy ``src`` (device) into the slot's pinned host buffer ``key`` (allocated on first use or a shape change)
    without blocking the host."""
    buf = slot[key]
    if buf is None or buf.shape != src.shape or buf.dtype != src.dtype:
        buf = slot[key] = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
    buf.copy_(src, non_blocking=True)
    return buf


def _cli(argv=None) -> int:
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("source")
    ap.add_argument("destination")
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--ext", default=None)
    ap.add_argument("--overwrite", action="store_true")
    ap.add_argument("--iters", type=int, default=24)
    ap.add_argument("--visualize", type=lambda s: s.lower() in ("1", "true", "yes"), default=True)
    ap.add_argument("--eval_mode", action="store_true")
    ap.add_argument("--num_workers", type=int, default=4)
    a = ap.parse_args(argv)
    main(a.source, a.destination, a.checkpoint, a.ext, a.overwrite, a.iters, a.visualize, a.eval_mode, a.num_workers)
    return 0


if __name__ == "__main__":
    sys.exit(_cli())
