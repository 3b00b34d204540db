"""RAFT 12-iteration inference throughput on MI355X (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload sintel|kitti|corr]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Both forms run N ranks. Under torchrun (WORLD_SIZE set) this process is one rank. Without WORLD_SIZE and with
--gpus N > 1, this process is only a launcher (``launch_ranks``): before any GPU call it starts N fresh rank processes
of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their environment), waits
for them, forwards rank 0's JSON line as its only stdout line and exits with the first non-zero rank exit code.

Default workload "sintel" = BASELINE configs[3] per rank: every GPU infers 8 Sintel pairs (436x1024, padded
440x1024 in predict.py's 'sintel' mode) per step, 12 GRU iterations, fp32, test_mode; the global batch is 8*N
pairs (weak scaling; N = 8 is configs[3]'s 64 pairs). A step is: rank 0 scatters the pairs over RCCL (inputs
resident in rank 0's HBM), every rank pads -> RAFT forward -> unpads, flows are gathered back to rank 0. With
N = 1 there is no collective. Synthetic frames (integer texture, known shift) and hash-generated weights: no
dataset or checkpoint is reachable offline.

Inputs: the 8 pairs of the reference-generated golden batch (tests/golden/raft_e2e_batch.npz: 'sintel8' / 'kitti8',
synthetic frames the repository's generator rebuilds bit for bit), tiled to the global batch.

Printed (rank 0, one JSON line): pairs/s for the whole job, the lookup kernel's roofline (algorithmic bytes per
launch / mean launch time from HIP events recorded on the launch stream inside the timed region), ``roofline.step``
(the whole step's executed f16 MFMA rate against the dense peak, counted per launch in one extra untimed forward),
the corr pyramid kernel's MFMA rate, ``epe_vs_reference`` (the LAST TIMED STEP's flows for the golden batch's pairs
against the reference's own flows for them), and the oracle (PyTorch-CPU restatement) timed on this host's cores on
the workload's per-GPU batch. ``--pairs-per-gpu 1 --iters 24`` is predict.py's batch-1 latency case.

r05: the RAFT workloads 'sintel' and 'kitti' replay each rank's forward from a HIP graph by default (model/graph.py:
the same kernels, both pair lanes, captured once before the timed region; inputs copied in per step): the same work
per step without the host's per-launch Python. The per-kernel timings then come from event-record nodes captured into
the graph around the timed launches (liboflow's native timing events; torch's refuse that on ROCm), read after the
timed region: they time its last replay. ``--eager`` times the eager forward instead.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "torch-optical-flow_amd")
for _p in (REPO, PKG, os.path.join(PKG, "methods", "raft")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "image-pairs/sec + corr-lookup HBM GB/s, RAFT 12-iter @ Sintel 1024×436"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_F32_PEAK_TFLOPS = 157.3  # dense fp32 MFMA (v_mfma_f32_32x32x2_f32), spec
MFMA_F16_PEAK_TFLOPS = 2500.0  # dense fp16 MFMA, spec (no sparsity)
PMC_TRAFFIC_FILE = os.path.join(REPO, "profiles", "lookup_traffic.json")
SPIN_CYCLES = 40_000_000  # torch.cuda._sleep ahead of the after-step legs: longer than the host's enqueue of their launches
BATCH_GOLDEN = os.path.join(REPO, "tests", "golden", "raft_e2e_batch.npz")
HD_GOLDEN = os.path.join(REPO, "tests", "golden", "raft_e2e_hd.npz")
# the reference forward's FLOPs per pair (12 iterations, measured with the torch profiler)
REF_GFLOP_PER_PAIR = {"sintel": 735.9, "kitti": 767.6}

WORKLOADS = {
    # name: (pairs per GPU, H, W, iters, padder mode, alternate_corr)           BASELINE.json configs[...]
    "sintel": (8, 436, 1024, 12, "sintel", False),  # [3] per rank (8 x 8 GPUs = 64); metric config
    "kitti": (8, 375, 1242, 12, "sintel", False),  # [2] KITTI 1242x375, batch 8, fp32
    "hd": (1, 1080, 1920, 12, "sintel", True),  # [4] 1080p, on-the-fly fp16 correlation
    "corr": (4, 1024, 1024, 12, None, False),  # [1] corr build + 12 lookups only, 128x128x256 fmaps, batch 4
}


def lookup_bytes(batch: int, dims, radius: int = 4, s_corr: int = 4) -> int:
    """B*N*[sum_l min(2r+2,H_l)*min(2r+2,W_l)*s_corr + 8 + L*(2r+1)^2*4] per launch."""
    h0, w0 = dims[0]
    n = h0 * w0
    p = 2 * radius + 2
    k = 2 * radius + 1
    per_q = sum(min(p, h) * min(p, w) * s_corr for h, w in dims) + 8 + len(dims) * k * k * 4
    return batch * n * per_q


def warp_leg(dev, reps: int = 20):
    """The flow-warp operator (`optical_flow.warp`, reference operator.py:8-33) at SURVEY §8(d)'s warp workload: frame
    (8, 3, 436, 1024), flow = normalize(N(0, 8^2) px) per pixel (seeded), default modes (bilinear, border,
    align_corners=False); timed after the timed region, ``reps`` launches back to back between one pair of HIP events
    on the launch stream (two frame/flow pairs
    alternating so that no launch finds its inputs in the Infinity Cache). Algorithmic bytes (2C + 2) * 4 per pixel
    (frame read + flow read + output write)."""
    import optical_flow
    from model import synthetic

    b, c, h, w = 8, 3, 436, 1024
    pairs = []
    for k in range(2):
        frame, _ = synthetic.synthetic_pair(b, h, w, seed=1 + k)
        flow = optical_flow.normalize(torch.from_numpy(synthetic.hash_normal(5 + k, (b, 2, h, w), 8.0)))
        pairs.append((frame.to(dev), flow.to(dev)))
    stream = torch.cuda.current_stream(dev)
    with torch.inference_mode():
        for fr, fl in pairs:
            optical_flow.warp(fr, fl)
        torch.cuda.synchronize(dev)
        # (as in lookup_api_leg: the launches back to back behind a spin kernel, one event pair around them)
        torch.cuda._sleep(SPIN_CYCLES)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(reps):
            fr, fl = pairs[i % 2]
            optical_flow.warp(fr, fl)
        e1.record(stream)
        torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    nbytes = (2 * c + 2) * 4 * b * h * w
    ach = nbytes / (ms * 1e-3) / 1e9
    return {"note": "optical_flow.warp (HIP warp_strip kernel, bilinear/border/align_corners=False) on frame "
                    "(8, 3, 436, 1024), flow normalize(N(0, 8^2) px), timed after the timed region; not part of the "
                    "RAFT step",
            "bound": "hbm", "launch_ms": round(ms, 5), "launches": reps, "algorithmic_bytes_per_launch": nbytes,
            "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic("sintel", 8, "warp"),
            "frac_traffic": frac_on_traffic(pmc_traffic("sintel", 8, "warp"), ms)}


def pyramid_cost(batch: int, dims, c: int = 256):
    h0, w0 = dims[0]
    n = h0 * w0
    flops = 2 * batch * n * n * c
    write = batch * n * sum(h * w for h, w in dims) * 4
    read = 2 * batch * n * c * 4
    return flops, write + read


def lookup_api_leg(ppg: int, dims, flow_low, dev, reps: int = 12):
    """The reference's lookup operator (CorrBlock.__call__, corr.py:56-77: NCHW fp32 out) on this workload's shapes,
    timed after the timed region (in the step the lookup runs inside convc1): a (ppg, 256, H/8, W/8) feature pair
    per pyramid (synthetic features, two pyramids alternating so that no launch finds its pyramid in the 256 MiB
    Infinity Cache), the step's own final coordinates (grid + its last low-res flow), ``reps`` launches back to back
    between one pair of HIP events on the launch stream. Roofline = SURVEY §8(d)'s algorithmic bytes / mean launch time."""
    from model import CorrBlock, synthetic
    from model.utils import coords_grid

    h0, w0 = dims[0]
    blocks = []
    for k in range(2):
        f1, f2 = synthetic.synthetic_fmaps(ppg, 256, h0, w0, stream=40 + k)
        blocks.append(CorrBlock(f1.to(dev), f2.to(dev)))
    coords = (coords_grid(ppg, h0, w0).to(dev) + flow_low[:ppg].float()).contiguous()
    st = torch.cuda.current_stream(dev)
    for i in range(2):
        blocks[i % 2](coords)
    torch.cuda.synchronize(dev)
    # the launches back to back, queued behind a spin kernel that keeps the GPU busy while the host enqueues them, with
    # one event pair around them: their average is the kernel plus the dispatch boundary between launches (r06: one
    # event pair per launch from an idle GPU added the host's enqueue latency, ~3 us; per launch behind a spin kernel
    # the event pair itself still added ~3 us to the 30 us warp against rocprof)
    torch.cuda._sleep(SPIN_CYCLES)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for i in range(reps):
        blocks[i % 2](coords)
    e1.record(st)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    ts = [ms] * reps
    nbytes = lookup_bytes(ppg, dims)
    ach = nbytes / (ms * 1e-3) / 1e9
    return {
        "note": "CorrBlock.__call__ (API form, NCHW fp32, corr_lookup_tiled kernel) on this workload's shapes and final "
        "coordinates, timed after the timed region; not part of the step (the step's lookup runs inside convc1)",
        "bound": "hbm", "launch_ms": round(ms, 5), "launches": len(ts), "algorithmic_bytes_per_launch": nbytes,
        "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
        "traffic": pmc_traffic("sintel" if h0 == 55 else "kitti", ppg, "corr_lookup_api"),
        "frac_traffic": frac_on_traffic(pmc_traffic("sintel" if h0 == 55 else "kitti", ppg, "corr_lookup_api"), ms),
    }


def fused_lookup_bytes(batch: int, dims, lanes: int, radius: int = 4) -> int:
    """Algorithmic HBM bytes of the fused lookup + convc1 per iteration over ``batch`` pairs in ``lanes`` launches:
    per query the lookup's window reads (SURVEY §8(d) term 1) + its coordinates (8 B) + the S32 output (256 channels
    x 4 B); per launch the level-regrouped weights (L * G k32 groups x 256 channels x 128 B)."""
    h0, w0 = dims[0]
    p = 2 * radius + 2
    g = ((2 * radius + 1) ** 2 + 31) // 32
    per_q = sum(min(p, h) * min(p, w) * 4 for h, w in dims) + 8 + 256 * 4
    return batch * h0 * w0 * per_q + lanes * len(dims) * g * 256 * 128


def fused_lookup_flops(batch: int, dims, radius: int = 4) -> int:
    """Executed f16 MFMA flops of the fused kernel per iteration: queries x (L * G * 32) x 256 x 2 x 3 split products."""
    g = ((2 * radius + 1) ** 2 + 31) // 32
    return batch * dims[0][0] * dims[0][1] * len(dims) * g * 32 * 256 * 2 * 3


def pmc_traffic(workload: str, ppg: int, kernel: str):
    """HBM bytes per launch of ``kernel`` measured by rocprofv3 PMC (FETCH_SIZE + WRITE_SIZE, the guide's gfx950
    corrections) on this build, as recorded in profiles/lookup_traffic.json by tools/pmc_traffic.py; None if absent."""
    if not os.path.exists(PMC_TRAFFIC_FILE):
        return None
    with open(PMC_TRAFFIC_FILE) as f:
        tr = json.load(f).get(f"{workload}:{ppg}:{kernel}")
    return tr.get("hbm_bytes_per_launch") if tr else None


def frac_on_traffic(traffic, launch_ms: float):
    """The launch's real HBM bytes (PMC, per launch) / its measured time, as a fraction of the HBM peak; None without
    PMC data."""
    if not traffic:
        return None
    return round(traffic / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)


def pyramid_entry(pk, ppg: int, dims, split: bool = False):
    """The corr pyramid kernel's rate. split: the RAFT forward's split-fp16 build (oflow_corr_pyramid_tiled_s32: three
    f16 MFMAs per product, so executed f16 flops = 3x the GEMM's, against the dense f16 peak); else fp32 MFMA."""
    pk_ms = mean_ms(pk)
    flops, nbytes = pyramid_cost(ppg, dims)
    exe = 3 * flops if split else flops
    peak = MFMA_F16_PEAK_TFLOPS if split else MFMA_F32_PEAK_TFLOPS
    tf = exe / (pk_ms * 1e-3) / 1e12
    return {
        "bound": "mfma",
        "kernel": "corr_pyramid_s32 (split-fp16 products)" if split else "corr_pyramid (fp32 MFMA)",
        "note": "in-step: runs after fnet; alone: tools/kbench.py",
        "launch_ms": round(pk_ms, 4),
        "achieved_tflops": round(tf, 2),
        "peak_tflops": peak,
        "frac": round(tf / peak, 4),
        "hbm_gbs": round(nbytes / (pk_ms * 1e-3) / 1e9, 1),
        "flops_per_launch": exe,
        "bytes_per_launch": nbytes,
    }


def mean_ms(events) -> float:
    return statistics.fmean(a.elapsed_time(b) for a, b in events)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cgroup_cpus():
    """CPUs this process's cgroup may use (cgroup v2 cpu.max quota / period, rounded up), or None without a quota."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q == "max":
            return None
        return max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        return None


def cpu_baseline(h: int, w: int, iters: int, pairs: int):
    """The oracle RAFT (PyTorch-CPU fp32 restatement of the reference, validated against its goldens) on this host:
    torch threads = the CPUs this process may run on (len(sched_getaffinity)), limited only by a cgroup
    CPU quota when one is set (more threads than the quota's CPUs just time-slice); 1 warm-up pair, then ``pairs``
    pairs as one batch (configs #1 and #3 / one 8-pair shard of #4 -- the workload's own per-GPU
    batch)."""
    from model import synthetic
    from oracle import raft as oraft

    affinity = len(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    threads = max(1, min(affinity, quota) if quota else affinity)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        model = oraft.RAFT().eval()
        model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
        img0, img1 = synthetic.synthetic_pair(pairs, h, w)
        padder = oraft.InputPadder(img0.shape)
        p0, p1 = padder.pad(img0, img1)
        with torch.inference_mode():
            model(p0[:1], p1[:1], iters=iters, test_mode=True)  # warm-up
            t = time.perf_counter()
            model(p0, p1, iters=iters, test_mode=True)
            sec = time.perf_counter() - t
    finally:
        torch.set_num_threads(prev)
    return {
        "value": round(pairs / sec, 4),
        "unit": "image-pairs/s",
        "cores": threads,
        "affinity_cpus": affinity,
        "cgroup_cpu_quota": quota,
        "cpu_model": _cpu_model(),
        "kind": "port",
        "sample": f"oracle RAFT (PyTorch-CPU fp32 restatement of the reference), {pairs} pair(s) {h}x{w} padded as one "
        f"batch, {iters} iters, test_mode, after a 1-pair warm-up: {sec:.2f} s ({sec / pairs:.2f} s/pair); "
        f"torch threads={threads} of {affinity} CPUs in the affinity mask (cgroup CPU quota: {quota or 'none'})",
    }


def batch_golden(workload: str, h: int, w: int, iters: int):
    """(tag, fixture) of the reference-generated batch golden matching this workload's frame size and iterations, or
    (None, None): 'sintel8' / 'kitti8' (tests/golden/gen_goldens.py BATCH_CASES: 8 pairs, 12 iterations) and 'hd1'
    (HD_CASES: one 1080x1920 pair, 12 iterations, the reference's dense fp32 CPU path)."""
    import numpy as np

    tag, path = {"sintel": ("sintel8", BATCH_GOLDEN), "kitti": ("kitti8", BATCH_GOLDEN),
                 "hd": ("hd1", HD_GOLDEN)}.get(workload, (None, None))
    if tag is None or not os.path.exists(path):
        return None, None
    g = np.load(path, allow_pickle=False)
    b, gh, gw, giters, s, seed = (int(v) for v in g[f"{tag}_cfg"])
    if (gh, gw, giters) != (h, w, iters):
        return None, None
    return tag, g


def step_epe(out, tag: str, g, n_pairs: int):
    """EPE of the timed step's own flows (``out`` = (flow_low, flow_up) of the last timed step, the global batch on
    rank 0) for its first ``n_pairs`` pairs -- which are the golden batch's pairs -- against the reference's flows."""
    b, h, w, iters, s, seed = (int(v) for v in g[f"{tag}_cfg"])
    n = min(n_pairs, b)
    low = out[0][:n].float().cpu()
    up = out[1][:n, :, ::s, ::s].float().cpu()
    el = torch.norm(low - torch.from_numpy(g[f"{tag}_low"][:n]), dim=1)
    eu = torch.norm(up - torch.from_numpy(g[f"{tag}_up"][:n]), dim=1)
    return {
        "case": f"golden '{tag}': the last timed step's flows for its first {n} pair(s) ({h}x{w}, {iters} iters; "
                f"the benchmarked batch's own pairs) vs the reference PyTorch-CPU flows for the same pairs",
        "pairs": n,
        "low_mean": float(el.mean()),
        "low_max": float(el.max()),
        "up_mean": float(eu.mean()),
        "up_max": float(eu.max()),
        "unit": "px",
        "tolerance": ("mean <= 2e-3, max <= 2e-2 px (SURVEY §8(c), fp16 on-the-fly corr)" if tag == "hd1"
                      else "mean <= 1e-4, max <= 1e-3 px (SURVEY §8(c))"),
    }


def golden_epe(model, dev, workload: str):
    """The reference's own flow for a golden pair (tests/golden/raft_e2e.npz, produced by the reference on CPU) vs this
    build's forward with the same weights, run through the benchmarked model before timing: EPE of the 1/8-res flow
    and of the (strided) full-res flow. Used where no batch golden matches the workload (hd, other iteration
    counts)."""
    import numpy as np

    from model import InputPadder, synthetic

    tag = "kitti" if workload == "kitti" else "sintel"
    g = np.load(os.path.join(REPO, "tests", "golden", "raft_e2e.npz"), allow_pickle=False)
    b, h, w, iters, s, seed = (int(v) for v in g[f"{tag}_cfg"])
    img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
    padder = InputPadder(img0.shape, mode=str(g[f"{tag}_mode"]))
    p0, p1 = (x.to(dev) for x in padder.pad(img0, img1))
    with torch.inference_mode():
        low, up = model(p0, p1, iters=iters, test_mode=True)
    up = padder.unpad(up)[..., ::s, ::s]
    el = torch.norm(low.float().cpu() - torch.from_numpy(g[f"{tag}_low"]), dim=1)
    eu = torch.norm(up.float().cpu() - torch.from_numpy(g[f"{tag}_up"]), dim=1)
    return {
        "case": f"golden '{tag}': {b} pair(s) {h}x{w}, {iters} iters, reference PyTorch-CPU flow",
        "low_mean": float(el.mean()),
        "low_max": float(el.max()),
        "up_mean": float(eu.mean()),
        "up_max": float(eu.max()),
        "unit": "px",
    }


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """``--gpus N`` (N > 1) outside torchrun: start N rank processes of this script and wait for them.

    The launcher itself never touches the GPU (it only imports torch, which initialises nothing) and never replaces
    itself (no exec): every rank is a fresh child process with RANK = LOCAL_RANK = r, WORLD_SIZE = N and a free
    MASTER_PORT on 127.0.0.1, and runs this script's rank path (one GPU each, RCCL). Rank 0's stdout JSON line is
    forwarded as the launcher's only stdout line; every other output line goes to stderr. When a rank exits non-zero
    the others are terminated (a peer blocked in a collective would otherwise wait forever) and the launcher returns
    that first non-zero exit code."""
    import subprocess
    import threading

    port = _free_port()
    procs, threads = [], []
    lock = threading.Lock()

    def pump(stream, r):
        for raw in iter(stream.readline, b""):
            line = raw.decode(errors="replace")
            json_line = False
            if r == 0 and line.startswith("{"):
                try:
                    json_line = "metric" in json.loads(line)
                except ValueError:
                    pass
            with lock:
                (sys.stdout if json_line else sys.stderr).write(line if json_line else f"[rank {r}] {line}")
                (sys.stdout if json_line else sys.stderr).flush()
        stream.close()

    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        p = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env,
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        procs.append(p)
        t = threading.Thread(target=pump, args=(p.stdout, r), daemon=True)
        t.start()
        threads.append(t)
    first_bad = 0
    try:
        pending = set(range(n))
        while pending:
            for r in sorted(pending):
                rc = procs[r].poll()
                if rc is None:
                    continue
                pending.discard(r)
                if rc != 0 and first_bad == 0:
                    first_bad = rc if rc > 0 else 128 - rc
                    print(f"bench: rank {r} exited with {rc}; stopping the other ranks", file=sys.stderr)
                    for q in pending:
                        procs[q].terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for t in threads:
            t.join(timeout=10)
    return first_bad


def _standin_rank(world: int, rank: int, fail_rank: int) -> int:
    """Test stand-in for a rank (``--standin-worker``, CPU only): a gloo group over the launcher's rendezvous, one
    all-reduce of (rank + 1), a per-rank line on stderr and rank 0's JSON line -- the launcher's plumbing without the
    GPU (tests/test_bench_launcher.py). ``fail_rank`` exits 3 before the rendezvous, leaving its peers blocked in
    it: the launcher must stop them and return 3."""
    if rank == fail_rank:
        print(f"standin rank {rank}: failing on purpose", file=sys.stderr, flush=True)
        return 3
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t)
    print(f"standin rank {rank} of {world}: sum {int(t.item())}", file=sys.stderr, flush=True)
    if rank == 0:
        print(f"not a json line from rank {rank}", flush=True)
        print(json.dumps({"metric": METRIC, "n_gpus": world, "rank_sum": int(t.item())}), flush=True)
    dist.destroy_process_group()
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="sintel", choices=sorted(WORKLOADS))
    ap.add_argument("--pairs-per-gpu", type=int, default=None)
    ap.add_argument("--iters", type=int, default=None, help="GRU iterations (default: the workload's 12)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-events", action="store_true", help="do not record per-kernel HIP events")
    ap.add_argument("--conv-events", action="store_true", help="also time every update-block conv launch")
    ap.add_argument("--update-impl", default="split", choices=["split", "fused", "module"])
    ap.add_argument("--graph", action="store_true",
                    help="replay each rank's forward from a HIP graph (model/graph.py: one launch per step); the default "
                         "for 'sintel' / 'kitti' with --inflight 1")
    ap.add_argument("--eager", action="store_true", help="run the eager forward (no HIP graph)")
    ap.add_argument("--lanes", type=int, default=None, help="RAFT.pair_lanes (default: the model's)")
    ap.add_argument("--no-conv-benchmark", action="store_true",
                    help="disable torch.backends.cudnn.benchmark (MIOpen exhaustive find of the conv algorithms)")
    ap.add_argument("--inflight", type=int, default=1,
                    help="steps in flight: step i is issued on stream i %% N (its own side streams), so step i+1's "
                         "encoders run beside step i's update loop (pairs are independent; every step's flows are its own)")
    ap.add_argument("--no-step-flops", action="store_true",
                    help="skip the untimed flop-counting forward (roofline.step), e.g. under a kernel-trace profiler")
    ap.add_argument("--no-comm-overlap", action="store_true",
                    help="N > 1: run scatter -> forward -> gathers back to back per step (default: the scatter of step "
                         "i+1 and the gathers of step i overlap step i's / i+1's forward, model/pair_sharding.py "
                         "infer_sharded_pipelined)")
    ap.add_argument("--range-guard", default=None, choices=["sync", "deferred", "off"],
                    help="RAFT.range_guard (default: the model's, 'deferred': checked after the timed region)")
    ap.add_argument("--standin-worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--standin-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])  # this process is only the launcher: no GPU call before this
    if args.standin_worker:
        return _standin_rank(int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
                             args.standin_fail_rank)
    if args.graph and args.eager:
        print("bench: --graph and --eager exclude each other", file=sys.stderr)
        return 2
    # graph replay by default for the RAFT workloads (one capture per rank; with --graph --inflight N, N captures,
    # step i replaying capture i %% N on stream i %% N: each capture owns its static buffers)
    args.graph = args.graph or (not args.eager and args.workload in ("sintel", "kitti") and args.inflight == 1
                                and args.update_impl == "split")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from model import RAFT, InputPadder, synthetic
    from model.pair_sharding import infer_sharded, infer_sharded_pipelined
    from optical_flow import _native
    # experiments only: OFLOW_EXP_CALLS="oflow_exp_set_bn64_8row=1;..." calls liboflow's int-argument experiment setters
    for call in filter(None, os.environ.get("OFLOW_EXP_CALLS", "").split(";")):
        name, val = call.split("=")
        if not name.startswith("oflow_exp_set_"):
            raise SystemExit(f"bench: OFLOW_EXP_CALLS takes oflow_exp_set_* setters, not {name}")
        fn = getattr(_native.load(), name)
        fn.argtypes, fn.restype = [ctypes.c_int], None
        fn(int(val))

    ppg, h, w, iters, pmode, alt = WORKLOADS[args.workload]
    ppg = args.pairs_per_gpu or ppg
    iters = args.iters or iters
    global_batch = ppg * world

    torch.backends.cudnn.benchmark = not args.no_conv_benchmark
    model = RAFT(alternate_corr=alt).eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    model.update_impl = args.update_impl
    if args.range_guard:
        model.range_guard = args.range_guard
    if args.lanes:
        model.pair_lanes = args.lanes

    img0 = img1 = None
    if args.workload == "corr":  # configs[1]: fmaps (B, 256, 128, 128) ~ N(0, 1.45^2), coords = grid + N(0, 4^2)
        from model import CorrBlock
        from model.utils import coords_grid

        f1, f2 = synthetic.synthetic_fmaps(ppg, 256, 128, 128, stream=0)
        f1, f2 = f1.to(dev), f2.to(dev)
        cgrid = (coords_grid(ppg, 128, 128) + torch.from_numpy(synthetic.hash_normal(1, (ppg, 2, 128, 128), 4.0))).to(dev)

        def corr_step():
            cb = CorrBlock(f1, f2)
            out = None
            for _ in range(iters):
                out = cb(cgrid)
            return out, out

    gtag, gfix = batch_golden(args.workload, h, w, iters) if args.workload != "corr" else (None, None)
    if args.workload != "corr" and rank == 0:
        # the golden batch's pairs (8 distinct pairs for sintel / kitti), tiled to the global batch, in rank 0's HBM
        npairs = int(gfix[f"{gtag}_cfg"][0]) if gtag else 2
        seed = int(gfix[f"{gtag}_cfg"][5]) if gtag else 0
        a0, a1 = synthetic.synthetic_pair(npairs, h, w, seed=seed)
        reps = -(-global_batch // npairs)
        img0 = a0.to(dev).repeat(reps, 1, 1, 1)[:global_batch].contiguous()
        img1 = a1.to(dev).repeat(reps, 1, 1, 1)[:global_batch].contiguous()
    padder = InputPadder((h, w), mode=pmode or "sintel")
    dims = _native.pyramid_dims((h + 7) // 8, (w + 7) // 8, 4)
    # without a batch golden for this workload: the 1-pair golden through the benchmarked model, before timing
    epe = golden_epe(model, dev, args.workload) if args.workload != "corr" and rank == 0 and not gtag else None
    shard_shape = (global_batch, 3, h, w)
    flow_shapes = ((2, dims[0][0], dims[0][1]), (2, h, w))

    def forward(s0, s1):
        p0, p1 = padder.pad(s0, s1)
        low, up = model(p0, p1, iters=iters, test_mode=True)
        return low, padder.unpad(up)

    fwd = forward
    graph_rec = None
    if args.graph and args.workload != "corr":
        from model.graph import GraphedRAFT

        # capture this rank's shard shape (padded), then every step copies the shard in and replays
        pp = padder.pad(*(torch.zeros((ppg, 3, h, w), device=dev),) * 2)
        # per-kernel timing inside the graph: native event-record nodes captured around the timed launches, re-recorded
        # by every replay (read after the timed region: they time its last replay)
        graph_rec = None if args.no_events else ({"_native": True, "*": True} if args.conv_events else {"_native": True})
        # one capture per step in flight (the first holds the timing nodes); fwd() replays them in turn, and issue(i)
        # runs step i on stream i % inflight, so consecutive replays of one capture stay ordered on one stream
        ngraphs = max(1, args.inflight) if world == 1 else 1
        with torch.inference_mode():
            graphs = [GraphedRAFT(model, pp[0], pp[1], iters=iters, recorder=graph_rec if g == 0 else None)
                      for g in range(ngraphs)]
        gturn = [0]

        def fwd(s0, s1):
            p0, p1 = padder.pad(s0, s1)
            graphed = graphs[gturn[0] % ngraphs]
            gturn[0] += 1
            low, up = graphed(p0, p1)
            # the graph's outputs are overwritten by the next replay; with N > 1 the pipelined driver's gathers send
            # private copies (model/pair_sharding.py infer_sharded_pipelined), so these may be returned as they are
            return low, padder.unpad(up)

    def step():
        if args.workload == "corr":
            return corr_step()
        if world > 1:
            return infer_sharded(fwd, img0, img1, dev, shape=shard_shape, flow_shapes=flow_shapes)
        return fwd(img0, img1)

    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(max(1, args.inflight) - 1)]

    def issue(i):
        with torch.cuda.stream(streams[i % len(streams)]):
            return step()

    # N > 1: communication overlapped with the forwards (scatter of step i+1 / gathers of step i on the RCCL stream)
    pipelined = world > 1 and args.workload != "corr" and not args.no_comm_overlap

    def run_steps(n):
        out = None
        if pipelined:
            for out in infer_sharded_pipelined(fwd, ((img0, img1) for _ in range(n)), dev, shard_shape, flow_shapes):
                pass
            return out
        for i in range(n):
            out = issue(i)
        return out

    with torch.inference_mode():
        nwarm = max(args.warmup, 1 if pipelined else len(streams))
        if args.graph and not pipelined:
            nwarm = -(-nwarm // len(streams)) * len(streams)  # the timed steps start at stream 0 / capture 0
        run_steps(nwarm)
        torch.cuda.synchronize(dev)
        # graph replays launch no Python: their per-kernel events are the graph's own nodes (graph_rec, captured above)
        rec = ({"*": True} if args.conv_events else {}) if not (args.no_events or args.graph) else None
        _native.set_event_recorder(rec)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out = run_steps(args.steps)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        _native.set_event_recorder(None)
        rec_forwards = args.steps  # forwards the recorder's events cover
        if args.graph and graph_rec is not None:
            rec, rec_forwards = graph_rec, 1  # the last replay's launches
        if getattr(model, "range_guard", "off") == "deferred":
            model.check_range(dev)  # every timed forward's split operands were in range (raises otherwise)
        if rank == 0 and gtag:
            epe = step_epe(out, gtag, gfix, global_batch)
        # one more (untimed) forward with the per-launch flop counter: the step roofline
        step_flops = None
        if args.workload != "corr" and not args.no_step_flops:
            cnt = {}
            _native.set_flop_counter(cnt)
            forward(img0[:ppg] if img0 is not None else torch.zeros((ppg, 3, h, w), device=dev),
                img1[:ppg] if img1 is not None else torch.zeros((ppg, 3, h, w), device=dev))
            _native.set_flop_counter(None)
            torch.cuda.synchronize(dev)
            step_flops = cnt

    # the RAFT forward builds its pyramid from split-fp16 features (split encoders + CorrBlock); the "corr" workload
    # calls the CorrBlock API (fp32 MFMA pyramid)
    split_pyr = model.split_corr and args.update_impl == "split" and args.workload != "corr" and not alt
    api_lookup = warp = None
    if rank == 0 and rec is not None and args.workload in ("sintel", "kitti") and not alt:
        api_lookup = lookup_api_leg(ppg, dims, out[0], dev)
        warp = warp_leg(dev)

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank == 0 and args.workload != "corr":
        assert out[1] is not None and out[1].shape == (global_batch, 2, h, w)
        assert torch.isfinite(out[1]).all()
    pairs = global_batch * args.steps
    line = {
        "metric": METRIC,
        "value": round(pairs / elapsed, 3),
        "unit": "image-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
        "ms_per_pair": round(1000.0 * elapsed / args.steps / ppg, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("fp16 features, fp32 accumulate (on-the-fly corr); " if alt
                  else "corr + convs split-fp16 (22-bit operands: fp16 hi + lo, 3 f16 MFMA per product, fp32 accumulate); "
                  "lookup fp32" if split_pyr
                  else "fp32 corr (fp32 MFMA); ")
        + ("" if split_pyr
           else "convs split-fp16 (22-bit operands: fp16 hi + lo, 3 MFMA per product, fp32 accumulate)"
           if args.update_impl == "split" else "update convs fp32 (MIOpen)"),
        "data": "synthetic (integer texture frames with a known (3, -1.5) px shift; hash-initialised weights)",
        "config": {
            "workload": (f"corr-build+{iters}-lookups-fmaps-{ppg}x256x128x128" if args.workload == "corr"
                         else f"raft-{iters}iter-{args.workload}-{h}x{w}" + ("-otf-fp16" if alt else "")),
            "pairs_per_gpu": ppg,
            "global_batch": global_batch,
            "iters": iters,
            "padded": f"{dims[0][0] * 8}x{dims[0][1] * 8}",
            "parallelism": f"pairs sharded over {world} GPU(s)"
            + ((", RCCL scatter/gather overlapped with the forwards" if pipelined else ", RCCL scatter/gather")
               if world > 1 else ""),
            "conv_benchmark": not args.no_conv_benchmark,
            "update_impl": args.update_impl,
            "hip_graph": bool(args.graph),
            "steps_in_flight": max(1, args.inflight),
        },
    }
    if rec and args.conv_events:
        convs = {k: v for k, v in rec.items() if k.startswith("conv") or k == "flow_prep"}
        line["conv_ms_per_step"] = {k: round(sum(a.elapsed_time(b) for a, b in v) / rec_forwards, 3) for k, v in convs.items()}
    if rec and alt:
        lk = rec.get("corr_lookup_otf", [])
        pp = rec.get("corr_otf_prepare", [])
        line["kernels"] = {
            "corr_lookup_otf": {"launch_ms": round(mean_ms(lk), 4), "launches": len(lk)},
            "corr_otf_prepare": {"launch_ms": round(mean_ms(pp), 4) if pp else None},
        }
    elif rec and rec.get("corr_lookup_convc1"):
        # the RAFT forward's lookup runs inside convc1 (csrc/corr_convc1.hip): one launch per lane per iteration
        lk = rec["corr_lookup_convc1"]
        pk = rec.get("corr_pyramid", [])
        lk_ms = mean_ms(lk)
        lanes = max(1, len(lk) // (iters * rec_forwards))
        lk_bytes = fused_lookup_bytes(ppg, dims, lanes) // lanes
        flops = fused_lookup_flops(ppg, dims) // lanes
        ach = lk_bytes / (lk_ms * 1e-3) / 1e9
        tf = flops / (lk_ms * 1e-3) / 1e12
        line["roofline"] = {
            "kernel": "corr_lookup_convc1 (the windowed lookup fused into convc1: gathers from the tiled pyramid, "
            "split-fp16 MFMA 1x1 conv, ReLU, S32 out; the lookup volume never reaches HBM)",
            "bound": "hbm",
            "achieved": round(ach, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(args.workload, ppg, "corr_lookup_convc1"),
            "frac_traffic": frac_on_traffic(pmc_traffic(args.workload, ppg, "corr_lookup_convc1"), lk_ms),
            "algorithmic_bytes_per_launch": lk_bytes,
            "launch_ms": round(lk_ms, 5),
            "launches": len(lk),
            "mfma": {"executed_f16_tflops": round(tf, 1), "peak_tflops": MFMA_F16_PEAK_TFLOPS,
                     "frac": round(tf / MFMA_F16_PEAK_TFLOPS, 4), "flops_per_launch": flops},
        }
        # compound bound: the launch cannot be shorter than its real (PMC) HBM bytes at peak bandwidth, nor than its
        # executed f16 MFMA work at the dense peak; frac = that bound / the measured launch time
        trf = line["roofline"]["traffic"]
        if trf:
            t_hbm = trf / (HBM_PEAK_GBS * 1e9) * 1e6
            t_mfma = flops / (MFMA_F16_PEAK_TFLOPS * 1e12) * 1e6
            line["roofline"]["compound"] = {"bound_us": round(max(t_hbm, t_mfma), 2), "hbm_us": round(t_hbm, 2),
                                            "mfma_us": round(t_mfma, 2),
                                            "frac": round(max(t_hbm, t_mfma) / (lk_ms * 1e3), 4)}
        line["kernels"] = {}
        if pk:
            line["kernels"]["corr_pyramid"] = pyramid_entry(pk, ppg, dims, split=split_pyr)
        if api_lookup is not None:
            line["kernels"]["corr_lookup_api"] = api_lookup
        if warp is not None:
            line["kernels"]["warp"] = warp
    elif rec and rec.get("corr_lookup"):
        lk = rec.get("corr_lookup", [])
        pk = rec.get("corr_pyramid", [])
        lk_ms = mean_ms(lk)
        # per launch: a step does `iters` full-batch lookups' worth of queries over len(lk)/steps launches
        lk_bytes = lookup_bytes(ppg, dims) * iters * args.steps // max(1, len(lk))
        ach = lk_bytes / (lk_ms * 1e-3) / 1e9
        traffic = pmc_traffic(args.workload, ppg, "corr_lookup")
        line["roofline"] = {
            "kernel": "corr_lookup" + ("_tiled_nhwc (RAFT forward: fp32 NHWC rows, convc1's input)"
                                       if args.workload != "corr" and args.update_impl == "split" else ""),
            "bound": "hbm",
            "achieved": round(ach, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": lk_bytes,
            "launch_ms": round(lk_ms, 5),
            "launches": len(lk),
        }
        if pk:
            line["kernels"] = {"corr_pyramid": pyramid_entry(pk, ppg, dims, split=split_pyr)}
    if step_flops and step_flops.get("exec_f16"):
        # whole-step roofline: per GPU, the flops one forward over this rank's ppg pairs issues, over the step time
        sec = elapsed / args.steps
        ex, us = step_flops["exec_f16"], step_flops["useful"]
        ref = REF_GFLOP_PER_PAIR.get(args.workload)
        step = {
            "note": "per GPU: matrix-core flops of one forward over the rank's pairs (counted per launch in an untimed "
                    "forward) / ms_per_step; executed = the f16 MFMAs issued (3 split products, channel padding to "
                    "32-channel groups and output blocks included); useful = fp32-equivalent flops of the layers' real "
                    "channels as executed (after Q11's skipped mask heads and the hoisted GRU context term)",
            "executed_f16_flops": ex,
            "executed_f16_tflops": round(ex / sec / 1e12, 1),
            "peak_tflops": MFMA_F16_PEAK_TFLOPS,
            "frac": round(ex / sec / 1e12 / MFMA_F16_PEAK_TFLOPS, 4),
            "useful_fp32eq_flops": us,
            "useful_fp32eq_gflop_per_pair": round(us / ppg / 1e9, 1),
            "useful_fp32eq_tflops": round(us / sec / 1e12, 1),
            "fma_f32_flops": step_flops.get("fma_f32", 0),
        }
        if ref and h == WORKLOADS[args.workload][1]:
            rt = ref * 1e9 * ppg / sec / 1e12
            step["reference_gflop_per_pair"] = ref
            step["reference_equivalent_tflops"] = round(rt, 1)
            step["reference_equivalent_frac_of_fp32_mfma"] = round(rt / MFMA_F32_PEAK_TFLOPS, 4)
        line.setdefault("roofline", {})["step"] = step
    if epe is not None:
        line["epe_vs_reference"] = {k: (round(v, 8) if isinstance(v, float) else v) for k, v in epe.items()}
    if rank == 0 and not args.no_cpu_baseline and args.workload in ("sintel", "kitti"):
        # after every rank's timing (the all-reduce above): the oracle on rank 0's host cores, a bounded sample
        line["cpu_baseline"] = cpu_baseline(h, w, iters, ppg)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
