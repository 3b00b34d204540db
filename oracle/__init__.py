"""ORACLE — CPU restatement of the reference RAFT inference hot path. TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this package,
and only as the checker / the timed CPU baseline. The product (``torch-optical-flow_amd/``) never imports,
calls or falls back to it: a product op on a tensor without the HIP library raises.

What it restates (reference = awaelchli/torch-optical-flow, read-only at /root/reference in the build container):
  * ``oracle.corr``     — CorrBlock build / pyramid / lookup, bilinear_sampler, coords_grid
                          (methods/raft/model/corr.py:37-87, methods/raft/model/utils.py:64-86), plus an
                          independent float64 pixel-space lookup for cross-checks.
  * ``oracle.operator`` — warp, warp_grid, scale, resize, normalize, denormalize, integrate
                          (optical_flow/operator/operator.py:8-165).
  * ``oracle.raft``     — the full RAFT forward (methods/raft/model/raft.py:64-147, extractor.py:35-231,
                          update.py:40-161, utils.py:38-91) on PyTorch-CPU fp32.

Pinning: ``tests/test_oracle_golden.py`` checks every function here against ``tests/golden/*.npz``, which
``tests/golden/gen_goldens.py`` produced by importing and running the reference itself on CPU in the build
container, plus the reference's own unit tests' exact vectors (tests/operator/test_operator.py:6-132).
Parity is therefore pinned (not "unpinned") for every row of SURVEY.md §8(a).
"""
