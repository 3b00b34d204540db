#!/usr/bin/env bash
# r06 s12: split-K for the motion conv and the GRU candidate convs (oflow_conv_s32_ex5): unit + RAFT GPU tests, then
# an in-process graph A/B (off / both / q only / motion only), then the default bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
V='off:update.KSPLIT_LAYERS=frozenset();on:update.KSPLIT_LAYERS=frozenset({"mo","q"});q:update.KSPLIT_LAYERS=frozenset({"q"});mo:update.KSPLIT_LAYERS=frozenset({"mo"})'
tools/gpu_job.sh \
 "400|r6s12_pytest|python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_conv_ksplit.py tests/test_gpu_conv_s32.py tests/test_gpu_raft.py -rf" \
 "300|r6s12_ab|VARIANTS='$V' python -u tools/exp/run_graph_ab.py" \
 "300|r6s12_bench|python -u bench.py --no-cpu-baseline"
