#!/usr/bin/env bash
# r05 s37: the tiled flow head staging two channel groups per pass: its tests, then graph bench A/B against the HEAD
# library (build/rev_head, tools/build_rev.sh HEAD head), alternated
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OLD="OFLOW_LIB=build/rev_head/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/rev_head/_lib/liboflow_torch.so"
tools/gpu_job.sh \
 "300|r5s37_test|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py -k flow_head2" \
 "300|r5s37_new1|python -u bench.py --no-cpu-baseline" \
 "300|r5s37_old1|$OLD python -u bench.py --no-cpu-baseline" \
 "300|r5s37_new2|python -u bench.py --no-cpu-baseline" \
 "300|r5s37_old2|$OLD python -u bench.py --no-cpu-baseline" \
 "300|r5s37_new3|python -u bench.py --no-cpu-baseline" \
 "300|r5s37_old3|$OLD python -u bench.py --no-cpu-baseline"
