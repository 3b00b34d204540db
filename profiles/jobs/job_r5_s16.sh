#!/usr/bin/env bash
# r05 s16: whole-step A/B of the fused kernel's quad mapping (in-tree) against the r04 kernel (build/rev_c1old, HEAD)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OLD="OFLOW_LIB=$PWD/build/rev_c1old/_lib/liboflow_hip.so OFLOW_OPS_LIB=$PWD/build/rev_c1old/_lib/liboflow_torch.so"
tools/gpu_job.sh \
 "200|r5s16_new1|python -u tools/exp/step_ab.py" \
 "200|r5s16_old1|env $OLD python -u tools/exp/step_ab.py" \
 "200|r5s16_new2|python -u tools/exp/step_ab.py" \
 "200|r5s16_old2|env $OLD python -u tools/exp/step_ab.py" \
 "200|r5s16_new3|python -u tools/exp/step_ab.py" \
 "200|r5s16_old3|env $OLD python -u tools/exp/step_ab.py"
