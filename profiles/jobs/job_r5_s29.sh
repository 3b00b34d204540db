#!/usr/bin/env bash
# r05 s29: flow_prep_tiled with coalesced 16-B chunks: GPU suite + whole-step A/B against HEAD (build/rev_base29)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OLD="OFLOW_LIB=$PWD/build/rev_base29/_lib/liboflow_hip.so OFLOW_OPS_LIB=$PWD/build/rev_base29/_lib/liboflow_torch.so"
tools/gpu_job.sh \
 "600|r5s29_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|r5s29_new1|python -u tools/exp/step_ab.py" \
 "200|r5s29_old1|env $OLD python -u tools/exp/step_ab.py" \
 "200|r5s29_new2|python -u tools/exp/step_ab.py" \
 "200|r5s29_old2|env $OLD python -u tools/exp/step_ab.py" \
 "200|r5s29_new3|python -u tools/exp/step_ab.py" \
 "200|r5s29_old3|env $OLD python -u tools/exp/step_ab.py"
