#!/usr/bin/env bash
# r05 s17: packed hi/lo split (v_cvt_pk + v_fma_mix) in every S32 writer (conv epilogues and staging, encoder, s32_io):
# GPU suite + whole-step A/B against HEAD (build/rev_base17)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OLD="OFLOW_LIB=$PWD/build/rev_base17/_lib/liboflow_hip.so OFLOW_OPS_LIB=$PWD/build/rev_base17/_lib/liboflow_torch.so"
tools/gpu_job.sh \
 "600|r5s17_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|r5s17_new1|python -u tools/exp/step_ab.py" \
 "200|r5s17_old1|env $OLD python -u tools/exp/step_ab.py" \
 "200|r5s17_new2|python -u tools/exp/step_ab.py" \
 "200|r5s17_old2|env $OLD python -u tools/exp/step_ab.py" \
 "200|r5s17_new3|python -u tools/exp/step_ab.py" \
 "200|r5s17_old3|env $OLD python -u tools/exp/step_ab.py"
