#!/usr/bin/env bash
# r05 s25: double-buffered halo in the register-direct convs: GPU suite + whole-step A/B against HEAD (build/rev_base25)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OLD="OFLOW_LIB=$PWD/build/rev_base25/_lib/liboflow_hip.so OFLOW_OPS_LIB=$PWD/build/rev_base25/_lib/liboflow_torch.so"
tools/gpu_job.sh \
 "600|r5s25_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|r5s25_new1|python -u tools/exp/step_ab.py" \
 "200|r5s25_old1|env $OLD python -u tools/exp/step_ab.py" \
 "200|r5s25_new2|python -u tools/exp/step_ab.py" \
 "200|r5s25_old2|env $OLD python -u tools/exp/step_ab.py" \
 "200|r5s25_new3|python -u tools/exp/step_ab.py" \
 "200|r5s25_old3|env $OLD python -u tools/exp/step_ab.py"
