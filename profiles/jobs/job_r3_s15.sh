#!/usr/bin/env bash
# r03 s15: register-direct conv weights (T > 1): tests, convbench vs the LDS-staged build, ablation, step A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
L() { echo "OFLOW_LIB=build/$1/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/$1/_lib/liboflow_torch.so"; }
tools/gpu_job.sh \
 "300|s15_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py tests/test_gpu_corr_convc1.py" \
 "200|s15_conv_new|python -u tools/convbench.py --no-lookup" \
 "200|s15_conv_blds|$(L blds) python -u tools/convbench.py --no-lookup" \
 "200|s15_abl8|$(L abl) python -u tools/convbench.py --no-lookup --ablate" \
 "120|s15_ab_new1|python -u tools/exp/step_ab.py" \
 "120|s15_ab_blds1|$(L blds) python -u tools/exp/step_ab.py" \
 "120|s15_ab_new2|python -u tools/exp/step_ab.py" \
 "120|s15_ab_blds2|$(L blds) python -u tools/exp/step_ab.py" \
 "120|s15_layers|python -u tools/exp/run_encoder_layers.py"
