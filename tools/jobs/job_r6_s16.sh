#!/usr/bin/env bash
# r06 s16: LDS-staged conv operand prefetch depth 2 (BD) vs 1 on the replayed 8-pair graph (alternated, bit-identity),
# warp / lookup variant A/Bs, conv unit tests with depth 2 forced through the hook
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
V='bd1:lib.oflow_exp_set_conv_bstage=1/1;bd2:lib.oflow_exp_set_conv_bstage=2/1'
tools/gpu_job.sh \
 "300|r6s16_ab|VARIANTS='$V' ROUNDS=8 python -u tools/exp/run_graph_ab.py" \
 "180|r6s16_warp_ab|HOOK=oflow_exp_set_warp_strip CPW=1,2 python -u tools/exp/run_warp_ab.py" \
 "180|r6s16_lookup_ab|python -u tools/exp/run_lookup_buf_ab.py"
