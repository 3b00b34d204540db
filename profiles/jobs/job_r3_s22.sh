#!/usr/bin/env bash
# r03 s22: stage-first-block output folded into its consumers: bit-identity vs HEAD, tests, layers, step A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
H=build/rev_head/_lib
tools/gpu_job.sh \
 "120|s22_dump_new|TAG=new python -u tools/exp/enc_dump.py" \
 "120|s22_dump_head|TAG=head OFLOW_LIB=$H/liboflow_hip.so OFLOW_OPS_LIB=$H/liboflow_torch.so python -u tools/exp/enc_dump.py" \
 "60|s22_cmp|python tools/exp/enc_dump.py --compare new head; rm -f gpurun_out/enc_*.pt" \
 "400|s22_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_raft.py tests/test_gpu_conv_s32.py" \
 "120|s22_layers|python -u tools/exp/run_encoder_layers.py" \
 "400|s22_ab_fold|SAMPLES=6 ATTRS='{\"fold\": {\"mod:model.extractor.FOLD_BLOCK0\": true}, \"nofold\": {\"mod:model.extractor.FOLD_BLOCK0\": false}, \"fold_\": {\"mod:model.extractor.FOLD_BLOCK0\": true}, \"nofold_\": {\"mod:model.extractor.FOLD_BLOCK0\": false}}' python -u tools/exp/attr_ab.py"
