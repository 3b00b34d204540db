#!/usr/bin/env bash
# r03 session 4: GPU parity of the native backward + stem-from-image, stem A/B, rocprof kernel trace of the bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "400|r3_s4_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_raft.py tests/test_gpu_ops.py" \
 "200|r3_s4_stem_ab|ATTRS='{\"patch\": {\"stem_from_image\": false}, \"image\": {\"stem_from_image\": true}}' python -u tools/exp/attr_ab.py" \
 "300|r3_s4_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_s4_prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline"
