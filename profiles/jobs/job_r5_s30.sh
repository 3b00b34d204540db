#!/usr/bin/env bash
# r05 s30: upper bound of batching norm_stats: the step with its 30 launches replaced by two fills (wrong flows, timing
# only), interleaved with the product; plus the new timing-event-node GPU test
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s30_test|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_raft.py -k timing_event" \
 "200|r5s30_base1|python -u tools/exp/step_ab.py" \
 "200|r5s30_skip1|OFLOW_EXP_SKIP_NORM_STATS=1 python -u tools/exp/step_ab.py" \
 "200|r5s30_base2|python -u tools/exp/step_ab.py" \
 "200|r5s30_skip2|OFLOW_EXP_SKIP_NORM_STATS=1 python -u tools/exp/step_ab.py"
