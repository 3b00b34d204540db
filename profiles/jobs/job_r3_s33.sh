#!/usr/bin/env bash
# r03 s33: fused lookup + convc1 on 32-query workgroups: bit-identity test, convc1 tests, in-process step A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|s33_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_corr_convc1.py" \
 "400|s33_ab|ATTRS='{\"q64\": {\"lib:oflow_exp_set_convc1_qm\": 64}, \"q32\": {\"lib:oflow_exp_set_convc1_qm\": 32}}' SAMPLES=8 python -u tools/exp/attr_ab.py" \
 "200|s33_bench64|python -u bench.py --no-cpu-baseline" && \
tools/gpu_job.sh \
 "200|s33_bench32|python -u -c \"import sys; sys.path.insert(0, 'torch-optical-flow_amd'); sys.argv = ['bench.py', '--no-cpu-baseline']; from optical_flow import _native as N; N.load().oflow_exp_set_convc1_qm(32); import runpy; runpy.run_path('bench.py', run_name='__main__')\""
