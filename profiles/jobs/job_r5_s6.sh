#!/usr/bin/env bash
# r05 s6: GRU epilogue addend pass as 16-B LDS accesses (conflict fix): tests, convbench A/B vs the base build, step A/B,
# PMC LDS conflicts of the step's conv kernels
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
B="OFLOW_LIB=build/rev_base/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/rev_base/_lib/liboflow_torch.so"
mkdir -p gpurun_out/r5s6_pmc
tools/gpu_job.sh \
 "400|r5s6_tests|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "200|r5s6_cb_new|python -u tools/convbench.py" \
 "200|r5s6_cb_base|env $B python -u tools/convbench.py" \
 "200|r5s6_ab1_new|python -u tools/exp/step_ab.py" \
 "200|r5s6_ab1_base|env $B python -u tools/exp/step_ab.py" \
 "200|r5s6_ab2_new|python -u tools/exp/step_ab.py" \
 "200|r5s6_ab2_base|env $B python -u tools/exp/step_ab.py" \
 "150|r5s6_pmc2|timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-include-regex conv_s32_kernel --output-format csv -d gpurun_out/r5s6_pmc/p2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-step-flops" \
 "60|r5s6_pmcsum|python3 tools/pmc_mfma.py \$(find gpurun_out/r5s6_pmc/p2 -name '*counter_collection.csv' | head -1) --json gpurun_out/r5s6_pmc_lds.json; find gpurun_out/r5s6_pmc -name '*.csv' -size +20M -delete"
