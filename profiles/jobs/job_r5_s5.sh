#!/usr/bin/env bash
# r05 s5: the VALU-lean fused lookup + convc1 (variant 4) vs the r04 kernel: in-process A/B (bit identity), stamps, PMC
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r5s5_pmc
tools/gpu_job.sh \
 "200|r5s5_c1ab|VARIANTS=1,4 python -u tools/exp/run_c1_variant_ab.py" \
 "200|r5s5_stamps|VARIANTS=1,4 python -u tools/exp/run_c1_stamps_variants.py" \
 "120|r5s5_pmc1|VARIANTS=1,4 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex corr_convc1 --output-format csv -d gpurun_out/r5s5_pmc/p1 -o run -- python3 tools/exp/run_c1_variant_ab.py" \
 "120|r5s5_pmc2|VARIANTS=1,4 timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-include-regex corr_convc1 --output-format csv -d gpurun_out/r5s5_pmc/p2 -o run -- python3 tools/exp/run_c1_variant_ab.py" \
 "60|r5s5_pmcsum|python3 tools/pmc_mfma.py \$(find gpurun_out/r5s5_pmc/p1 -name '*counter_collection.csv' | head -1) \$(find gpurun_out/r5s5_pmc/p2 -name '*counter_collection.csv' | head -1) --json gpurun_out/r5s5_pmc_mfma.json"
