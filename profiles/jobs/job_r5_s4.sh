#!/usr/bin/env bash
# r05 s4: fused lookup + convc1 variants 1 / 2 / 3: per-workgroup clock stamps, then two PMC passes over the in-process
# A/B (each kernel variant alone: SQ wave-state / MFMA busy; instruction mix / LDS bank conflicts)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r5s4_pmc
tools/gpu_job.sh \
 "200|r5s4_stamps|VARIANTS=1,2,3 python -u tools/exp/run_c1_stamps_variants.py" \
 "120|r5s4_pmc1|timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex corr_convc1 --output-format csv -d gpurun_out/r5s4_pmc/p1 -o run -- python3 tools/exp/run_c1_variant_ab.py" \
 "120|r5s4_pmc2|timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-include-regex corr_convc1 --output-format csv -d gpurun_out/r5s4_pmc/p2 -o run -- python3 tools/exp/run_c1_variant_ab.py" \
 "60|r5s4_pmcsum|python3 tools/pmc_mfma.py \$(find gpurun_out/r5s4_pmc/p1 -name '*counter_collection.csv' | head -1) \$(find gpurun_out/r5s4_pmc/p2 -name '*counter_collection.csv' | head -1) --json gpurun_out/r5s4_pmc_mfma.json"
