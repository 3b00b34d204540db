#!/usr/bin/env bash
# Matrix-core utilisation of the step's MFMA kernels (split-fp16 convolutions, split pyramid, fused lookup + convc1):
# rocprofv3 PMC passes over a short bench run, one counter set per pass (MI355X_MICROARCH.md §rocprofv3 PMC slots:
# <= 8 SQ + <= 2 GRBM per pass), --kernel-trace-free counter collection only, each pass under its own hard limit.
# PMC collection serialises the dispatches, so the counters describe each kernel running alone.
# Output: gpurun_out/pmcm/p<i>/.../*counter_collection.csv ; summarise with tools/pmc_mfma.py.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcm
KRE="conv_s32_kernel|corr_pyramid_s32|corr_convc1"
i=0
for ctrs in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctrs --kernel-include-regex "$KRE" --output-format csv \
    -d gpurun_out/pmcm/p$i -o run -- python3 bench.py --eager --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcm/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
