#!/usr/bin/env bash
# Write-path counters of the split pyramid (full kernel and its epilogue-only ablation) under run_pyr_stagger_ab.py
# (EPI_ONLY=1): one counter set per pass, each pass under its own hard limit (<= 4 TCC, 2 TA, 2 TD, 4 TCP, 8 SQ).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp SAMPLES=1 EPI_ONLY=1
OUT=gpurun_out/pmcpyr
mkdir -p $OUT
i=0
for ctrs in \
  "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
  "TCC_WRITE_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_LEVEL_sum TCC_BUSY_sum TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "corr_pyramid_s32" --output-format csv \
    -d $OUT/p$i -o run -- python3 tools/exp/run_pyr_stagger_ab.py > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
