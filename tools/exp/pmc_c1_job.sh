#!/usr/bin/env bash
# Memory-pipe counters of the fused lookup + convc1 kernel and its experiment variants (run_c1_variant_ab.py under
# rocprofv3 --pmc, one counter set per pass, each pass under its own hard limit; <= 2 TA, 2 TD, 4 TCP, 4 TCC, 8 SQ).
# Output: gpurun_out/pmcc1/p<i>/.../*counter_collection.csv ; summarise with tools/exp/pmc_c1_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcc1
mkdir -p $OUT
export VARIANTS="${VARIANTS:-1,7}"
i=0
for ctrs in \
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "corr_convc1" --output-format csv \
    -d $OUT/p$i -o run -- python3 tools/exp/run_c1_variant_ab.py > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
