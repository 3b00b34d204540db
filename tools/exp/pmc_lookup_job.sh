set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM" "TCC_EA0_RDREQ_sum" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-include-regex "lookup" -d gpurun_out/pmc/p$i -o run -- python3 tools/exp/pmc_lookup.py > gpurun_out/pmc/p$i.log 2>&1
  echo "pass $i rc=$?"
done
