# PMC passes over the split-fp16 conv kernels (tools/convbench.py layers); one rocprofv3 run per counter set.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcc
timeout -k 10 120 python3 tools/convbench.py --no-lookup > gpurun_out/pmcc/convbench.json 2>gpurun_out/pmcc/convbench.err || exit 1
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA" "TCC_EA0_RDREQ_sum" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-include-regex "conv_s32" -d gpurun_out/pmcc/p$i -o run -- python3 tools/convbench.py --no-lookup --iters 3 > gpurun_out/pmcc/p$i.log 2>&1
  echo "pass $i rc=$?"
  python3 tools/pmc_db.py $(find gpurun_out/pmcc/p$i -name "*.db") --kernel conv_s32 > gpurun_out/pmcc/p$i.txt 2>&1
  find gpurun_out/pmcc/p$i -name "*.db" -delete
done
