#!/usr/bin/env bash
# Two separate rocprofv3 PMC passes (HBM reads, HBM writes) over a short bench run, restricted to the lookup kernels and the warp
# (the fused lookup + convc1 of the step and the API lookup leg timed after it). MI355X_MICROARCH.md §HBM: one counter
# group per pass, --kernel-trace only, each pass under its own hard time limit.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for ctr in TCC_EA0_RDREQ_sum WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "corr_convc1|corr_lookup_tiled|warp_strip" --output-format csv \
    -d gpurun_out/pmc/p$i -o run -- python3 bench.py --eager --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i ($ctr) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
