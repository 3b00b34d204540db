#!/usr/bin/env bash
# r04 s1: GPU suite (batch goldens, range guard, warp backward mask), smoke, bench with the range guard sync / deferred /
# off, configs[1], [2], [4] on the current build, MFMA-utilisation PMC passes, rocprof kernel trace of the bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "900|r4s1_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|r4s1_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r4s1_bench|python -u bench.py" \
 "200|r4s1_bench_deferred|python -u bench.py --range-guard deferred --no-cpu-baseline" \
 "200|r4s1_bench_off|python -u bench.py --range-guard off --no-cpu-baseline" \
 "200|r4s1_bench_sync2|python -u bench.py --no-cpu-baseline" \
 "300|r4s1_bench_kitti|python -u bench.py --workload kitti" \
 "200|r4s1_bench_corr|python -u bench.py --workload corr" \
 "200|r4s1_bench_hd|python -u bench.py --workload hd" \
 "400|r4s1_pmcm|bash tools/pmc_mfma_job.sh" \
 "60|r4s1_pmcm_sum|python3 tools/pmc_mfma.py \$(find gpurun_out/pmcm/p1 -name '*counter_collection.csv' | head -1) \$(find gpurun_out/pmcm/p2 -name '*counter_collection.csv' | head -1) --json gpurun_out/r4s1_pmc_mfma.json; find gpurun_out/pmcm -name '*.csv' -size +20M -delete" \
 "300|r4s1_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4s1_prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "60|r4s1_phases|T=\$(find gpurun_out/r4s1_prof -name '*kernel_trace.csv' | head -1); python3 tools/step_phases.py \$T --steps 4 && python3 tools/prof_summary.py \$T --steps 6 --skip-last 2 > gpurun_out/r4s1_breakdown.txt; cp \$(find gpurun_out/r4s1_prof -name '*kernel_stats.csv' | head -1) gpurun_out/r4s1_kernel_stats.csv; rm -f \$T"
