#!/usr/bin/env bash
# r03 s32: final round evidence: GPU suite, smoke, bench, rocprof kernel trace + phases, PMC traffic (convc1, API lookup,
# warp), bench with the regenerated traffic
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "700|s32_pytest|python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|s32_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|s32_bench|python -u bench.py" \
 "300|s32_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s32_prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline" \
 "60|s32_phases|T=\$(find gpurun_out/s32_prof -name '*kernel_trace.csv' | head -1); python3 tools/step_phases.py \$T --steps 4 && python3 tools/prof_summary.py \$T --steps 6 --skip-last 2 > gpurun_out/s32_breakdown.txt; cp \$(find gpurun_out/s32_prof -name '*kernel_stats.csv' | head -1) gpurun_out/s32_kernel_stats.csv; rm -f \$T" \
 "300|s32_pmc|bash tools/pmc_job.sh" \
 "60|s32_traffic|R=\$(find gpurun_out/pmc/p1 -name '*counter_collection.csv' | head -1); W=\$(find gpurun_out/pmc/p2 -name '*counter_collection.csv' | head -1); cp \$R gpurun_out/s32_pmc_rdreq.csv; cp \$W gpurun_out/s32_pmc_write_size.csv; python3 tools/pmc_traffic.py gpurun_out/s32_pmc_rdreq.csv gpurun_out/s32_pmc_write_size.csv sintel:8:corr_lookup_convc1 corr_convc1 && python3 tools/pmc_traffic.py gpurun_out/s32_pmc_rdreq.csv gpurun_out/s32_pmc_write_size.csv sintel:8:corr_lookup_api corr_lookup_tiled && python3 tools/pmc_traffic.py gpurun_out/s32_pmc_rdreq.csv gpurun_out/s32_pmc_write_size.csv sintel:8:warp warp_strip && cp profiles/lookup_traffic.json gpurun_out/s32_lookup_traffic.json; rm -rf gpurun_out/pmc" \
 "300|s32_bench2|python -u bench.py"
