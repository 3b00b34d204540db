#!/usr/bin/env bash
# r06 s28 (final evidence on the final r06 tree: + early lane state, pack_s32 16-B stores, whole-tile partials): GPU suite, smoke, benches,
# PMC passes, MFMA-utilisation PMC passes, rocprof kernel trace + phases of the default bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "900|r6s28_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|r6s28_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r6s28_bench|python -u bench.py" \
 "200|r6s28_bench2|python -u bench.py --no-cpu-baseline" \
 "200|r6s28_bench_eager|python -u bench.py --eager --no-cpu-baseline" \
 "300|r6s28_bench_kitti|python -u bench.py --workload kitti --no-cpu-baseline" \
 "200|r6s28_bench_corr|python -u bench.py --workload corr --no-cpu-baseline" \
 "200|r6s28_bench_hd|python -u bench.py --workload hd --no-cpu-baseline" \
 "300|r6s28_pmc|bash tools/pmc_job.sh" \
 "60|r6s28_traffic|R=\$(find gpurun_out/pmc/p1 -name '*counter_collection.csv' | head -1); W=\$(find gpurun_out/pmc/p2 -name '*counter_collection.csv' | head -1); cp \$R gpurun_out/r6s28_pmc_rdreq.csv; cp \$W gpurun_out/r6s28_pmc_write_size.csv; python3 tools/pmc_traffic.py gpurun_out/r6s28_pmc_rdreq.csv gpurun_out/r6s28_pmc_write_size.csv sintel:8:corr_lookup_convc1 corr_convc1 && python3 tools/pmc_traffic.py gpurun_out/r6s28_pmc_rdreq.csv gpurun_out/r6s28_pmc_write_size.csv sintel:8:corr_lookup_api corr_lookup_tiled && python3 tools/pmc_traffic.py gpurun_out/r6s28_pmc_rdreq.csv gpurun_out/r6s28_pmc_write_size.csv sintel:8:warp warp_strip && cp profiles/lookup_traffic.json gpurun_out/r6s28_lookup_traffic.json; rm -rf gpurun_out/pmc" \
 "400|r6s28_pmcm|bash tools/pmc_mfma_job.sh" \
 "60|r6s28_pmcm_sum|python3 tools/pmc_mfma.py \$(find gpurun_out/pmcm/p1 -name '*counter_collection.csv' | head -1) \$(find gpurun_out/pmcm/p2 -name '*counter_collection.csv' | head -1) --json gpurun_out/r6s28_pmc_mfma.json; find gpurun_out/pmcm -name '*.csv' -size +20M -delete" \
 "300|r6s28_prof_graph|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6s28_profg -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "60|r6s28_profg_sum|cp \$(find gpurun_out/r6s28_profg -name '*kernel_stats.csv' | head -1) gpurun_out/r6s28_graph_kernel_stats.csv; python3 tools/exp/lane_overlap.py \$(find gpurun_out/r6s28_profg -name '*kernel_trace.csv' | head -1) > gpurun_out/r6s28_graph_overlap.txt; rm -rf gpurun_out/r6s28_profg" \
 "300|r6s28_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6s28_prof -o run -- python3 bench.py --eager --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "60|r6s28_phases|T=\$(find gpurun_out/r6s28_prof -name '*kernel_trace.csv' | head -1); python3 tools/step_phases.py \$T --steps 4 && python3 tools/prof_summary.py \$T --steps 6 --skip-last 2 > gpurun_out/r6s28_breakdown.txt; cp \$(find gpurun_out/r6s28_prof -name '*kernel_stats.csv' | head -1) gpurun_out/r6s28_kernel_stats.csv; rm -f \$T"
