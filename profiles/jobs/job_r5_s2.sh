#!/usr/bin/env bash
# r05 s2: 8-wave fused lookup + convc1 (A/B vs the 4-wave kernel, convc1 tests, GPU suite, bench), then two-lane graph
# capture probes (no side streams in the lanes; lane buffers on main with HIP API log)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r5s2_c1ab|python -u tools/exp/run_c1_variant_ab.py" \
 "600|r5s2_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "300|r5s2_bench|python -u bench.py --no-cpu-baseline" \
 "240|r5s2_probe_noside|VARIANT=noside PAIRS=8 python -X faulthandler -u tools/exp/graph_lanes_probe.py" \
 "240|r5s2_probe_initmain|AMD_LOG_LEVEL=3 VARIANT=initmain PAIRS=8 python -X faulthandler -u tools/exp/graph_lanes_probe.py"
