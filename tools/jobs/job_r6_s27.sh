#!/usr/bin/env bash
# r06 s27: instance-norm partials without per-value bounds selects on whole tiles (no fma contraction); GPU suite, kernel traces of both builds, then
# alternated bench runs against HEAD (OFLOW_LIB=build/ab_old) on the same box
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
B="python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-step-flops"
P="rocprofv3 --kernel-trace --stats --output-format csv -o run"
tools/gpu_job.sh \
 "600|r6s27_pytest|python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "300|r6s27_prof_old|OFLOW_LIB=build/ab_old/liboflow_hip.so $P -d gpurun_out/r6s27_po -- python3 bench.py --eager --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "300|r6s27_prof_new|$P -d gpurun_out/r6s27_pn -- python3 bench.py --eager --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "60|r6s27_stats|cp \$(find gpurun_out/r6s27_po -name '*kernel_stats.csv' | head -1) gpurun_out/r6s27_old_kernel_stats.csv; cp \$(find gpurun_out/r6s27_pn -name '*kernel_stats.csv' | head -1) gpurun_out/r6s27_new_kernel_stats.csv; rm -rf gpurun_out/r6s27_po gpurun_out/r6s27_pn" \
 "120|r6s27_old1|OFLOW_LIB=build/ab_old/liboflow_hip.so $B" \
 "120|r6s27_new1|$B" \
 "120|r6s27_old2|OFLOW_LIB=build/ab_old/liboflow_hip.so $B" \
 "120|r6s27_new2|$B" \
 "120|r6s27_old3|OFLOW_LIB=build/ab_old/liboflow_hip.so $B" \
 "120|r6s27_new3|$B"
