#!/usr/bin/env bash
# r04 s5: kernel trace of the bench (kept) for a per-stream timeline of the encoder phase
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r4s5_prof|rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4s5_prof -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-step-flops --no-events" \
 "60|r4s5_keep|T=\$(find gpurun_out/r4s5_prof -name '*kernel_trace.csv' | head -1); python3 -c \"import csv,sys; r=list(csv.DictReader(open('\$T'))); w=csv.writer(open('gpurun_out/r4s5_trace_min.csv','w')); w.writerow(['s','e','stream','name']); [w.writerow([x['Start_Timestamp'],x['End_Timestamp'],x['Stream_Id'],x['Kernel_Name'][:90]]) for x in r]\"; rm -f \$T; ls -la gpurun_out/r4s5_trace_min.csv"
