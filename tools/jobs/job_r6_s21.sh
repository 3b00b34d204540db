#!/usr/bin/env bash
# r06 s21: the committed conv loop built with a raised full-unroll threshold (the input-normalising 8-row conv unrolled);
# GPU suite on the new build, then alternated bench runs against the r06 s17 build (OFLOW_LIB=build/ab_old) on the same box
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
B="python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-step-flops"
tools/gpu_job.sh \
 "600|r6s21_pytest|python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "120|r6s21_old1|OFLOW_LIB=build/ab_old/liboflow_hip.so $B" \
 "120|r6s21_new1|$B" \
 "120|r6s21_old2|OFLOW_LIB=build/ab_old/liboflow_hip.so $B" \
 "120|r6s21_new2|$B" \
 "120|r6s21_old3|OFLOW_LIB=build/ab_old/liboflow_hip.so $B" \
 "120|r6s21_new3|$B" \
 "120|r6s21_eold|OFLOW_LIB=build/ab_old/liboflow_hip.so $B --eager" \
 "120|r6s21_enew|$B --eager"
