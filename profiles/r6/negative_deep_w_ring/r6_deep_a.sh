#!/bin/bash
# Round 6, session 2: gemm_big DEEP (three-deep W ring) against the default schedule, same binary
# (KA_GB_DEEP env), each interleaved with rocBLAS; then a full-matrix correctness pass of DEEP.
set -o pipefail
O=gpurun_out/r6deep_a
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
C="256,28672,4096,3 384,28672,4096,3 4096,28672,4096,3 4096,4096,4096,0 4096,4096,14336,0 2944,28672,4096,3"
for v in 0 1 0 1; do
  echo "== KA_GB_DEEP=$v" >> $O/perf.log
  KA_GB_DEEP=$v GB_ROUNDS=5 timeout -k 10 240 tools/gemm_big_bench $C >> $O/perf.log 2>&1
  rc=$?; [ $rc -le 1 ] || stop perf$v $rc
done
echo "== full check DEEP" >> $O/full.log
KA_GB_DEEP=1 GB_FULL=1 GB_FULL_REPS=3 GB_ROUNDS=1 timeout -k 10 240 tools/gemm_big_bench 256,28672,4096,3 4077,4096,4096,0 4077,28672,4096,3 3000,4096,14336,0 1000,4096,512,0 >> $O/full.log 2>&1
rc=$?; [ $rc -le 1 ] || stop full $rc
echo ALL DONE
