#!/bin/bash
# Round 5, GPU call o: which split-tail configurations give wrong rows (full-matrix repeats)?
set -o pipefail
O=gpurun_out/r5o
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
run() {  # label, env, cases
  echo "== $1" >> $O/cfg.log
  env $2 GB_FULL=1 GB_FULL_REPS=10 GB_ROUNDS=1 timeout -k 10 300 tools/gemm_big_bench_m2 $3 >> $O/cfg.log 2>&1
  rc=$?; [ $rc -le 1 ] || stop $1 $rc
}
run tn6_2944 "X=1" "4096,6144,4096,0 2944,6144,4096,0 4096,6144,4096,0 2944,6144,4096,0"
run tn6_3072_exact "X=1" "4096,6144,4096,0 3072,6144,4096,0 4096,6144,4096,0 3072,6144,4096,0"
run tn6_4300 "X=1" "4096,6144,4096,0 4300,6144,4096,0 4096,6144,4096,0 4300,6144,4096,0"
run tn8_2944_forced "KA_GB_TN=8" "4096,6144,4096,0 2944,6144,4096,0 4096,6144,4096,0 2944,6144,4096,0"
run tn8_4300_n4096 "X=1" "4096,4096,4096,0 4300,4096,4096,0 4096,4096,4096,0 4300,4096,4096,0"
run tn8_swiglu_2944 "X=1" "4096,28672,4096,3 2944,28672,4096,3 4096,28672,4096,3 2944,28672,4096,3"
echo ALL DONE
