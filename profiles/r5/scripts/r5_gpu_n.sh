#!/bin/bash
# Round 5, GPU call n: the split tail's intermittent wrong rows (rows 56-63 of a partial last m-tile,
# TN 6): full-matrix repeats over alternating shapes, per hand-off variant.
set -o pipefail
O=gpurun_out/r5n
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
CASES="4096,6144,4096,0 2944,6144,4096,0 777,6144,4096,0 2944,6144,4096,0 1000,1152,2048,0 2944,6144,4096,0 2944,28672,4096,3 2944,6144,4096,0"
for v in m2 m2p m3 m2; do
  echo "== $v" >> $O/tail_stress.log
  GB_FULL=1 GB_FULL_REPS=12 GB_ROUNDS=1 timeout -k 10 300 tools/gemm_big_bench_$v $CASES >> $O/tail_stress.log 2>&1
  rc=$?; [ $rc -le 1 ] || stop $v $rc
done
echo ALL DONE
