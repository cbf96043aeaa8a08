#!/bin/bash
# Round 5, GPU call t: gemm_big intermittent wrong rows 56-63 — clamped (duplicate-address) rows vs
# distinct rows, and M0 set once per 4-piece group vs for every LDS-DMA piece.
set -o pipefail
O=gpurun_out/r5t
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
CASES="4096,6144,4096,0 2944,6144,4096,0 4096,6144,4096,0 4096,1152,4096,0 4096,6144,4096,0 2944,6144,4096,0 4096,6144,4096,0 4096,1152,4096,0"
for v in c1 c1e m2 e; do
  echo "== $v" >> $O/m0.log
  GB_FULL=1 GB_FULL_REPS=10 GB_ROUNDS=1 timeout -k 10 300 tools/gemm_big_bench_$v $CASES >> $O/m0.log 2>&1
  rc=$?; [ $rc -le 1 ] || stop $v $rc
done
echo ALL DONE
