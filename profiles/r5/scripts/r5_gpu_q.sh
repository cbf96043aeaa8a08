#!/bin/bash
# Round 5, GPU call q: split tail TN 6 wrong rows — diagnostic builds: d1 drains all vector memory at the
# top of every unit, d2 retires each unit (vmcnt(0) + barrier) after its epilogue.
set -o pipefail
O=gpurun_out/r5q
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
CASES="4096,6144,4096,0 2944,6144,4096,0 4096,6144,4096,0 2944,6144,4096,0 4096,6144,4096,0 2944,6144,4096,0"
for v in m2 d1 d2; do
  echo "== $v" >> $O/diag.log
  GB_FULL=1 GB_FULL_REPS=10 GB_ROUNDS=1 timeout -k 10 300 tools/gemm_big_bench_$v $CASES >> $O/diag.log 2>&1
  rc=$?; [ $rc -le 1 ] || stop $v $rc
done
echo ALL DONE
