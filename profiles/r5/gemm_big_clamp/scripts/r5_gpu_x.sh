#!/bin/bash
# Round 5, GPU call x: drain-at-barrier-1 (db1) with the DMA window ending at group 12 / 16 / 20
# instead of 28, against the counted-wait default (def) and def with the window at 16 (e16).
set -o pipefail
O=gpurun_out/r5x
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
CASES="2944,6144,4096,0 4096,4096,4096,0 4096,4096,14336,0 4096,28672,4096,3 4096,8192,28672,0"
for v in def db1 db1e12 db1e16 db1e20 e16 def db1e12 db1e16; do
  echo "== $v" >> $O/perf.log
  GB_ROUNDS=5 timeout -k 10 300 tools/gemm_big_bench_$v $CASES >> $O/perf.log 2>&1
  rc=$?; [ $rc -le 1 ] || stop $v $rc
done
echo ALL DONE
