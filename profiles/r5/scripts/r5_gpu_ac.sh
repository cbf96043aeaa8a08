#!/bin/bash
# Round 5, GPU call ac: gemm_big drained-schedule knobs (DMA window end 18-24, barrier-1 group 5/6),
# then the headline bench at low concurrency (p50 latency at C = 1 / 2 / 4 / 8).
set -o pipefail
O=gpurun_out/r5ac
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
CASES="2944,6144,4096,0 4096,4096,4096,0 4096,4096,14336,0 4096,28672,4096,3 4096,8192,28672,0"
for v in d20 d18 d22 d24 b5 b6 d20; do
  echo "== $v" >> $O/perf.log
  GB_ROUNDS=5 timeout -k 10 300 tools/gemm_big_bench_$v $CASES >> $O/perf.log 2>&1
  rc=$?; [ $rc -le 1 ] || stop $v $rc
done
for c in 1 2 4 8; do
  timeout -k 10 300 python -u bench.py --concurrency $c --steps 20 --warmup 3 > $O/bench_c$c.log 2>&1 || stop bench_c$c $?
done
echo ALL DONE
