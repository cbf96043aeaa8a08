#!/bin/bash
# Round 5, GPU call e: gemm_big row-error map (partial last m-tile), schedule 2 A/B, bench re-check.
set -o pipefail
O=gpurun_out/r5e
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
timeout -k 10 300 python -u scripts/gb_rows_diag.py > $O/rows_diag.log 2>&1
rc=$?; [ $rc -le 1 ] || stop rows_diag $rc
CASES="4096,4096,4096,0 4096,6144,4096,0 2944,6144,4096,0 4096,28672,4096,3 2944,28672,4096,3 4096,4096,14336,0"
for b in gemm_big_bench gemm_big_bench_s2 gemm_big_bench gemm_big_bench_s2; do
  echo "== $b" >> $O/s2_ab.log
  timeout -k 10 300 tools/$b $CASES >> $O/s2_ab.log 2>&1
  rc=$?; [ $rc -le 1 ] || stop $b $rc
done
KA_PREFILL_GEMM=blas timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_blas.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop bench_blas $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_auto.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop bench_auto $rc
echo ALL DONE
