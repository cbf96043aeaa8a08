#!/bin/bash
# Round 5, GPU call f: split-tail hand-off modes on full matrices; mixed-step A/B hipBLASLt vs the
# prefill plan (QKV on gemm_big).
set -o pipefail
O=gpurun_out/r5f
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
for m in 1 2 3 0 1 2 3; do
  echo "== mode $m" >> $O/tail_modes.log
  GB_FULL=1 GB_FULL_REPS=4 GB_ROUNDS=1 timeout -k 10 300 tools/gemm_big_bench_m$m 2944,6144,4096,0 4096,1152,4096,0 2944,28672,4096,3 >> $O/tail_modes.log 2>&1
  rc=$?; [ $rc -le 1 ] || stop mode$m $rc
done
KA_PREFILL_GEMM=blas timeout -k 10 400 python -u scripts/phase_profile.py > $O/phase_blas.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop phase_blas $rc
timeout -k 10 400 python -u scripts/phase_profile.py > $O/phase_auto.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop phase_auto $rc
KA_PREFILL_GEMM=blas timeout -k 10 400 python -u scripts/phase_profile.py > $O/phase_blas2.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop phase_blas2 $rc
timeout -k 10 400 python -u scripts/phase_profile.py > $O/phase_auto2.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop phase_auto2 $rc
echo ALL DONE
