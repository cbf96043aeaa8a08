#!/bin/bash
# Round 6 session 3: gemv_ring with batched X staging: the skinny / GEMV tests at the default and with the
# ring variant extended to 16 rows (KA_GEMV_MAX_M=16), then decode graph A/B of that switch.
set -o pipefail
O=gpurun_out/r6s3_gemv
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "skinny or gemv or linear or swiglu" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
KA_GEMV_MAX_M=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "skinny or gemv or linear or swiglu" > $O/pytest16.log 2>&1
rc=$?; echo "pytest16 rc $rc"; tail -1 $O/pytest16.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
for v in 4 16; do
  KA_GEMV_MAX_M=$v timeout -k 10 400 python -u scripts/bench_decode_graph.py --model llama3-8b --buckets 4,8,16 --reps 50 > $O/g8b_m${v}_$pass.log 2>&1 || exit 1
  KA_GEMV_MAX_M=$v timeout -k 10 500 python -u scripts/bench_decode_graph.py --model llama3-70b --tp 8 --buckets 8 --reps 30 > $O/tp8_m${v}_$pass.log 2>&1 || exit 1
  echo "max_m $v pass $pass: $(grep 'B=' $O/g8b_m${v}_$pass.log) | $(grep 'B=' $O/tp8_m${v}_$pass.log)"
done
done
