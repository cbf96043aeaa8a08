#!/bin/bash
# Round 6 session 3: batched split-K slices in silu_mul / rope (ld4, ld8): tests, then same-box A/B
# against the previous commit's library (abtest/H) on the 70B TP = 8 rank at B = 8 and 8B B = 8 / 256.
set -o pipefail
O=gpurun_out/r6s3_silu
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "silu or rope or splitk or swiglu" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
for v in new old; do
  if [ $v = old ]; then L="KA_HIP_LIB_DIAG=1 KA_HIP_LIB=$GRAFT_REPO_ROOT/abtest/H/libkagent_hip.so"; else L=""; fi
  env $L timeout -k 10 500 python -u scripts/bench_decode_graph.py --model llama3-70b --tp 8 --buckets 8 --reps 30 > $O/tp8_${v}_$pass.log 2>&1 || exit 1
  env $L timeout -k 10 500 python -u scripts/bench_decode_graph.py --model llama3-8b --buckets 8,256 --reps 50 > $O/g8b_${v}_$pass.log 2>&1 || exit 1
  echo "$v $pass: $(grep 'B=' $O/tp8_${v}_$pass.log) | $(grep 'B=' $O/g8b_${v}_$pass.log)"
done
done
