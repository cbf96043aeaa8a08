#!/bin/bash
# Round 6 session 3: 512-thread split-K RMSNorm for hidden 8192 (the 70B TP rank): tests, then A/B of the
# TP = 8 rank's B = 8 step against the previous commit's library (abtest/H2).
set -o pipefail
O=gpurun_out/r6s3_norm512
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_custom_allreduce_gpu.py -k "rmsnorm or norm or allreduce" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
for v in new old; do
  if [ $v = old ]; then L="KA_HIP_LIB_DIAG=1 KA_HIP_LIB=$GRAFT_REPO_ROOT/abtest/H2/libkagent_hip.so"; else L=""; fi
  env $L timeout -k 10 500 python -u scripts/bench_decode_graph.py --model llama3-70b --tp 8 --buckets 8,64 --reps 30 > $O/tp8_${v}_$pass.log 2>&1 || exit 1
  echo "$v $pass: $(grep 'B=' $O/tp8_${v}_$pass.log)"
done
done
