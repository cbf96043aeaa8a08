#!/bin/bash
# Round 6 session 3: KV block copy with batched loads vs the previous commit's library (abtest/K).
set -o pipefail
O=gpurun_out/r6s3_kvcopy
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "block_copy or prefix or reuse" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  timeout -k 10 200 python -u scripts/bench_kv_copy.py > $O/new_$pass.log 2>&1 || exit 1
  KA_HIP_LIB_DIAG=1 KA_HIP_LIB=$GRAFT_REPO_ROOT/abtest/K/libkagent_hip.so timeout -k 10 200 python -u scripts/bench_kv_copy.py > $O/old_$pass.log 2>&1 || exit 1
  echo "pass $pass new: $(grep pairs $O/new_$pass.log | tr '\n' ' ') | old: $(grep pairs $O/old_$pass.log | tr '\n' ' ')"
done
