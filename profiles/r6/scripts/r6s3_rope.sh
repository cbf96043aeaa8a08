#!/bin/bash
# Round 6 session 3: prefill RoPE + KV append window kernel with batched loads (in-tree, 4 items per
# batch; R8: 8) against the previous kernel (abtest/B), plus the rope / split-K kernel tests.
set -o pipefail
O=gpurun_out/r6s3_rope
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rope" > $O/pytest_rope.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $O/pytest_rope.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  timeout -k 10 200 python -u scripts/bench_rope.py > $O/rope_new_$pass.log 2>&1 || exit 1
  KA_HIP_LIB_DIAG=1 KA_HIP_LIB=$GRAFT_REPO_ROOT/abtest/R8/libkagent_hip.so timeout -k 10 200 python -u scripts/bench_rope.py > $O/rope_r8_$pass.log 2>&1 || exit 1
  KA_HIP_LIB_DIAG=1 KA_HIP_LIB=$GRAFT_REPO_ROOT/abtest/B/libkagent_hip.so timeout -k 10 200 python -u scripts/bench_rope.py > $O/rope_old_$pass.log 2>&1 || exit 1
done
grep -h "T=" $O/rope_*_1.log $O/rope_*_2.log
