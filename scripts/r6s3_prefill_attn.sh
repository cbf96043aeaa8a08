#!/bin/bash
# Round 6 session 3: prefill attention with scalar block-table reads per tile vs the previous build.
set -o pipefail
O=gpurun_out/r6s3_pattn
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill or mixed_step or decode" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  timeout -k 10 200 python -u scripts/bench_prefill_attn.py 2>&1 | grep prefill > $O/new_$pass.log || exit 1
  KA_HIP_LIB_DIAG=1 KA_HIP_LIB=$GRAFT_REPO_ROOT/abtest/B/libkagent_hip.so timeout -k 10 200 python -u scripts/bench_prefill_attn.py 2>&1 | grep prefill > $O/old_$pass.log || exit 1
  echo "pass $pass new: $(cat $O/new_$pass.log) | old: $(cat $O/old_$pass.log)"
done
