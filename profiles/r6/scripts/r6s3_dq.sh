#!/bin/bash
# Round 6 session 3: batched split-K slices in the fused decode attention prologue (the three
# reductions of a thread together; >4 slices 4 at a time) and in rmsnorm's remainder: tests, then
# same-box A/B against abtest/B on the 8B context sweep and the 70B TP = 8 rank at B = 1 / 8.
set -o pipefail
O=gpurun_out/r6s3_dq
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "decode or rmsnorm or cascade" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in new old; do
  if [ $v = old ]; then export KA_HIP_LIB_DIAG=1 KA_HIP_LIB=$GRAFT_REPO_ROOT/abtest/B/libkagent_hip.so; fi
  timeout -k 10 300 python -u scripts/bench_decode_attn_ctx.py --ctx 33,121,131 > $O/ctx_$v.log 2>&1 || exit 1
  timeout -k 10 500 python -u scripts/bench_decode_graph.py --model llama3-70b --tp 8 --buckets 1,8 --reps 30 > $O/tp8_$v.log 2>&1 || exit 1
  echo "$v: $(grep -h 'us$' $O/ctx_$v.log | awk '{print $3, $NF, $(NF-1)}' | tr '\n' ' ') | $(grep 'B=' $O/tp8_$v.log)"
done
