#!/bin/bash
# Round 6 session 3: the decode attention prologue / chunk-loop changes: kernel tests, the B = 256
# context sweep, the decode graph step at B = 1 / 8 / 256.
set -o pipefail
O=gpurun_out/r6s3_attn
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "decode or cascade or mixed_step" > $O/pytest_attn.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $O/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_decode_attn_ctx.py > $O/ctx_new.log 2>&1
rc=$?; echo "ctx rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/bench_decode_graph.py --model llama3-8b --buckets 1,8,256 --reps 50 > $O/graph_new.log 2>&1
rc=$?; echo "graph rc $rc"; exit $rc
