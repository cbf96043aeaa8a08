#!/bin/bash
# Round 5, GPU call l: full-depth parity incl. the B = 2 persistent kernel; the persistent kernel's
# phase breakdown at B = 1 and B = 2.
set -o pipefail
O=gpurun_out/r5l
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_model_full_depth_gpu.py > $O/full_depth.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop full_depth $rc
timeout -k 10 400 python -u scripts/bench_decode_graph.py --buckets 1,2 --persistent 1 > $O/phases.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop phases $rc
echo ALL DONE
