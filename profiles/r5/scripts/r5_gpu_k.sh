#!/bin/bash
# Round 5, GPU call k: the persistent decode kernel at B = 2 (one weight stream for both sequences,
# one attention leader per sequence and KV group) — model tests, then the decode graph ladder at
# B = 1 / 2 / 4 with the persistent kernel capped at 1 and at 2.
set -o pipefail
O=gpurun_out/r5k
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "persistent" > $O/tests.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop tests $rc
KA_PERSISTENT_MAX_B=2 timeout -k 10 400 python -u scripts/bench_decode_graph.py --buckets 1,2,4 --persistent 1 > $O/ladder_pb2.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop ladder2 $rc
KA_PERSISTENT_MAX_B=1 timeout -k 10 400 python -u scripts/bench_decode_graph.py --buckets 1,2,4 --persistent 1 > $O/ladder_pb1.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop ladder1 $rc
echo ALL DONE
