#!/bin/bash
# Round 6 session 3: latency-chain fixes in rmsnorm (split-K slices), masked argmax and decode attention:
# kernel + model tests, then the decode graph step per bucket and the driver-form headline.
set -o pipefail
O=gpurun_out/r6s3_lat
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py > $O/pytest_kern_model.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $O/pytest_kern_model.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/bench_decode_graph.py --model llama3-8b --buckets 1,4,8,256 --reps 50 > $O/graph.log 2>&1
rc=$?; echo "graph rc $rc"; grep "B=" $O/graph.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1
rc=$?; echo "bench rc $rc"; tail -1 $O/bench_driver.log | cut -c1-300; exit $rc
