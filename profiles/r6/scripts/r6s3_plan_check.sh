#!/bin/bash
# Round 6 session 3: the re-tuned decode plan in the tree: the dispatched-plan LDS-DMA stress test, the
# model tests, and the driver-form bench.
set -o pipefail
O=gpurun_out/r6s3_plan_check
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_model_full_depth_gpu.py -k "dispatched or decode or persistent or parity or agreement" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver_$pass.log 2>&1
  rc=$?; echo "bench $pass rc $rc"; tail -1 $O/bench_driver_$pass.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
done
