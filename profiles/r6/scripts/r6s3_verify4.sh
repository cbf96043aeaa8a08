#!/bin/bash
# Round 6 session 3: the full GPU suite, smoke() and the driver-form bench at the current tree.
set -o pipefail
O=gpurun_out/r6s3_verify4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_full.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest_gpu_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1
rc=$?; echo "bench rc $rc"; tail -1 $O/bench_driver.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
for c in 1 4 8; do
  timeout -k 10 300 python -u bench.py --concurrency $c --transport tcp --steps 5 --warmup 2 > $O/bench_c$c.log 2>&1
  rc=$?; echo "c$c rc $rc"; [ $rc -eq 0 ] || exit $rc
done
