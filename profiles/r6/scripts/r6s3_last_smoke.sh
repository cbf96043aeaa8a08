#!/bin/bash
# Round 6 session 3: the in-tree library as rebuilt at the last commit: smoke() and the kernel tests.
set -o pipefail
O=gpurun_out/r6s3_last
mkdir -p $O
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc $rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py > $O/pytest_kernels.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest_kernels.log; exit $rc
