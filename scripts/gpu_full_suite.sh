#!/bin/bash
# Round 5, GPU call m: the whole GPU suite at HEAD, then smoke().
set -o pipefail
O=gpurun_out/${GPU_OUT:-r5m}
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu_full.log 2>&1
rc=$?; [ $rc -le 1 ] || stop pytest $rc
echo "pytest rc $rc"
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop smoke $rc
echo ALL DONE
