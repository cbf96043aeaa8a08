#!/bin/bash
# Round 5, first GPU call: smoke (full depth), the full-depth parity tests, the gemm_big / gemm_mfma
# tests touched by the ADVICE fixes, the gemm_big vs rocBLAS shapes, then the driver-form bench.
# Every GPU step has its own time limit; a fault / abort / timeout ends the script.
set -o pipefail
O=gpurun_out/r5a
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop smoke $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_model_full_depth_gpu.py -s > $O/pytest_full_depth.log 2>&1
rc=$?; [ $rc -le 1 ] || stop full_depth $rc
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big or gemm_mfma or swiglu or plan" > $O/pytest_kernels.log 2>&1
rc=$?; [ $rc -le 1 ] || stop kernels $rc
timeout -k 10 300 tools/gemm_big_bench 4096,6144,4096,0 2944,6144,4096,0 4096,4096,4096,0 4096,4096,14336,0 4096,28672,4096,3 4080,6144,4096,0 4080,4096,4096,4 4080,4096,14336,4 > $O/gemm_big_bench.log 2>&1
rc=$?; [ $rc -le 1 ] || stop gemm_big_bench $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop bench $rc
echo ALL DONE
