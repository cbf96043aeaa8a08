#!/bin/bash
# Round 5, GPU call j: grouped gemm_big for the MoE prefill experts — kernel tests, then the Mixtral
# block at 1024 / 4096 / 8192 tokens against the sorted hipBLASLt path and the grouped ring kernel.
set -o pipefail
O=gpurun_out/r5j
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "moe or gemm_big" > $O/tests.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop tests $rc
timeout -k 10 400 python -u scripts/bench_moe_prefill.py > $O/moe_prefill.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop bench $rc
echo ALL DONE
