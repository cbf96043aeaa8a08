#!/bin/bash
# Round 6 session 2: the persistent decode kernel on the Llama-3-70B TP = 8 rank geometry (GQA 8,
# 12-slot rings, virtual communicator): parity tests, then the virtual-rank decode timing.
set -o pipefail
O=gpurun_out/r6s2_tp
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_model_gpu.py::test_persistent_decode_matches_kernel_chain_and_fp32" > $O/pytest_persistent.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/bench_virtual_rank.py --model llama3-70b --tp 8 --buckets 1,2,8 --reps 30 > $O/vrank70.log 2>&1
rc=$?; echo "vrank rc $rc"; exit $rc
