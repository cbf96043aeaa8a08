#!/bin/bash
# Round 6 session 2: the persistent decode kernel's in-kernel all-reduce (TP = 2 processes sharing the
# GPU), the persistent parity tests, the one-shot collective tests.
set -o pipefail
O=gpurun_out/r6s2_tp
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  "tests/test_tp_single_gpu.py::test_tp_persistent_decode_in_kernel_allreduce_two_ranks" \
  "tests/test_model_gpu.py::test_persistent_decode_matches_kernel_chain_and_fp32" \
  tests/test_custom_allreduce_gpu.py \
  "tests/test_tp_single_gpu.py::test_tp_processes_one_gpu_graphs_oneshot_collectives" > $O/pytest_tp_ar.log 2>&1
rc=$?; echo "pytest rc $rc"; exit $rc
