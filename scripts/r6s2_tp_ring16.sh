#!/bin/bash
# GQA-8 per-wave attention output in the leader's idle ring: 16-slot rings (B = 1) / 14 (B = 2) for the 70B
# TP rank.  Parity tests, then the virtual-rank timing and the phase stamps.
set -o pipefail
O=gpurun_out/r6s2_ring16
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  "tests/test_model_gpu.py::test_persistent_decode_matches_kernel_chain_and_fp32" \
  "tests/test_tp_single_gpu.py::test_tp_persistent_decode_in_kernel_allreduce_two_ranks" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/bench_virtual_rank.py --model llama3-70b --tp 8 --buckets 1,2,8 --reps 30 > $O/vrank70.log 2>&1
rc=$?; echo "vrank rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/bench_decode_graph.py --model llama3-70b --tp 8 --buckets 1,2 --persistent 1 --reps 30 > $O/stamps70.log 2>&1
rc=$?; echo "stamps rc $rc"; exit $rc
