#!/bin/bash
# Round 6, call e: full-depth parity against the fp32 truth; the TP path with split-K partials
# reduced inside the one-shot all-reduce + RMSNorm (2-rank IPC test, multi-process TP token tests,
# the collective's cost inside a captured graph); the 70B TP = 8 virtual-rank decode steps.
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_model_full_depth_gpu.py -v -s --timeout 600 --timeout-method thread > $O/full_depth.log 2>&1
echo "full depth rc=$?"; grep -E "agreement|repeats|passed|failed" $O/full_depth.log | tail -12
timeout -k 10 400 python -u -m pytest tests/test_custom_allreduce_gpu.py tests/test_tp_single_gpu.py -v --timeout 300 --timeout-method thread > $O/pytest_tp.log 2>&1
echo "tp tests rc=$?"; grep -E "passed|failed|PASS|FAIL" $O/pytest_tp.log | tail -8
timeout -k 10 300 python -u scripts/bench_custom_ar.py --world 2 > $O/custom_ar_w2.log 2>&1; echo "ar w2 rc=$?"; tail -6 $O/custom_ar_w2.log
timeout -k 10 300 python -u scripts/bench_custom_ar.py --world 8 --rows 1,8,64 > $O/custom_ar_w8.log 2>&1; echo "ar w8 rc=$?"; tail -5 $O/custom_ar_w8.log
timeout -k 10 600 python -u scripts/bench_virtual_rank.py --model llama3-70b --tp 8 --buckets 1,8,64,256 > $O/vrank70.log 2>&1; echo "vrank rc=$?"; tail -12 $O/vrank70.log
