#!/bin/bash
# Round 6, call c: pp2 safe variants, the dispatched-plan stress (>= 500 launches per combination),
# the new stress / parity GPU tests.
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
P="512,28672,4096,19,1,0 256,128256,4096,19,1,0 256,6144,4096,19,2,2 384,28672,4096,19,1,0 256,128256,4096,2,1,0 256,128256,4096,3,1,0"
for rep in 1 2; do for s in pp0 pp1 pp2; do
  echo "== $s rep $rep" >> $O/time_pp.log
  timeout -k 10 120 tools/gemm_bench_$s $P >> $O/time_pp.log 2>&1 || exit 1
done; done
echo "pp A/B done"
timeout -k 10 600 python -u scripts/gm_plan_stress.py --launches 500 > $O/gm_plan_stress.log 2>&1 || { echo "stress rc=$?"; tail -5 $O/gm_plan_stress.log; exit 1; }
tail -3 $O/gm_plan_stress.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -v -k "gm_dispatched or gemm_big_alternating" --timeout 200 --timeout-method thread > $O/pytest_stress.log 2>&1
echo "stress tests rc=$?"
timeout -k 10 900 python -u -m pytest tests/test_model_full_depth_gpu.py -v -s --timeout 600 --timeout-method thread > $O/full_depth.log 2>&1
echo "full depth rc=$?"
grep -E "agreement|repeats|passed|failed|PASS|FAIL" $O/full_depth.log $O/pytest_stress.log | tail -30
