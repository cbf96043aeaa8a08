#!/bin/bash
# Round 5, GPU call d: tail hand-off fix, barrier-1 placement A/B, PMC of gemm_big vs rocBLAS (O 4096^3),
# plan re-write with the small-batch SwiGLU decision + the prefill plan, decode ladder, bench.
set -o pipefail
O=gpurun_out/r5d
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big or lm_head or swiglu" > $O/pytest_kernels.log 2>&1
rc=$?; [ $rc -le 1 ] || stop kernels $rc
CASES="4096,4096,4096,0 4096,6144,4096,0 2944,6144,4096,0 4096,28672,4096,3 2944,28672,4096,3 4096,4096,14336,0"
for b in gemm_big_bench gemm_big_bench_b15 gemm_big_bench_b16 gemm_big_bench gemm_big_bench_b16; do
  echo "== $b" >> $O/b1_ab.log
  timeout -k 10 300 tools/$b $CASES >> $O/b1_ab.log 2>&1
  rc=$?; [ $rc -le 1 ] || stop $b $rc
done
CASES="4096,4096,4096,0" timeout -k 10 400 bash tools/pmc_gemm_big.sh > $O/pmc.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop pmc $rc
cp -r gpurun_out/pmc_big $O/ 2>/dev/null
PLAN_COPY_TO=$O/tuned timeout -k 10 900 python -u scripts/write_gemm_plan.py llama3-8b > $O/plan_write.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop plan_write $rc
timeout -k 10 600 python -u scripts/bench_decode_graph.py --buckets 1,2,4,8,16,32,48,64,96,128,160,192,256,320,384,448,512 --persistent 1 > $O/decode_ladder.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop ladder $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop bench $rc
echo ALL DONE
