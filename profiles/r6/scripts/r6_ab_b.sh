#!/bin/bash
# Round 6, call b: ring-kernel schedules with the split DMA issue (tools/gemm_bench_*), decode graph
# steps with the drained persistent / ring schedules against the counted build (tools/lib_counted/),
# then the full-depth parity tests with token agreement (tests/test_model_full_depth_gpu.py).
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
C="256,28672,4096,2,1,3 256,6144,4096,2,4,2 256,4096,14336,2,8,2 256,4096,4096,12,4,2 256,4096,4096,4,4,2
128,28672,4096,4,1,3 128,6144,4096,4,4,2 128,4096,14336,4,8,2 128,4096,4096,4,8,2
64,28672,4096,5,1,3 64,4096,14336,5,8,2 64,6144,4096,4,4,2 160,28672,4096,2,1,3 320,4096,4096,12,2,2"
for rep in 1 2; do
for s in s0 s1_0 s1_1 s2_1; do
  echo "== $s rep $rep" >> $O/time.log
  timeout -k 10 120 tools/gemm_bench_$s $C >> $O/time.log 2>&1 || exit 1
done
done
P="512,28672,4096,19,1,0 256,128256,4096,19,1,0 256,6144,4096,19,2,2 384,28672,4096,19,1,0"
for rep in 1 2; do for s in pp0 pp1; do
  echo "== $s rep $rep" >> $O/time_pp.log
  timeout -k 10 120 tools/gemm_bench_$s $P >> $O/time_pp.log 2>&1 || exit 1
done; done
GB_STRESS=300 GB_LDX0=1 timeout -k 10 120 tools/gemm_bench_pp1 $P >> $O/stress_pp.log 2>&1 || exit 1
echo "gemm A/B done"
timeout -k 10 300 python -u scripts/bench_decode_graph.py --buckets 1,2,256 --persistent 1 > $O/graph_safe.log 2>&1 || exit 1
KA_HIP_LIB_DIAG=1 KA_HIP_LIB=tools/lib_counted/libkagent_hip.so timeout -k 10 300 python -u scripts/bench_decode_graph.py --buckets 1,2,256 --persistent 1 > $O/graph_counted.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_decode_graph.py --buckets 1,2,256 --persistent 1 > $O/graph_safe2.log 2>&1 || exit 1
echo "graph A/B done"
timeout -k 10 900 python -u -m pytest tests/test_model_full_depth_gpu.py -x -v -s --timeout 600 --timeout-method thread > $O/full_depth.log 2>&1
echo "full depth rc=$?"
tail -5 $O/graph_safe.log $O/graph_counted.log $O/graph_safe2.log
grep -E "agreement|passed|failed" $O/full_depth.log
