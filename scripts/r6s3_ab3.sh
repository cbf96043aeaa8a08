#!/bin/bash
# Round 6 session 3: same-box Z (session-2 kernels) vs B (latency fixes): the driver-form headline,
# interleaved, plus one decode-graph pass each for the box's reference.
set -o pipefail
O=gpurun_out/r6s3_ab3
mkdir -p $O
for v in Z B; do
  KA_HIP_LIB_DIAG=1 KA_HIP_LIB=$GRAFT_REPO_ROOT/abtest/$v/libkagent_hip.so timeout -k 10 300 python -u scripts/bench_decode_graph.py --model llama3-8b --buckets 256 --reps 50 > $O/graph_${v}.log 2>&1
  rc=$?; echo "$v rc $rc: $(grep 'B=' $O/graph_${v}.log)"; [ $rc -eq 0 ] || exit $rc
done
for pass in 1 2; do
for v in Z B; do
  KA_HIP_LIB_DIAG=1 KA_HIP_LIB=$GRAFT_REPO_ROOT/abtest/$v/libkagent_hip.so timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_${v}_$pass.log 2>&1
  rc=$?; echo "$v bench $pass rc $rc: $(tail -1 $O/bench_${v}_$pass.log | cut -c1-120)"; [ $rc -eq 0 ] || exit $rc
done
done
