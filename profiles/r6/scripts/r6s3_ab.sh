#!/bin/bash
# Round 6 session 3: same-box A/B/C of the decode graph step: A = attention change only (f17af4d),
# B = + rmsnorm slice loads + masked-argmax batching, C = + masked-argmax batching only.
set -o pipefail
O=gpurun_out/r6s3_ab
mkdir -p $O
for pass in 1 2; do
for v in A B C; do
  KA_HIP_LIB_DIAG=1 KA_HIP_LIB=abtest/$v/libkagent_hip.so timeout -k 10 300 python -u scripts/bench_decode_graph.py --model llama3-8b --buckets 8,256 --reps 50 > $O/graph_${v}_$pass.log 2>&1
  rc=$?; echo "$v pass $pass rc $rc: $(grep 'B=' $O/graph_${v}_$pass.log)"; [ $rc -eq 0 ] || exit $rc
done
done
