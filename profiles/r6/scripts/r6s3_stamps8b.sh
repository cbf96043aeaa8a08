#!/bin/bash
# Round 6 session 3: phase stamps of the Llama-3-8B persistent decode kernel at B = 1 and 2.
set -o pipefail
O=gpurun_out/r6s3_smallb
mkdir -p $O
timeout -k 10 400 python -u scripts/bench_decode_graph.py --model llama3-8b --buckets 1,2 --persistent 1 --reps 30 > $O/stamps8b.log 2>&1
