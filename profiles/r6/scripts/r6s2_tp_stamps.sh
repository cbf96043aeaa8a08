#!/bin/bash
# Phase stamps of the persistent decode kernel on the Llama-3-70B TP = 8 rank (virtual communicator).
set -o pipefail
O=gpurun_out/r6s2_tp
mkdir -p $O
timeout -k 10 600 python -u scripts/bench_decode_graph.py --model llama3-70b --tp 8 --buckets 1,2 --persistent 1 --reps 30 > $O/stamps70.log 2>&1
