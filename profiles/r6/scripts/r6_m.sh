#!/bin/bash
# Round 6, call m: the BASELINE configs other than the headline, at HEAD: #5 the mixed stream (hits + misses
# + /execute + /metrics scrapes), #4 Mixtral-8x7B (TP = 1, full model), #3's model Llama-3-70B (TP = 1).
set -o pipefail
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --mix --transport asgi > $O/bench_mix.log 2>&1; echo "mix rc=$?"; tail -1 $O/bench_mix.log | cut -c1-600
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --model mixtral-8x7b --concurrency 128 --transport tcp --no-prefix-off-pass > $O/bench_mixtral.log 2>&1; echo "mixtral rc=$?"; tail -1 $O/bench_mixtral.log | cut -c1-400
