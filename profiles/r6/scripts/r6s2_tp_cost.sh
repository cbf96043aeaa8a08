#!/bin/bash
# Round 6 session 2: 8B persistent B=1/2 graph step after the kernel changes (regression check), then
# the TP = 2 two-ranks-one-GPU decode step: persistent + in-kernel all-reduce vs chain + one-shot kernels.
set -o pipefail
O=gpurun_out/r6s2_tp
mkdir -p $O
timeout -k 10 400 python -u scripts/bench_decode_graph.py --model llama3-8b --buckets 1,2 --persistent 1 --reps 50 > $O/decode8b_persistent.log 2>&1
rc=$?; echo "8b rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u scripts/bench_tp_persistent_2rank.py --model llama3-70b-8l --reps 50 > $O/tp2_two_ranks.log 2>&1
rc=$?; echo "tp2 rc $rc"; exit $rc
