#!/bin/bash
# Round 6, call h: HEAD measurements — the driver-form bench twice, low-concurrency latency, and the
# rocprofv3 kernel stats + phase profiles (scripts/profile_head.sh).
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver_$rep.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench_driver_$rep.log; exit 1; }
  tail -1 $O/bench_driver_$rep.log | cut -c1-400
done
for c in 1 2 4 8; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --concurrency $c --transport tcp --no-prefix-off-pass > $O/bench_c$c.log 2>&1 || { echo "bench c$c rc=$?"; exit 1; }
  tail -1 $O/bench_c$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C=$c', d['value'], d.get('p50_ms'), d['detail'].get('decode_ms_per_step'), d['detail'].get('prefill_ms_per_step'))"
done
TAG=r6h/head bash scripts/profile_head.sh > $O/profile_head.log 2>&1; echo "profile rc=$?"; tail -3 $O/profile_head.log
