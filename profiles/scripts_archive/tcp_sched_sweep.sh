#!/bin/bash
# TCP-transport scheduler sweep (one GPU call): closed loop C=256, 20 steps; one JSON line per config.
set -o pipefail
OUT=${OUT:-gpurun_out/tcp_sweep}; mkdir -p $OUT
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --transport tcp --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/$name.log 2>&1 || return 1
  echo "$name $(tail -1 $OUT/$name.log | python3 -c 'import json,sys; d=json.load(sys.stdin); x=d["detail"]; print(d["value"], d["p50_ms"], x["p99_ms"], x["decode_steps"], x["prefill_steps"], x["decode_ms_per_step"], x["prefill_ms_per_step"], x["queue_wait_ms_mean"], x.get("client_mean_ms"), x.get("server_ms"), x.get("cpu_cores"))')"
}
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  run $name $envs || exit 1
done
