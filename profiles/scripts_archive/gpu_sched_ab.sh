#!/bin/bash
# Scheduler policy A/B: the wave hold (KA_PREFILL_HOLD_STEPS) and idle-burst
# gather (KA_GATHER_MAX_MS) heuristics on vs off, under closed-loop EOS-terminated variable-length
# outputs and under open-loop Poisson arrivals.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sched
run() {  # name, env..., -- args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 400 python bench.py "$@" > gpurun_out/sched/$name.log 2>&1 || { echo "FAILED: $name"; tail -5 gpurun_out/sched/$name.log; exit 1; }
  python - "$name" gpurun_out/sched/$name.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s} {d['value']:8.1f} req/s  p50 {d['p50_ms']:7.1f}  p99 {d['detail']['p99_ms']:7.1f}  "
      f"prefill steps {d['detail'].get('prefill_steps')}  decode {d['detail'].get('decode_ms_per_step')} ms")
PY
}
for pol in ${POLICIES:-default hold nogather neither}; do
  case $pol in
    default) E=(KA_X=1);;
    hold) E=(KA_PREFILL_HOLD_STEPS=8);;
    nogather) E=(KA_GATHER_MAX_MS=0);;
    neither) E=(KA_PREFILL_HOLD_STEPS=0 KA_GATHER_MAX_MS=0);;
  esac
  run varlen_$pol "${E[@]}" -- --steps 20 --warmup 5 --variable-len
  run open900_$pol "${E[@]}" -- --steps 10 --warmup 3 --load open --rate 900 --variable-len
  [ -n "$FIXED" ] && run fixed16_$pol "${E[@]}" -- --steps 20 --warmup 5
done
