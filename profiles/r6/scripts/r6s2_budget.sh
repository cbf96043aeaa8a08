#!/bin/bash
# Round 6 session 2: the engine's per-step token budget at the current kernels (driver form, TCP only).
set -o pipefail
O=gpurun_out/r6s2_budget
mkdir -p $O
for rep in 1 2; do
  for b in 4096 4352 4608 5120; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --transport tcp --no-prefix-off-pass --max-batched-tokens $b > $O/b${b}_r$rep.log 2>&1 || { echo "rc=$? b=$b"; exit 1; }
    python3 -c "
import json,sys;d=json.loads(open('$O/b${b}_r$rep.log').read().strip().splitlines()[-1]);t=d['detail']
print('budget $b rep $rep', d['value'], d['p50_ms'], t['decode_ms_per_step'], t['prefill_ms_per_step'], t['prefill_steps'], t['decode_steps'])"
  done
done
