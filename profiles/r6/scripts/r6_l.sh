#!/bin/bash
# Round 6, call l: wave-gather A/B at the headline config (TCP only, 3 reps per setting, interleaved).
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
for rep in 1 2 3; do
  for cfg in "1.5 15" "3 15" "3 30"; do
    set -- $cfg
    KA_GATHER_QUIET_MS=$1 KA_GATHER_MAX_MS=$2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --transport tcp --no-prefix-off-pass > $O/q$1_m$2_r$rep.log 2>&1 || { echo "rc=$?"; tail -3 $O/q$1_m$2_r$rep.log; exit 1; }
    tail -1 $O/q$1_m$2_r$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); dd=d['detail']; print('quiet $1 max $2 rep $rep', d['value'], d['p50_ms'], dd['prefill_steps'], dd['decode_steps'], dd['decode_ms_per_step'], dd['prefill_ms_per_step'])"
  done
done
