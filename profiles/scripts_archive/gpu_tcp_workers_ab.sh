set -o pipefail
mkdir -p gpurun_out/tcp_ab
summ() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); x=d["detail"]; print(d["value"], d["p50_ms"], x["p99_ms"], x.get("decode_ms_per_step"), x.get("prefill_ms_per_step"), x.get("queue_wait_ms_mean"))'; }
for spec in 2:2 4:4 4:6 6:6; do
  IFS=: read w c <<< "$spec"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --transport tcp --api-workers $w --client-procs $c > gpurun_out/tcp_ab/w${w}_c$c.log 2>&1 || { echo FAIL; tail -3 gpurun_out/tcp_ab/w${w}_c$c.log; exit 1; }
  echo "tcp w=$w c=$c: $(tail -1 gpurun_out/tcp_ab/w${w}_c$c.log | summ)"
done
