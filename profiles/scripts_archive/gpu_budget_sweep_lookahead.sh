set -o pipefail
mkdir -p gpurun_out/budget2
summ() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); x=d["detail"]; print(d["value"], d["p50_ms"], x["p99_ms"], x["decode_steps"], x["prefill_steps"], x.get("decode_ms_per_step"), x.get("prefill_ms_per_step"))'; }
for r in 1 2; do for b in 3072 4096 5120 6144 8192; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --max-batched-tokens $b > gpurun_out/budget2/b${b}_r$r.log 2>&1 || { echo FAIL; exit 1; }
  echo "b=$b r=$r: $(tail -1 gpurun_out/budget2/b${b}_r$r.log | summ)"
done; done
