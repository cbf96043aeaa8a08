set -o pipefail
mkdir -p gpurun_out/big_ab
summ() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); x=d["detail"]; print(d["value"], d["p50_ms"], x["p99_ms"], x["decode_steps"], x["prefill_steps"], x.get("decode_ms_per_step"), x.get("prefill_ms_per_step"))'; }
for b in 16384 4096; do
  timeout -k 10 500 python bench.py --model mixtral-8x7b --concurrency 128 --steps 10 --warmup 3 --max-batched-tokens $b > gpurun_out/big_ab/mixtral_b$b.log 2>&1 || { echo FAIL; exit 1; }
  echo "mixtral b=$b: $(tail -1 gpurun_out/big_ab/mixtral_b$b.log | summ)"
done
for b in 16384; do
  timeout -k 10 500 python bench.py --model llama3-70b --concurrency 64 --steps 8 --warmup 2 --max-batched-tokens $b > gpurun_out/big_ab/l70_b$b.log 2>&1 || { echo FAIL; exit 1; }
  echo "70b b=$b: $(tail -1 gpurun_out/big_ab/l70_b$b.log | summ)"
done
