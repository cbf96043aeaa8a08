set -o pipefail
O=gpurun_out/tailm; mkdir -p $O
for m in 0 1 3 2 0 1 3 2; do
  echo "== mode $m" >> $O/tail_modes.log
  GB_FULL=1 GB_FULL_REPS=6 GB_ROUNDS=1 timeout -k 10 300 tools/gemm_big_bench_m$m 2944,6144,4096,0 4096,1152,4096,0 2944,28672,4096,3 >> $O/tail_modes.log 2>&1
  rc=$?; [ $rc -le 1 ] || { echo "STOP mode $m rc $rc"; exit $rc; }
done
echo ALL DONE
