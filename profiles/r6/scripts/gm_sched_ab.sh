#!/bin/bash
# A/B of the ring-kernel LDS-DMA wait schedules (KA_GM_SCHED 0 counted / 1 set / 2 pair) on the
# decode plan's shapes, then the alternating-launch stress (GB_STRESS) with and without the
# duplicate-address amplifier (GB_LDX0).  Binaries: tools/gemm_bench_s{0,1,2} (built on the CPU side; profiles/r6/gm_sched/).
set -o pipefail
O=gpurun_out/r6_gm
mkdir -p $O
C="256,28672,4096,2,1,3 256,6144,4096,2,4,2 256,4096,14336,2,8,2 256,4096,4096,12,4,2 256,4096,4096,4,4,2
128,28672,4096,4,1,3 128,6144,4096,4,4,2 128,4096,14336,4,8,2 128,4096,4096,4,8,2
64,28672,4096,5,1,3 64,4096,14336,5,8,2 64,6144,4096,4,4,2 160,28672,4096,2,1,3 320,4096,4096,12,2,2
512,28672,4096,19,1,0 256,128256,4096,19,1,0 256,6144,4096,19,2,2"
for rep in 1 2; do
for s in 0 1 2; do
  echo "== sched $s rep $rep" | tee -a $O/time.log
  timeout -k 10 120 tools/gemm_bench_s$s $C >> $O/time.log 2>&1 || exit 1
done
done
S="256,28672,4096,2,1,3 256,6144,4096,2,4,2 256,4096,14336,2,8,2 256,4096,4096,12,4,2 128,6144,4096,4,4,2 64,4096,14336,5,8,2 100,6144,4096,4,4,2 200,4096,4096,12,4,2 256,128256,4096,19,1,0 512,28672,4096,19,1,0"
for s in 0 1 2; do
  for a in 1 0; do
    echo "== stress sched $s ldx0 $a" | tee -a $O/stress.log
    GB_STRESS=300 GB_LDX0=$a timeout -k 10 200 tools/gemm_bench_s$s $S >> $O/stress.log 2>&1 || exit 1
  done
done
grep -E "stress|==" $O/stress.log | tail -80
