#!/bin/bash
# Direct-weight decode kernels (cfg 30-35) against rocBLAS and the best LDS-DMA ring configuration
# per shape, Llama-3-8B decode shapes at M = 256 / 128.
B=${GEMM_BENCH:-tools/gemm_bench}
P=""
for M in 256 128; do
  if [ $M = 256 ]; then D="30 31 34 35"; else D="32 33 31"; fi
  P="$P $M,28672,4096,-1,1,0 $M,28672,4096,2,1,0"
  for c in $D; do P="$P $M,28672,4096,$c,1,0"; done
  P="$P $M,128256,4096,-1,1,0"
  for c in $D; do P="$P $M,128256,4096,$c,1,0"; done
  P="$P $M,4096,14336,4,8,2"
  for c in $D; do P="$P $M,4096,14336,$c,7,2"; done
done
$B $P
