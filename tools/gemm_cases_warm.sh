#!/bin/bash
# Decode shapes with W streamed from HBM (default: weights rotate past the Infinity Cache) and with
# W resident in the Infinity Cache (GB_WARM=1): how much of the decode GEMM time is HBM streaming.
B=${GEMM_BENCH:-tools/gemm_bench}
P="256,28672,4096,-1,1,0 256,28672,4096,2,1,3 256,28672,4096,3,1,0 256,6144,4096,-1,1,0 256,6144,4096,4,2,2 256,4096,4096,-1,1,0 256,4096,4096,4,4,2 256,4096,14336,4,4,2 256,4096,14336,-1,1,0 256,128256,4096,-1,1,0 128,28672,4096,-1,1,0 128,28672,4096,24,1,3 128,4096,14336,4,8,2 128,4096,4096,4,8,2 128,6144,4096,4,4,2"
echo "## cold"; $B $P
echo "## warm"; GB_WARM=1 $B $P
