#!/bin/bash
# Round 5, GPU call y: the drained gemm_big (default now) in the alternating-shape diag on four shapes,
# and the gemm_mfma ring kernels under the same launch pattern.
set -o pipefail
O=gpurun_out/r5y
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
DIAG_REPS=100 timeout -k 10 400 python -u profiles/r5/gemm_big_clamp/gb_wrong_rows_diag.py > $O/gb_diag.log 2>&1 || stop gb_diag $?
DIAG_REPS=60 timeout -k 10 500 python -u profiles/r5/gemm_big_clamp/gm_stress_diag.py > $O/gm_diag.log 2>&1 || stop gm_diag $?
echo ALL DONE
