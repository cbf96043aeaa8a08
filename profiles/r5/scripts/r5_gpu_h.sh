#!/bin/bash
# Round 5, GPU call h: kernel census of one Llama-3-70B TP = 8 rank (virtual rank, collectives left out)
# under rocprofv3, and the persisted plans of Llama-3-70B at TP = 1 (BASELINE config #3 shapes).
set -o pipefail
O=gpurun_out/r5h2
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_vrank70 -o vrank70 -- python3 -u scripts/bench_virtual_rank.py --model llama3-70b --tp 8 --buckets 1,8,64,256 --reps 5 > $O/vrank70_prof.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop prof_vrank70 $rc
export KA_GEMM_PLAN=write PLAN_COPY_TO=$O/tuned KA_AUTOTUNE_ROUNDS=3
PLAN_BUCKETS=1,2,4,8,16,32,64,128,256 timeout -k 10 1000 python -u scripts/write_gemm_plan.py llama3-70b > $O/plan_70b.log 2>&1
rc=$?; [ $rc -eq 0 ] || stop plan_70b $rc
echo ALL DONE
