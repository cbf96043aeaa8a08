#!/bin/bash
# Round 6 session 3: the 70B TP = 8 rank (virtual communicator) at B = 8: graph step and kernel census.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6s3_tp8b
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 -u scripts/bench_decode_graph.py --model llama3-70b --tp 8 --buckets 8 --reps 40 > $O/b8.log 2>&1
rc=$?; echo "rc $rc"; grep "B=" $O/b8.log; exit $rc
