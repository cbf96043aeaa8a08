#!/bin/bash
# Round 6 session 3: where a B = 4 / 8 decode graph step goes (kernel trace + stats per bucket).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6s3_smallb
mkdir -p $O
for b in 4 8; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_b$b -o run -- python3 -u scripts/bench_decode_graph.py --model llama3-8b --buckets $b --persistent 0 --reps 50 > $O/b$b.log 2>&1
  rc=$?; echo "b$b rc $rc"; [ $rc -eq 0 ] || exit $rc
done
