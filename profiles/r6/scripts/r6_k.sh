#!/bin/bash
# Round 6, call k: kernel-boundary idle time in the B = 256 and B = 8 decode graphs (rocprofv3 kernel trace of
# graph replays; scripts/trace_gaps.py).
set -o pipefail
R=$(pwd)
O=gpurun_out/r6k
mkdir -p $O
export TMPDIR=/tmp
for B in 256 8; do
  rm -rf /tmp/kt_$B && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_$B -o run -- python3 "$R/scripts/bench_decode_graph.py" --buckets $B --persistent 0 --reps 10 > "$R/$O/trace_b$B.log" 2>&1) || { echo "trace B=$B rc=$?"; exit 1; }
  f=$(find /tmp/kt_$B -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_gaps.py "$f" --last $((B == 256 ? 2400 : 2400)) > $O/gaps_b$B.txt 2>&1; echo "B=$B"; head -14 $O/gaps_b$B.txt
done
