#!/bin/bash
# GPU busy fraction over the timed region of the headline bench (rocprofv3 kernel trace, last 2 s of
# a 12-step run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/busy
export TMPDIR=/tmp
rm -rf /tmp/ka_busy
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/ka_busy -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 12 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/busy/bench.log" 2>&1
rc=$?
cd "$GRAFT_REPO_ROOT"
[ $rc -eq 0 ] || { echo "bench failed rc=$rc"; tail -5 gpurun_out/busy/bench.log; exit $rc; }
python scripts/trace_busy.py /tmp/ka_busy --window ${TRACE_WINDOW:-2.0} > gpurun_out/busy/trace_busy.txt 2>&1
head -30 gpurun_out/busy/trace_busy.txt
tail -1 gpurun_out/busy/bench.log | cut -c1-300
