#!/bin/bash
# HEAD profile: rocprofv3 kernel stats of a short bench, phase profiles at C = 256 and C = 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=gpurun_out/${TAG:-r5head}
mkdir -p $OUT
export TMPDIR=/tmp
rm -rf /tmp/ka_prof && (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/ka_prof -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --transport tcp > "$R/$OUT/prof.log" 2>&1) &&
mkdir -p $OUT/prof && find /tmp/ka_prof -name "*stats.csv" -exec cp {} $OUT/prof/ \; &&
timeout -k 10 400 python scripts/phase_profile.py --concurrency 256 > $OUT/phase_c256.log 2>&1 &&
timeout -k 10 400 python scripts/phase_profile.py --concurrency 1 > $OUT/phase_c1.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
