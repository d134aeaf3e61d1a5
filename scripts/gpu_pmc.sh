#!/bin/bash
# Hardware counters for the query kernels (own run: --pmc with kernel trace only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$REPO/gpurun_out/pmc"
timeout -k 10 120 rocprofv3 -L > "$REPO/gpurun_out/pmc/avail.txt" 2>&1 || true
export HS_BENCH_DIR=/tmp/hs_bench
timeout -k 10 900 rocprofv3 --pmc ${PMC:-FETCH_SIZE OccupancyPercent MemUnitBusy VALUUtilization} --kernel-include-regex "${KREGEX:-hs_jit}" \
  --kernel-trace --output-format csv -d "$REPO/gpurun_out/pmc" -o pmc -- \
  python3 "$REPO/bench.py" --steps 3 --warmup 1 --no-crosscheck --sf ${SF:-100} \
  > "$REPO/gpurun_out/pmc/bench.json" 2> "$REPO/gpurun_out/pmc/bench.log"
rc=$?
find "$REPO/gpurun_out/pmc" -name "*counter_collection.csv" -exec cp {} "$REPO/gpurun_out/pmc/counters.csv" \;
exit $rc
