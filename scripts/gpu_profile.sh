#!/bin/bash
# Kernel-level profile of the SF100 bench (build + queries) with rocprofv3 (kernel trace + stats only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
cd /tmp && export TMPDIR=/tmp
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$REPO/gpurun_out/prof"
export HS_BENCH_DIR=/tmp/hs_bench HS_PROFILE=1
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof" -o run -- \
  python3 "$REPO/bench.py" --steps 10 --warmup 2 --no-crosscheck > "$REPO/gpurun_out/prof/bench.json" 2> "$REPO/gpurun_out/prof/bench.log"
rc=$?
find "$REPO/gpurun_out/prof" -name "*kernel_stats.csv" -exec cp {} "$REPO/gpurun_out/prof/kernel_stats.csv" \; 
exit $rc
