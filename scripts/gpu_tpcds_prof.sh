#!/bin/bash
# Kernel trace + stats of the TPC-DS star-join config (benchmarks/configs.py tpcds_3way).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$REPO/gpurun_out/tprof"
export HS_BENCH_DIR=/tmp/hs_bench
timeout -k 10 800 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/tprof" -o run -- \
  python3 "$REPO/benchmarks/configs.py" --config tpcds_3way --steps 10 \
  > "$REPO/gpurun_out/tprof/tpcds.jsonl" 2> "$REPO/gpurun_out/tprof/tpcds.log"
rc=$?
find "$REPO/gpurun_out/tprof" -name "*kernel_stats.csv" -exec cp {} "$REPO/gpurun_out/tprof/kernel_stats.csv" \;
exit $rc
