#!/bin/bash
# Kernel-level profile of one index build (scripts/build_bench.py) with rocprofv3 (kernel trace + stats only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$REPO/gpurun_out/bprof"
export HS_BENCH_DIR=/tmp/hs_bench
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/bprof" -o run -- \
  python3 "$REPO/scripts/build_bench.py" --sf ${SF:-100} --codec ${CODEC:-snappy} ${INDEX_ARGS:---index li_orderkey} \
  > "$REPO/gpurun_out/bprof/build.jsonl" 2> "$REPO/gpurun_out/bprof/build.log"
rc=$?
find "$REPO/gpurun_out/bprof" -name "*kernel_stats.csv" -exec cp {} "$REPO/gpurun_out/bprof/kernel_stats.csv" \;
exit $rc
