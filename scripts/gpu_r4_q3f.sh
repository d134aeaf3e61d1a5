#!/bin/bash
# TPC-H Q3 full shape (GROUP BY l_orderkey, o_orderdate, o_shippriority ORDER BY revenue DESC
# LIMIT 10) at SF100: the stage profile (HS_PROFILE=1) and a rocprofv3 kernel-stats pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
TAG=${TAG:-q3f}
CFG='[{}]'
[ -n "$CONFIGS" ] && CFG="$CONFIGS"
HS_PROFILE=1 timeout -k 10 600 python3 scripts/qk_sweep.py --sf 100 --reps 20 --only-q3-full \
  --configs "$CFG" > gpurun_out/${TAG}.jsonl 2> gpurun_out/${TAG}.log || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof_${TAG}" \
  -o run -- python3 "$REPO/scripts/qk_sweep.py" --sf 100 --reps 20 --only-q3-full --configs '[{}]' \
  > "$REPO/gpurun_out/${TAG}_prof.jsonl" 2> "$REPO/gpurun_out/${TAG}_prof.log" || exit $?
