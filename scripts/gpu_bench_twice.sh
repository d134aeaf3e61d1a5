#!/bin/bash
# Two SF100 bench runs back to back on the same data (second run: warm page cache).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-crosscheck > gpurun_out/bench_twice_$i.json 2> gpurun_out/bench_twice_$i.log || exit 1
done
