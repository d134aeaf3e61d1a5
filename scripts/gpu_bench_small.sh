#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
timeout -k 10 400 python bench.py --sf 1 --steps 5 --warmup 2 > gpurun_out/bench_sf1.json 2> gpurun_out/bench_sf1.log || exit $?
timeout -k 10 700 python bench.py --sf 10 --steps 10 --warmup 2 > gpurun_out/bench_sf10.json 2> gpurun_out/bench_sf10.log || exit $?
