#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
df -h /tmp > gpurun_out/bench_sf100.df
timeout -k 10 1000 python bench.py > gpurun_out/bench_sf100.json 2> gpurun_out/bench_sf100.log
rc=$?
df -h /tmp >> gpurun_out/bench_sf100.df
free -g >> gpurun_out/bench_sf100.df
exit $rc
