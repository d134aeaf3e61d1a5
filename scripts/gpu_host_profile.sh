#!/bin/bash
# Host-side cProfile of the SF100 bench's timed steps (HS_BENCH_PROFILE=1) + stage profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench HS_BENCH_PROFILE=1 HS_PROFILE=${HS_PROFILE:-0}
timeout -k 10 600 python bench.py --steps ${STEPS:-40} --warmup 3 --no-crosscheck \
  > gpurun_out/host_profile.json 2> gpurun_out/host_profile.log
