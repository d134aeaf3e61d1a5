#!/bin/bash
# One GPU iteration: kernel + e2e tests, smoke, SF100 bench, rocprofv3 kernel profile.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
mkdir -p gpurun_out
bash scripts/gpu_e2e.sh || exit $?
bash scripts/gpu_bench_sf100.sh || exit $?
bash scripts/gpu_profile.sh || exit $?
