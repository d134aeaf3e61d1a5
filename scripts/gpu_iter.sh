#!/bin/bash
# One iteration: GPU tests (one pytest process), SF100 bench, 2-rank gloo rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread \
  ${TESTS_K:+-k "$TESTS_K"} > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest rc=$?" >> gpurun_out/gpu_tests.log; exit 1; }
[ -n "$SKIP_BENCH" ] || bash scripts/gpu_bench_sf100.sh || exit 1
[ -n "$SKIP_DIST" ] || bash scripts/gpu_dist_rehearsal.sh || exit 1
