#!/bin/bash
# Round-4 iteration: selected GPU tests, then a host cProfile of the bench's timed steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_project_gpu.py tests/test_gpu_e2e.py} -x -v -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/r4_tests.log 2>&1 || exit $?
if [ -n "$PROFILE_SF" ]; then
  HS_BENCH_PROFILE=1 timeout -k 10 500 python bench.py --sf $PROFILE_SF --steps ${STEPS:-100} --warmup 5 \
    --no-crosscheck > gpurun_out/r4_prof.json 2> gpurun_out/r4_prof.log || exit $?
fi
