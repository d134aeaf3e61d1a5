#!/bin/bash
# Round-4 iteration on the GPU box: selected GPU tests, an SF100 bench (recording the kernel
# sources the bench generates), and a rocprofv3 kernel-stats pass.  Every GPU step has its own
# time limit and the steps stop at the first failure.
#   TESTS="..."   pytest targets (default: merge-join + e2e)
#   BENCH_SF=100  bench scale factor (empty: skip)
#   PROF=1        rocprofv3 --kernel-trace --stats over a short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
TAG=${TAG:-r4}
if [ -n "${TESTS-x}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_jit.py tests/test_gpu_e2e.py} -x -v -m gpu \
    --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
fi
if [ -n "$BENCH_SF" ]; then
  HS_JIT_RECORD=gpurun_out/aot_${TAG} timeout -k 10 600 python bench.py --sf $BENCH_SF \
    --steps ${STEPS:-100} --warmup 5 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json \
    2> gpurun_out/${TAG}_bench.log || exit $?
fi
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" \
    -o run -- python "$GRAFT_REPO_ROOT/bench.py" --sf ${PROF_SF:-100} --steps 40 --warmup 5 \
    --no-crosscheck > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.json" \
    2> "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" || exit $?
fi
