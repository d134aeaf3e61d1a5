#!/bin/bash
# Round-4 GPU iteration: GPU tests (a plain test failure, rc 1, does not stop the chain; a crash,
# abort, fault or time limit does), an SF100 bench with the host breakdown, and a rocprofv3
# kernel-stats pass over a short bench.  Every GPU step has its own time limit.
#   TESTS   pytest targets (default: all GPU tests; "-" skips)
#   TAG     output prefix under gpurun_out/
#   NOPROF  skip the rocprofv3 pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
TAG=${TAG:-r4s3}
if [ "${TESTS}" != "-" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 240 \
    --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py --sf ${SF:-100} --steps ${STEPS:-100} --warmup 5 \
  --host-breakdown 100 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json \
  2> gpurun_out/${TAG}_bench.log || exit $?
[ -n "$NOPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/prof_${TAG}" \
  -o run -- python "$REPO/bench.py" --sf ${SF:-100} --steps 40 --warmup 5 \
  --no-crosscheck > "$REPO/gpurun_out/${TAG}_prof.json" \
  2> "$REPO/gpurun_out/${TAG}_prof.log" || exit $?
