#!/bin/bash
# Round-4 profiling iteration: selected GPU tests (rc 1 does not stop the chain), a rocprofv3
# kernel-stats pass over the merge-join sweep ($CONFIGS), and the SF100 bench with the host
# cProfile of the timed steps (HS_BENCH_PROFILE, when HPROF=1).  Each GPU step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
TAG=${TAG:-p}
if [ -n "${TESTS}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS} -v -m gpu --timeout 240 \
    --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -z "$NOBENCH" ]; then
  HS_BENCH_PROFILE=${HPROF} timeout -k 10 600 python bench.py --sf ${SF:-100} --steps ${STEPS:-100} \
    --warmup 5 --host-breakdown 100 > gpurun_out/${TAG}_bench.json \
    2> gpurun_out/${TAG}_bench.log || exit $?
fi
if [ -n "$CONFIGS" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/prof_${TAG}" -o run \
    --output-format csv -- python3 "$REPO/scripts/qk_sweep.py" --sf ${SF:-100} --reps 20 \
    --only-merge --configs "$CONFIGS" > "$REPO/gpurun_out/${TAG}_sweep.jsonl" \
    2> "$REPO/gpurun_out/${TAG}_sweep.log" || exit $?
fi
