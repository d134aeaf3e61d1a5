#!/bin/bash
# Round-4 merge-join iteration: selected GPU tests (a plain failure, rc 1, does not stop the
# chain), a merge-join timing sweep over $CONFIGS at SF100 and the SF100 bench.  Each GPU step
# has its own time limit; a crash / abort / time limit ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
TAG=${TAG:-mj}
if [ "${TESTS}" != "-" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS} -v -m gpu --timeout 240 \
    --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$CONFIGS" ]; then
  timeout -k 10 600 python3 scripts/qk_sweep.py --sf ${SF:-100} --reps ${REPS:-20} --only-merge \
    --configs "$CONFIGS" > gpurun_out/${TAG}_sweep.jsonl 2> gpurun_out/${TAG}_sweep.log || exit $?
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python bench.py --sf ${SF:-100} --steps ${STEPS:-100} --warmup 5 \
    --host-breakdown 100 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit $?
fi
