#!/bin/bash
# Round-3 iteration: targeted GPU tests, then a merge-join knob sweep (qk_sweep --only-merge).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_native_parquet.py tests/test_jit.py} -m gpu -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/iter_tests${TAG}.log 2>&1 || exit $?
if [ -n "$CONFIGS" ]; then
  timeout -k 10 600 python3 scripts/qk_sweep.py --sf ${SF:-100} --reps ${REPS:-12} ${SWEEP_MODE:---only-merge} \
    --configs "${CONFIGS}" > gpurun_out/iter_sweep${TAG}.jsonl 2> gpurun_out/iter_sweep${TAG}.log || exit $?
fi
if [ -n "$CONFIGS2" ]; then
  timeout -k 10 600 python3 scripts/qk_sweep.py --sf ${SF:-100} --reps ${REPS:-12} ${SWEEP_MODE2} \
    --configs "${CONFIGS2}" > gpurun_out/iter_sweep2${TAG}.jsonl 2> gpurun_out/iter_sweep2${TAG}.log || exit $?
fi
