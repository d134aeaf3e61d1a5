#!/bin/bash
# Merge-join knob sweep (scripts/qk_sweep.py --merge-join) at SF${SF:-100}.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
timeout -k 10 900 python3 scripts/qk_sweep.py --sf ${SF:-100} --reps ${REPS:-12} --merge-join ${EXTRA} \
  --configs "${CONFIGS}" > gpurun_out/mj_sweep${TAG}.jsonl 2> gpurun_out/mj_sweep${TAG}.log
