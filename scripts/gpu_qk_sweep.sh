#!/bin/bash
# Query-kernel knob sweep (scripts/qk_sweep.py) on SF100 bench data; JSON lines in gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
timeout -k 10 ${TLIM:-700} python -u scripts/qk_sweep.py --sf ${SF:-100} ${SWEEP_ARGS} \
  > gpurun_out/qk_sweep${TAG}.jsonl 2> gpurun_out/qk_sweep${TAG}.log
