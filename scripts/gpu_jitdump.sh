#!/bin/bash
# Dump the generated query kernels (HS_JIT_DUMP) of the bench queries at SF${SF:-10}.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/jitdump
export HS_BENCH_DIR=/tmp/hs_bench HS_JIT_DUMP="$(pwd)/gpurun_out/jitdump"
timeout -k 10 600 python3 scripts/qk_sweep.py --sf ${SF:-10} --reps 3 --configs '[{}]' --merge-join --q3-full \
  > gpurun_out/jitdump/run.jsonl 2> gpurun_out/jitdump/run.log
