#!/bin/bash
# BASELINE.json side configurations on 1 MI355X, one JSON line each (benchmarks/configs.py).
# Each config runs under its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
SF=${SF:-100}
for c in ${CONFIGS:-csv10k sf10_filter q3_3way hybrid}; do
  # each config builds its own indexes: drop earlier index / copy dirs so /tmp does not fill up
  rm -rf "$HS_BENCH_DIR"/indexes_* "$HS_BENCH_DIR"/cfg_* 2>/dev/null
  timeout -k 10 ${CFG_TIMEOUT:-420} python benchmarks/configs.py --config $c --sf $SF \
    >> gpurun_out/configs.jsonl 2> gpurun_out/config_$c.log || { echo "config $c rc=$?" >> gpurun_out/config_$c.log; exit 1; }
done
