#!/bin/bash
# Round-4 side evidence on one MI355X.  PART=baseline: the SF100 bench (data + indexes), then
# the CPU baseline over the same files (warm resident tables, cold indexed, unindexed; 16
# threads).  PART=configs: BASELINE.json side configurations (benchmarks/configs.py) in
# $CONFIGS.  Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
TAG=${TAG:-side}
if [ "$PART" = "baseline" ]; then
  timeout -k 10 600 python bench.py --sf 100 --steps 100 --warmup 5 \
    > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit $?
  timeout -k 10 840 python scripts/cpu_baseline.py --sf 100 --threads 16 --reps ${REPS:-3} \
    --out gpurun_out/${TAG}_cpu_baseline_sf100.json > gpurun_out/${TAG}_cpu.log 2>&1 || exit $?
fi
if [ "$PART" = "configs" ]; then
  for c in ${CONFIGS:-sf10_filter q3_3way hybrid}; do
    rm -rf "$HS_BENCH_DIR"/indexes_* "$HS_BENCH_DIR"/cfg_* 2>/dev/null
    timeout -k 10 ${CFG_TIMEOUT:-420} python benchmarks/configs.py --config $c --sf ${SF:-100} \
      ${CFG_ARGS} >> gpurun_out/${TAG}_configs.jsonl 2> gpurun_out/${TAG}_config_$c.log \
      || { echo "config $c rc=$?" >> gpurun_out/${TAG}_config_$c.log; exit 1; }
  done
fi
