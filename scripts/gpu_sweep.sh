#!/bin/bash
# Run the SF100 bench once per configuration line of $SWEEP (";"-separated, each a list of
# NAME=VALUE environment settings, e.g. "HS_JIT_SCAN_VEC=4;HS_JIT_SCAN_VEC=0").
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
i=0
IFS=';' read -ra CFGS <<< "$SWEEP"
for cfg in "${CFGS[@]}"; do
  i=$((i+1))
  echo "$cfg" > gpurun_out/sweep_$i.cfg
  env $cfg timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-crosscheck \
    > gpurun_out/sweep_$i.json 2> gpurun_out/sweep_$i.log || exit 1
done
