#!/bin/bash
# Run the SF100 bench once per value of an environment knob: VAR=HS_JIT_JI_ITEMS VALUES="2 4 8"
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
for v in $VALUES; do
  env $VAR=$v timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-crosscheck \
    > gpurun_out/sweep_${VAR}_$v.json 2> gpurun_out/sweep_${VAR}_$v.log || exit 1
done
