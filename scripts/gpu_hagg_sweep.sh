#!/bin/bash
# q3_full (hash-mode GROUP BY + top-k) stage times at SF${SF:-100} for hash-table sizes
# (HS_HAGG_SLOTS_PER_GROUP) and lane-major match lists.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
for spg in ${SPGS:-1 2 4 8}; do
  HS_HAGG_SLOTS_PER_GROUP=$spg timeout -k 10 400 python3 scripts/qk_sweep.py --sf ${SF:-100} --reps 8 --only-q3-full \
    --configs '[{}, {"MJ_HASH_LANEMAJOR": true}]' > gpurun_out/hagg_spg$spg.jsonl 2> gpurun_out/hagg_spg$spg.log || exit $?
done
