#!/bin/bash
# Native Parquet GPU tests, then index-build timings (scripts/build_bench.py) under decode knobs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
timeout -k 10 300 python -u -m pytest tests/test_native_parquet.py -x -v -m gpu --timeout 120 \
  --timeout-method thread > gpurun_out/pq_tests.log 2>&1 || exit $?
OUT=gpurun_out/build_sweep${TAG}.jsonl
: > $OUT
for cfg in ${CFGS:-"HS_PQ_BATCH_DECODE=1" "HS_PQ_BATCH_DECODE=0"}; do
  echo "{\"cfg\": \"$cfg\"}" >> $OUT
  env $cfg timeout -k 10 400 python -u scripts/build_bench.py --sf ${SF:-100} --repeat ${REPEAT:-1} \
    >> $OUT 2>> gpurun_out/build_sweep${TAG}.log || exit $?
done
