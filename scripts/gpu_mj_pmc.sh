#!/bin/bash
# Counter passes (one rocprofv3 run each, kernel trace only) over the merge-join Q3 workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
OUT="$REPO/gpurun_out/mjpmc${TAG}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export HS_BENCH_DIR=/tmp/hs_bench
if [ -z "$CONFIGS" ]; then CONFIGS='[{}]'; fi
timeout -k 10 600 python3 "$REPO/scripts/qk_sweep.py" --sf ${SF:-100} --reps 2 --only-merge --configs '[{}]' > "$OUT/warm.jsonl" 2> "$OUT/warm.log" || exit $?
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH FETCH_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex hs_jit_merge --kernel-trace --output-format csv \
    -d "$OUT/p$i" -o pmc -- python3 "$REPO/scripts/qk_sweep.py" --sf ${SF:-100} --reps 3 --only-merge --configs "$CONFIGS" \
    > "$OUT/run$i.jsonl" 2> "$OUT/run$i.log" || exit $?
  find "$OUT/p$i" -name "*counter_collection.csv" -exec cp {} "$OUT/counters$i.csv" \;
  rm -rf "$OUT/p$i"
done
python3 "$REPO/scripts/pmc_summary.py" "$OUT"/counters*.csv > "$OUT/summary.txt"
