#!/bin/bash
# Merge-join cost decomposition (qk_sweep MJ_EXP variants), resident column encodings, and one
# counter pass with FETCH_SIZE over the merge join and the Q6 scan (kernel trace only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
OUT="$REPO/gpurun_out/mjm${TAG}"
mkdir -p "$OUT"
export HS_BENCH_DIR=/tmp/hs_bench
DECOMP=${DECOMP:-'[{}, {"MJ_EXP": "notail"}, {"MJ_EXP": "nowalk"}, {"MJ_EXP": "nostage"}, {"MJ_EXP": "nowalk,notail"}]'}
timeout -k 10 600 python3 scripts/qk_sweep.py --sf ${SF:-100} --reps ${REPS:-12} --only-merge --show-compact \
  --configs "$DECOMP" > "$OUT/decomp.jsonl" 2> "$OUT/decomp.log" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-include-regex "hs_jit_(merge|scan)" --kernel-trace --stats --output-format csv \
  -d "$OUT/p1" -o pmc -- python3 "$REPO/scripts/qk_sweep.py" --sf ${SF:-100} --reps 3 --merge-join --configs '[{}]' \
  > "$OUT/pmc_run.jsonl" 2> "$OUT/pmc_run.log" || exit $?
find "$OUT/p1" -name "*counter_collection.csv" -exec cp {} "$OUT/counters1.csv" \;
find "$OUT/p1" -name "*kernel_stats.csv" -exec cp {} "$OUT/kstats1.csv" \;
rm -rf "$OUT/p1"
python3 "$REPO/scripts/pmc_summary.py" "$OUT"/counters1.csv > "$OUT/summary.txt"
