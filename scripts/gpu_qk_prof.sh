#!/bin/bash
# Kernel trace + stats of the qk_sweep workload (scripts/qk_sweep.py), no counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
OUT="$REPO/gpurun_out/qprof${TAG}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export HS_BENCH_DIR=/tmp/hs_bench
DEFCFG="[{}]"
timeout -k 10 600 python3 "$REPO/scripts/qk_sweep.py" --sf ${SF:-100} --reps 2 --configs '[{}]' > "$OUT/warm.jsonl" 2> "$OUT/warm.log" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p" -o run -- \
  python3 "$REPO/scripts/qk_sweep.py" --sf ${SF:-100} --reps ${REPS:-8} --configs "${CONFIGS:-$DEFCFG}" ${SWEEP_EXTRA} \
  > "$OUT/run.jsonl" 2> "$OUT/run.log" || exit $?
find "$OUT/p" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/p" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace.csv" \;
rm -rf "$OUT/p"
