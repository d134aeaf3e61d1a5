#!/bin/bash
# Merge-join microbenchmark (scripts/mj_micro.py) timing sweep, then one counter pass pair per
# configuration in $PMC_CONFIGS (kernel trace only, one rocprofv3 run per counter group, each
# under its own time limit); stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
OUT="$REPO/gpurun_out/mjm${TAG}"
mkdir -p "$OUT"
if [ -z "$CONFIGS" ]; then CONFIGS='[{}]'; fi
timeout -k 10 300 python3 scripts/mj_micro.py --sf ${SF:-100} --configs "$CONFIGS" \
  > "$OUT/sweep.jsonl" 2> "$OUT/sweep.log" || exit $?
[ -z "$PMC_CONFIGS" ] && exit 0
cd /tmp && export TMPDIR=/tmp
echo "$PMC_CONFIGS" | python3 -c "import json,sys; [print(json.dumps(c)) for c in json.load(sys.stdin)]" > "$OUT/pmc_configs.txt"
j=0
while read -r CFG; do
  j=$((j+1))
  i=0
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH FETCH_SIZE" ; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $P --kernel-include-regex "hs_jit_(merge|run)" --kernel-trace --output-format csv \
      -d "$OUT/c${j}p$i" -o pmc -- python3 "$REPO/scripts/mj_micro.py" --sf ${SF:-100} --iters 3 \
      --configs "[$CFG]" > "$OUT/c${j}run$i.jsonl" 2> "$OUT/c${j}run$i.log" || exit $?
    find "$OUT/c${j}p$i" -name "*counter_collection.csv" -exec cp {} "$OUT/c${j}counters$i.csv" \;
    rm -rf "$OUT/c${j}p$i"
  done
  echo "config $CFG" > "$OUT/c${j}summary.txt"
  python3 "$REPO/scripts/pmc_summary.py" "$OUT"/c${j}counters*.csv >> "$OUT/c${j}summary.txt"
done < "$OUT/pmc_configs.txt"
