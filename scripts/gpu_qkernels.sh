#!/bin/bash
# Query-kernel investigation: dump the generated kernel sources of the SF100 bench, list the
# available counters, then one rocprofv3 --pmc pass per counter group (kernel trace only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
OUT="$REPO/gpurun_out/qk"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export HS_BENCH_DIR=/tmp/hs_bench
export HS_JIT_DUMP="$OUT/src"
SF=${SF:-100}
timeout -k 10 600 python3 "$REPO/bench.py" --steps 10 --warmup 2 --no-crosscheck --sf $SF \
  > "$OUT/bench.json" 2> "$OUT/bench.log" || exit $?
unset HS_JIT_DUMP
timeout -k 10 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
i=0
for grp in ${PMC_GROUPS:-"FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES TCC_HIT_sum TCC_MISS_sum"}; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-hs_jit}" \
    --kernel-trace --output-format csv -d "$OUT/pmc$i" -o pmc -- \
    python3 "$REPO/bench.py" --steps 3 --warmup 1 --no-crosscheck --sf $SF \
    > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.log" || exit $?
  find "$OUT/pmc$i" -name "*counter_collection.csv" -exec cp {} "$OUT/counters$i.csv" \;
  find "$OUT/pmc$i" -name "*kernel_trace.csv" -exec cp {} "$OUT/trace$i.csv" \;
  rm -rf "$OUT/pmc$i"
done
exit 0
