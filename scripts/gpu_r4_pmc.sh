#!/bin/bash
# Counter passes (rocprofv3 --pmc, kernel trace only, one run per counter group) over the SF10 (SF env)
# merge-join sweep's two-phase kernels (hs_jit_run_*): FETCH_SIZE for the effective bandwidth,
# LDS instructions / bank conflicts, VALU / VMEM instruction counts, wave-cycle occupancy.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
OUT="$REPO/gpurun_out/pmc_${TAG:-r4}"
mkdir -p "$OUT"
export HS_BENCH_DIR=/tmp/hs_bench
# data + indexes (and a warm-up of the sweep) outside the counter runs
timeout -k 10 600 python3 scripts/qk_sweep.py --sf ${SF:-10} --reps 3 --only-merge --configs '[{}]' \
  > "$OUT/warm.jsonl" 2> "$OUT/warm.log" || exit $?
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-include-regex hs_jit_run --kernel-trace \
    --output-format csv -d "$OUT/p$i" -o pmc -- python3 "$REPO/scripts/qk_sweep.py" --sf ${SF:-10} \
    --reps 3 --only-merge --configs '[{}]' > "$OUT/run$i.jsonl" 2> "$OUT/run$i.log" || exit $?
  find "$OUT/p$i" -name "*counter_collection.csv" -exec cp {} "$OUT/counters$i.csv" \;
  find "$OUT/p$i" -name "*kernel_trace.csv" -exec cp {} "$OUT/trace$i.csv" \;
  rm -rf "$OUT/p$i"
done
python3 "$REPO/scripts/pmc_summary.py" "$OUT"/counters*.csv > "$OUT/summary.txt"
