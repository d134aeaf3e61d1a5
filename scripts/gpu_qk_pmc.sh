#!/bin/bash
# PMC counters of the generated query kernels on the qk_sweep workload: one rocprofv3 --pmc pass
# per counter group (kernel trace only), every pass under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
OUT="$REPO/gpurun_out/qpmc${TAG}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export HS_BENCH_DIR=/tmp/hs_bench
DEFCFG='[{}]'
CFGS="${CONFIGS:-$DEFCFG}"
# data + indexes once, outside the profiler
timeout -k 10 600 python3 "$REPO/scripts/qk_sweep.py" --sf ${SF:-100} --reps 2 --configs '[{}]' > "$OUT/warm.jsonl" 2> "$OUT/warm.log" || exit $?
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL ${PMC_KILL:-120} rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-hs_jit}" \
    --kernel-trace --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 "$REPO/scripts/qk_sweep.py" --sf ${SF:-100} --reps 4 --configs "$CFGS" ${SWEEP_EXTRA} \
    > "$OUT/p$i.jsonl" 2> "$OUT/p$i.log" || exit $?
  find "$OUT/p$i" -name "*counter_collection.csv" -exec cp {} "$OUT/counters$i.csv" \;
  rm -rf "$OUT/p$i"
done <<< "${GROUPS_LIST:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS
SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE
FETCH_SIZE GRBM_GUI_ACTIVE}"
exit 0
