#!/bin/bash
# One parameterized runner for every GPU-box job (gpurun):
#
#   gpurun -- 'TAG=x bash scripts/gpu.sh tests smoke bench prof'
#
# Steps run in the order given; each GPU step has its own time limit and the chain stops at the
# first crash / abort / time limit (a plain pytest failure, rc 1, lets later steps run so the
# record is complete).  Outputs land in gpurun_out/<TAG>_<step>.* (copy what is judged into
# profiles/).  Knobs (env):
#   TAG           output prefix (default run)
#   TESTS         test files / dirs for `tests` (default tests)
#   PYTEST_ARGS   extra pytest args for `tests` (no spaces inside one argument)
#   BENCH_ARGS    args for `bench` / `prof` / `hostprof` (default SF100, 100 / 40 steps)
#   SF            scale factor for `pmc`, `configs`, `q3f`, `dist` (defaults 10 / 100 / 100 / 2)
#   CONFIGS       benchmarks/configs.py configs for `configs` (default "sf10_filter q3_3way hybrid")
#   PMC_REGEX     kernel-name regex for `pmc` (default hs_jit_)
#   QK_ARGS       extra scripts/qk_sweep.py args for `pmc` (e.g. --only-q3-full)
#   Q3F_ARGS      extra scripts/qk_sweep.py args for `q3f` (e.g. --no-profile --cprofile=20)
#   NPROC         ranks for `dist` (gloo, all on cuda:0; default 4)
#   HS_PROFILE    1 = per-stage host/device tracer in the bench log
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
mkdir -p gpurun_out
export HS_BENCH_DIR=${HS_BENCH_DIR:-/tmp/hs_bench}
TAG=${TAG:-run}
O="$REPO/gpurun_out/$TAG"

step_tests() {
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -v -m gpu --timeout 240 \
    --timeout-method thread -x ${PYTEST_ARGS} > "${O}_tests.log" 2>&1
  local rc=$?
  echo "tests rc=$rc" >> "${O}_tests.log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ]
}

step_smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > "${O}_smoke.log" 2>&1
}

step_bench() {
  timeout -k 10 ${BENCH_TIMEOUT:-700} python bench.py ${BENCH_ARGS:---sf 100 --steps 100 --warmup 5 --host-breakdown 100} \
    > "${O}_bench.json" 2> "${O}_bench.log"
}

step_hostprof() {
  HS_BENCH_PROFILE=1 timeout -k 10 600 python bench.py ${BENCH_ARGS:---sf 100 --steps 40 --warmup 3 --no-crosscheck} \
    > "${O}_hostprof.json" 2> "${O}_hostprof.log"
}

step_prof() {
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d "${O}_prof" -o run \
     -- python3 "$REPO/bench.py" ${BENCH_ARGS:---sf 100 --steps 40 --warmup 5 --no-crosscheck} \
     > "${O}_prof.json" 2> "${O}_prof.log") || return $?
  find "${O}_prof" -name "*kernel_stats.csv" -exec cp {} "${O}_kernel_stats.csv" \;
}

step_benchtrace() {
  # kernel trace of the whole bench (name, start, end, queue, stream per dispatch); the timed
  # steps are the run of tags / bits-scan / scan kernels after the join-index side run
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 700 rocprofv3 --kernel-trace --output-format csv -d "${O}_btrace" -o run \
     -- python3 "$REPO/bench.py" ${BENCH_ARGS:---sf 100 --steps 60 --warmup 5 --no-crosscheck} \
     > "${O}_benchtrace.json" 2> "${O}_benchtrace.log") || return $?
  local f
  f=$(find "${O}_btrace" -name "*kernel_trace.csv" | head -n 1)
  python3 -c "
import csv, sys
r = csv.DictReader(open(sys.argv[1]))
w = csv.writer(open(sys.argv[2], 'w'))
w.writerow(['name', 'start', 'end', 'queue', 'stream'])
for x in r:
    w.writerow([x['Kernel_Name'][:60], x['Start_Timestamp'], x['End_Timestamp'], x['Queue_Id'], x['Stream_Id']])
" "$f" "${O}_bench_ktrace.csv"
  rm -rf "${O}_btrace"
}

step_pmc() {
  local sf=${SF:-10}
  timeout -k 10 600 python3 scripts/qk_sweep.py --sf $sf --reps 3 --configs '[{}]' ${QK_ARGS} \
    > "${O}_pmc_warm.jsonl" 2> "${O}_pmc_warm.log" || return $?
  local i=0
  # (a WRITE_SIZE pass hangs under rocprofv3 on this pool: left out)
  for P in "FETCH_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU TCP_TOTAL_CACHE_ACCESSES_sum"; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp &&
     timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "${PMC_REGEX:-hs_jit_}" --kernel-trace \
       --output-format csv -d "${O}_pmc/p$i" -o pmc -- python3 "$REPO/scripts/qk_sweep.py" --sf $sf \
       --reps 3 --configs '[{}]' ${QK_ARGS} > "${O}_pmc_run$i.jsonl" 2> "${O}_pmc_run$i.log") || return $?
    find "${O}_pmc/p$i" -name "*counter_collection.csv" -exec cp {} "${O}_pmc/counters$i.csv" \;
    find "${O}_pmc/p$i" -name "*kernel_trace.csv" -exec cp {} "${O}_pmc/trace$i.csv" \;
    rm -rf "${O}_pmc/p$i"
  done
  python3 scripts/pmc_summary.py "${O}_pmc"/counters*.csv "${O}_pmc"/trace*.csv > "${O}_pmc_summary.txt" 2>&1 || true
}

step_configs() {
  for c in ${CONFIGS:-sf10_filter q3_3way hybrid}; do
    rm -rf "$HS_BENCH_DIR"/indexes_* "$HS_BENCH_DIR"/cfg_* 2>/dev/null
    timeout -k 10 ${CFG_TIMEOUT:-420} python benchmarks/configs.py --config $c --sf ${SF:-100} \
      ${CFG_ARGS} >> "${O}_configs.jsonl" 2> "${O}_config_$c.log" || return $?
  done
  # the TPC-DS SF300 source files fill most of the box's /tmp: a later step's index write
  # failed with ENOSPC behind them (g33)
  rm -rf "$HS_BENCH_DIR"/indexes_* "$HS_BENCH_DIR"/cfg_* "$HS_BENCH_DIR"/tpcds_sf* 2>/dev/null
  return 0
}

step_cfgprof() {
  # kernel trace of one benchmarks/configs.py config (CONFIG, default hybrid); each timed loop
  # is bracketed by a spin kernel (HS_CFG_MARK): the kernels between two marks are one loop
  rm -rf "$HS_BENCH_DIR"/indexes_* "$HS_BENCH_DIR"/cfg_* 2>/dev/null
  (cd /tmp && export TMPDIR=/tmp && export HS_CFG_MARK=1 &&
   timeout -k 10 ${CFG_TIMEOUT:-500} rocprofv3 --kernel-trace --output-format csv -d "${O}_cfgprof" -o run \
     -- python3 "$REPO/benchmarks/configs.py" --config ${CONFIG:-hybrid} --sf ${SF:-100} ${CFG_ARGS} \
     > "${O}_cfgprof.jsonl" 2> "${O}_cfgprof.log") || return $?
  local f
  f=$(find "${O}_cfgprof" -name "*kernel_trace.csv" | head -n 1)
  python3 - "$f" "${O}_cfg_ktrace.csv" <<'PYEOF'
import csv, sys
r = csv.DictReader(open(sys.argv[1]))
w = csv.writer(open(sys.argv[2], 'w'))
w.writerow(['name', 'start', 'end', 'queue'])
for x in r:
    w.writerow([x['Kernel_Name'][:60], x['Start_Timestamp'], x['End_Timestamp'], x['Queue_Id']])
PYEOF
  rm -rf "${O}_cfgprof"
}

step_qk() {
  # query-kernel sweep: QK_CONFIGS (JSON list of kernel_config fields), QK_ARGS (e.g. --only-merge)
  local cfg="$QK_CONFIGS"
  [ -z "$cfg" ] && cfg='[{}]'
  timeout -k 10 ${QK_TIMEOUT:-600} python3 scripts/qk_sweep.py --sf ${SF:-100} --reps ${REPS:-20} \
    --configs "$cfg" ${QK_ARGS} > "${O}_qk.jsonl" 2> "${O}_qk.log"
}

step_qkprof() {
  # kernel trace of a query-kernel sweep (QK_CONFIGS, QK_ARGS); per-kernel durations of the
  # hs_jit_ kernels in dispatch order (config i's dispatches follow config i-1's)
  local cfg="$QK_CONFIGS"
  [ -z "$cfg" ] && cfg='[{}]'
  case "$cfg" in @/*) ;; @*) cfg="@$REPO/${cfg#@}" ;; esac   # the profiler runs from /tmp
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 ${QK_TIMEOUT:-600} rocprofv3 --kernel-trace --output-format csv -d "${O}_qkprof" \
     -o run -- python3 "$REPO/scripts/qk_sweep.py" --sf ${SF:-100} --reps ${REPS:-20} \
     --configs "$cfg" --no-profile ${QK_ARGS} > "${O}_qkprof.jsonl" 2> "${O}_qkprof.log") || return $?
  local f
  f=$(find "${O}_qkprof" -name "*kernel_trace.csv" | head -n 1)
  python3 -c "
import csv, sys
w = csv.writer(open(sys.argv[2], 'w'))
w.writerow(['name', 'start', 'end', 'vgpr', 'lds', 'grid'])
for x in csv.DictReader(open(sys.argv[1])):
    if x['Kernel_Name'].startswith('hs_'):
        w.writerow([x['Kernel_Name'][:48], x['Start_Timestamp'], x['End_Timestamp'],
                    x.get('VGPR_Count', ''), x.get('LDS_Block_Size', ''), x.get('Grid_Size', '')])
" "$f" "${O}_qk_ktrace.csv"
  rm -rf "${O}_qkprof"
}

step_pmcbench() {
  # one counter pass (PMC_COUNTERS) over the SF100 bench, counters on PMC_REGEX kernels only
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -s KILL ${PMC_TIMEOUT:-600} rocprofv3 --pmc ${PMC_COUNTERS:-FETCH_SIZE} \
     --kernel-include-regex "${PMC_REGEX:-hs_jit_run_bits_scan}" --kernel-trace --output-format csv \
     -d "${O}_pmcb" -o pmc -- python3 "$REPO/bench.py" --sf ${SF:-100} --steps 2 --warmup 1 \
     --no-crosscheck --no-side > "${O}_pmcb.json" 2> "${O}_pmcb.log") || return $?
  find "${O}_pmcb" -name "*counter_collection.csv" -exec cp {} "${O}_pmcb_counters.csv" \;
  find "${O}_pmcb" -name "*kernel_trace.csv" -exec cp {} "${O}_pmcb_trace.csv" \;
  rm -rf "${O}_pmcb"
  python3 scripts/pmc_summary.py "${O}_pmcb_counters.csv" "${O}_pmcb_trace.csv" > "${O}_pmcb_summary.txt" 2>&1 || true
}

step_hbm() {
  (rocm-smi --showclocks --showmemuse > "${O}_smi.txt" 2>&1 || true)
  timeout -k 10 120 python3 scripts/diag/hbm_probe.py 4 > "${O}_hbm.json" 2> "${O}_hbm.log"
}

step_q3f() {
  local cfg="$Q3F_CONFIGS"
  [ -z "$cfg" ] && cfg='[{}]'
  timeout -k 10 600 python3 scripts/qk_sweep.py --sf ${SF:-100} --reps 20 --only-q3-full \
    --configs "$cfg" ${Q3F_ARGS} > "${O}_q3f.jsonl" 2> "${O}_q3f.log"
}

step_q3fprof() {
  local cfg="$Q3F_CONFIGS"
  [ -z "$cfg" ] && cfg='[{}]'
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "${O}_q3fprof" -o run \
     -- python3 "$REPO/scripts/qk_sweep.py" --sf ${SF:-100} --reps 20 --only-q3-full \
     --configs "$cfg" --no-profile ${Q3F_ARGS} > "${O}_q3fprof.jsonl" 2> "${O}_q3fprof.log") \
    || return $?
  # the timed queries are the trace's tail (the head is data generation and index builds)
  local f
  f=$(find "${O}_q3fprof" -name "*kernel_trace.csv" | head -n 1)
  python3 -c "import sys; L=open(sys.argv[1]).readlines(); open(sys.argv[2], 'w').writelines(L[:1] + L[-3000:])" \
    "$f" "${O}_q3f_kernel_trace.csv"
  rm -rf "${O}_q3fprof"
}

step_dist() {
  local n=${NPROC:-4}
  HS_BENCH_DIR=/tmp/hs_bench_dist HS_DIST_BACKEND=gloo timeout -k 10 700 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus $n --sf ${SF:-2} --steps ${DIST_STEPS:-100} --warmup 3 \
    --buckets 16 ${DIST_ARGS} > "${O}_dist$n.json" 2> "${O}_dist$n.log"
}

step_build() {
  timeout -k 10 600 python scripts/build_bench.py --sf ${SF:-100} --codec ${CODEC:-snappy} \
    --repeat ${REPS:-2} ${BUILD_ARGS} >> "${O}_build.jsonl" 2>> "${O}_build.log"
}

step_buildprof() {
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
     -d "${O}_buildprof" -o run -- python3 "$REPO/scripts/build_bench.py" --sf ${SF:-100} \
     --codec ${CODEC:-snappy} ${BUILD_ARGS} > "${O}_buildprof.jsonl" 2> "${O}_buildprof.log") || return $?
  find "${O}_buildprof" -name "*kernel_stats.csv" -exec cp {} "${O}_build_kernel_stats.csv" \;
  find "${O}_buildprof" -name "*memory_copy_stats.csv" -exec cp {} "${O}_build_copy_stats.csv" \;
  # blit copies (grid size ~ bytes) and the SDMA copies, with timestamps, for the timeline
  local f
  f=$(find "${O}_buildprof" -name "*kernel_trace.csv" | head -n 1)
  [ -n "$f" ] && python3 -c "import sys; L=open(sys.argv[1]).readlines(); open(sys.argv[2], 'w').writelines(L[:1] + [l for l in L[1:] if 'copyBuffer' in l or 'snappy' in l or 'inflate' in l or 'gather' in l or 'rs_' in l])" "$f" "${O}_build_ktrace.csv"
  f=$(find "${O}_buildprof" -name "*memory_copy_trace.csv" | head -n 1)
  [ -n "$f" ] && cp "$f" "${O}_build_ctrace.csv"
  rm -rf "${O}_buildprof"
}

step_d2hprobe() {
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
     -d "${O}_d2h" -o run -- python3 "$REPO/scripts/diag/d2h_probe.py" \
     > "${O}_d2hprobe.jsonl" 2> "${O}_d2hprobe.log") || return $?
  find "${O}_d2h" -name "*kernel_stats.csv" -exec cp {} "${O}_d2h_kernel_stats.csv" \;
  find "${O}_d2h" -name "*memory_copy_stats.csv" -exec cp {} "${O}_d2h_copy_stats.csv" \;
  find "${O}_d2h" -name "*kernel_trace.csv" -exec cp {} "${O}_d2h_ktrace.csv" \;
  find "${O}_d2h" -name "*memory_copy_trace.csv" -exec cp {} "${O}_d2h_ctrace.csv" \;
  rm -rf "${O}_d2h"
}

step_cpubase() {
  timeout -k 10 840 python scripts/cpu_baseline.py --sf ${SF:-100} --threads 16 --reps ${REPS:-3} \
    --out "${O}_cpu_baseline.json" > "${O}_cpu.log" 2>&1
}

for s in "$@"; do
  echo "[gpu.sh] step $s $(date +%T)"
  "step_$s"
  rc=$?
  echo "[gpu.sh] step $s rc=$rc $(date +%T)"
  [ $rc -eq 0 ] || exit $rc
done
