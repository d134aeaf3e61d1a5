#!/bin/bash
# Phase-1 (run tags) tunables on the headline: bench.py at SF100 per setting (gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/sweep_rt2.jsonl
: > $out
for cfg in "" "HS_JIT_RT2_UNROLL=2" "HS_JIT_RT2_UNROLL=8" "HS_JIT_RT2_GRID=4096" "HS_JIT_RT2_GRID=16384"; do
  echo "[sweep] ${cfg:-default} $(date +%T)"
  env $cfg timeout -k 10 240 python3 bench.py --sf 100 --steps 40 --warmup 5 --no-side --no-crosscheck \
    > gpurun_out/sweep_one.json 2> gpurun_out/sweep_one.log || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep_one.json')); print(json.dumps({'cfg': sys.argv[1], 'qps': d['value'], 'ms_per_step': d['ms_per_step'], 'q3_ms': d['latency']['q3_join_ms']}))" "${cfg:-default}" >> $out
done
