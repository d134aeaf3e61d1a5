#!/bin/bash
# Round-4 validation on one MI355X: every GPU test, smoke(), the SF100 bench (100 timed steps),
# a rocprofv3 kernel-stats pass over a 40-step bench, and the Hybrid Scan config with the stage
# profile.  Each GPU step has its own time limit; a crash / abort / time limit ends the script
# (a plain test failure, rc 1, does not).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
REPO="$(pwd)"
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
TAG=${TAG:-fin}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 240 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --sf 100 --steps 100 --warmup 5 --host-breakdown 100 \
  > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof_${TAG}" \
  -o run -- python "$REPO/bench.py" --sf 100 --steps 40 --warmup 5 --no-crosscheck \
  > "$REPO/gpurun_out/${TAG}_prof.json" 2> "$REPO/gpurun_out/${TAG}_prof.log" || exit $?
cd "$REPO"
[ -n "$NOHYB" ] && exit 0
HS_PROFILE=1 TAG=$TAG PART=configs CONFIGS="${CONFIGS:-hybrid}" bash scripts/gpu_r4_side.sh
