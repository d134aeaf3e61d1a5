#!/bin/bash
# Hybrid Scan iteration: the device e2e tests (rc 1 does not stop the chain), then the hybrid and
# q3_3way side configs with the stage profile (HS_PROFILE=1).  Each step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench
TAG=${TAG:-hyb}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_e2e.py} -v -m gpu --timeout 240 \
  --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
HS_PROFILE=1 TAG=$TAG PART=configs CONFIGS="${CONFIGS:-hybrid q3_3way}" bash scripts/gpu_r4_side.sh
rc=$?
[ $rc -ne 0 ] && exit $rc
if [ -n "$RECORD" ]; then
  # kernel sources the bench generates, for the ahead-of-time set (hyperspace_amd/_native/aot)
  HS_JIT_RECORD=gpurun_out/aot_${TAG} timeout -k 10 600 python bench.py --sf 100 --steps 100 \
    --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit $?
fi
