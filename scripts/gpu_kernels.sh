#!/bin/bash
# First GPU check: kernel numerics.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/kernels_test.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/kernels_test.log
exit $rc
