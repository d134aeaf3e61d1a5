set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_parquet.py tests/test_jit.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_snappy.log 2>&1 && bash scripts/gpu_bench_sf100.sh
