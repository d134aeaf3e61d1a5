#!/bin/bash
# Record the kernel sources of the benchmark workload on a GPU box (run through gpurun), for the
# ahead-of-time set in hyperspace_amd/_native/aot/ (compiled by __graft_entry__.build()):
#   gpurun -- bash scripts/record_aot.sh && cp gpurun_out/aot/*.hip hyperspace_amd/_native/aot/
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/aot
HS_JIT_RECORD=gpurun_out/aot timeout -k 10 600 python3 -u bench.py --steps 3 \
  > gpurun_out/record_aot.json 2> gpurun_out/record_aot.log
