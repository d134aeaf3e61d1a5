#!/bin/bash
# Kernel-level sweep of the generated join kernel on an SF-shaped device table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python scripts/microbench_join.py --sf ${SF:-100} --quick --no-scan \
  --items ${ITEMS:-1,2,4} --grids ${GRIDS:-8192,16384} --stage ${STAGE:-0,1} --pipe ${PIPE:-1,0} --direct ${DIRECT:-1,0} \
  > gpurun_out/mb6.jsonl 2> gpurun_out/mb6.log
