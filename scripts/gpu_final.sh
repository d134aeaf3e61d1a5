#!/bin/bash
# Round-end validation: GPU tests (one pytest process), smoke, SF100 bench, kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
SKIP_DIST=1 bash scripts/gpu_iter.sh || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/smoke.log 2>&1 || exit 1
bash scripts/gpu_profile.sh
