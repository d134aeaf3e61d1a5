#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box: NPROC (default 2) ranks share cuda:0, collectives over gloo (host-staged).
# Exercises the distributed build (all-to-all shuffle), bucket ownership, partial-aggregate
# all-reduce and row all-gather exactly as the RCCL path does, minus RCCL itself.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export HS_BENCH_DIR=/tmp/hs_bench_dist HS_DIST_BACKEND=gloo
N=${NPROC:-2}
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $N --sf ${SF:-2} --steps 5 --warmup 2 \
  --buckets 16 > gpurun_out/dist$N.json 2> gpurun_out/dist$N.log
rc=$?
echo "dist rc=$rc" >> gpurun_out/dist$N.log
exit $rc
