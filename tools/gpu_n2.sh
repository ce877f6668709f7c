#!/bin/bash
# Rehearsal of the driver's N>1 bench launch on a one-GPU box: 2 ranks share GPU 0 and talk
# over gloo (STORB_BENCH_DEVICE / STORB_DIST_BACKEND); the driver's 8-GPU runs set neither.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
STORB_BENCH_DEVICE=0 STORB_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 \
  > $O/bench_n2.log 2>&1 || { tail -30 $O/bench_n2.log; exit 1; }
tail -1 $O/bench_n2.log
