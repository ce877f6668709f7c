#!/bin/bash
# Rehearsal of the N = 2 launch on a one-GPU box: two ranks under torch.distributed.run share
# cuda:0 over gloo (STORB_BENCH_DEVICE / STORB_DIST_BACKEND overrides; the driver's runs set
# neither and get one GPU per rank over RCCL).  Checks the partition, the timed region's
# barriers and the max / sum reductions end to end; the rates are meaningless (one GPU).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export STORB_BENCH_DEVICE=0 STORB_DIST_BACKEND=gloo
for W in c2c3 c4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --workload $W --no-cpu --no-e2e --c4-chunks 16384 \
    > $O/rehearse_n2_$W.log 2>&1 || { tail -30 $O/rehearse_n2_$W.log; exit 1; }
  grep '^{' $O/rehearse_n2_$W.log
done
