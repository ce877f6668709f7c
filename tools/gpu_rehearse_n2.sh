#!/bin/bash
# Rehearsal of the N = 2 launch on a one-GPU box: `bench.py --gpus 2` spawns its two ranks itself
# (no torch.distributed.run), both on cuda:0 over gloo (STORB_BENCH_DEVICE / STORB_DIST_BACKEND
# overrides; the driver's runs set neither and get one GPU per rank over RCCL).  Checks the
# launch, the partition, the timed region's barriers and the max / sum reductions end to end;
# the rates are meaningless (one GPU, two ranks).  The c2c3 line's nested in-process measurement
# (rank 0 drives both "devices" from one process while rank 1 waits) runs on two contexts of cuda:0.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export STORB_BENCH_DEVICE=0 STORB_DIST_BACKEND=gloo
for W in c2c3 c4 c5; do
  timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --workload $W --no-cpu --no-e2e \
    --c4-chunks 16384 --c5-bytes 268435456 --inproc-devices 0,0 > $O/rehearse_n2_$W.log 2>&1 || { tail -30 $O/rehearse_n2_$W.log; exit 1; }
  grep '^{' $O/rehearse_n2_$W.log
done
