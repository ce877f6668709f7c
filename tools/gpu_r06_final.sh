#!/bin/bash
# Round 6 evidence, part 1: tools/gpu_round.sh without the configs sweep (GPU tests, smoke, PMC
# c2/c4/c5 on this build, bench lines, kernel stats, --gpus 2 rehearsal with the nested
# in-process form).  Part 2: tools/gpu_r06_final2.sh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
SKIP_CONFIGS=1 bash tools/gpu_round.sh || exit 1
