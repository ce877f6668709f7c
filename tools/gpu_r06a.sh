#!/bin/bash
# Round 6, first call: the GPU suite + smoke on the shared-pool build, then the wide-kernel counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/gpu_tests.sh && bash tools/gpu_r06_pmc.sh
