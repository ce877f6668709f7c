#!/bin/bash
# Round 4: wide-decode counters for the one-wave, wave-pair (own rings / shared transposes) and
# two-kernel decodes, then the host-allocator runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
VARS="auto,pshared/pshared,two@SEC_SYN=1+SEC_SYN_FUSED=0+SEC_SYN_PAIR=0" bash tools/gpu_syn_pmc.sh || exit 1
bash tools/gpu_upload_malloc.sh
