#!/bin/bash
# LDS-table A/B (kernels.hip SEC_LDS_TAB), one process per workload, variants interleaved in-process.
#   VARIANTS (default base,noldstab), WORKLOADS (default: the 8-row-group shapes and C2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
: > $O/ldstab.jsonl
for W in ${WORKLOADS:-1024,1048576,16,24 1024,1048576,32,48 256,1048576,64,96 c2}; do
  timeout -k 10 300 python3 -u tools/sweep.py --workload $W --us 1 --rounds 7 --variants ${VARIANTS:-base,noldstab} >> $O/ldstab.jsonl 2> $O/ldstab.err || { tail -20 $O/ldstab.err; exit 1; }
done
cat $O/ldstab.jsonl
