#!/bin/bash
# In-process A/B (tools/sweep.py) over several workloads, one process per workload, variants
# interleaved in-process; output gpurun_out/ab.jsonl.
#   VARIANTS (default base,noldstab: the SEC_LDS_TAB A/B), WORKLOADS (default: the 8-row-group
#   shapes and C2), SWEEP_ARGS (extra sweep.py arguments, e.g. --recover)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
: > $O/ab.jsonl
for W in ${WORKLOADS:-1024,1048576,16,24 1024,1048576,32,48 256,1048576,64,96 c2}; do
  timeout -k 10 300 python3 -u tools/sweep.py --workload $W --us 1 --rounds 7 ${SWEEP_ARGS:-} --variants ${VARIANTS:-base,noldstab} >> $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
done
cat $O/ab.jsonl
