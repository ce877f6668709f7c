#!/bin/bash
# wide-k A/B: W kernels with 8-vector batches + block pairs for 8-row groups (base) against the
# earlier 16-vector batches without pairs (prevwide); 8-row groups routed to W from k > 8; + GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== pytest gpu" && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
V=${V:-base,prevwide,base@SEC_WIDE_K8=8}
for w in 512,2097152,16,24 1024,786432,12,20 256,4194304,32,48 64,4194304,64,96 c2 c4 c5; do
  timeout -k 10 300 python -u tools/sweep.py --variants $V --us 1 --workload $w >> $O/wide.jsonl 2>$O/wide.err || { tail -20 $O/wide.err; exit 1; }
done
cat $O/wide.jsonl
