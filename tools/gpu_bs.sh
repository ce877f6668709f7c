#!/bin/bash
# Bit-sliced encode (kernels_bs.hip): its GPU parity tests, then an in-process A/B against the
# v_perm / xb kernels (SEC_BS=0) on C4, C5 and the policy's wide shapes at their chunk sizes;
# output gpurun_out/bs_ab.jsonl.  TESTS=0 skips the tests, WORKLOADS overrides the list.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
if [ "${TESTS:-1}" != 0 ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bs.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_bs.log 2>&1 || { tail -40 $O/pytest_bs.log; exit 1; }
  tail -1 $O/pytest_bs.log
fi
: > $O/bs_ab.jsonl
for W in ${WORKLOADS:-c4 c5 1024,1048576,16,24 256,4194304,8,12 64,16777216,16,24 1024,1048576,32,48 16,67108864,32,48 256,1048576,64,96 4,268435456,64,96}; do
  timeout -k 10 300 python3 -u tools/sweep.py --workload $W --us 1 --rounds ${ROUNDS:-5} --variants ${VARIANTS:-base,base@SEC_BS=0} >> $O/bs_ab.jsonl 2> $O/bs_ab.err || { tail -20 $O/bs_ab.err; exit 1; }
done
cat $O/bs_ab.jsonl
