#!/bin/bash
# SHA-1: the default build (next-block prefetch below 65536 messages) against prefetch off (sha1nopf), twice each, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sha1.py > $O/sha1_tests.log 2>&1 || { tail -30 $O/sha1_tests.log; exit 1; }
tail -1 $O/sha1_tests.log
for i in ${ROUNDS:-1 2}; do
  for L in ${LIBS:-storb_amd/lib/libstorbec.so storb_amd/lib/libstorbec_sha1nopf.so}; do
    timeout -k 10 300 python -u tools/sha1_study.py $L >> $O/sha1pf.jsonl 2>$O/sha1pf.err || { tail -20 $O/sha1pf.err; exit 1; }
  done
done
cat $O/sha1pf.jsonl
