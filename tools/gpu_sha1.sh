#!/bin/bash
# SHA-1 kernel: GPU tests, then the study with the previous build (base) and the current one
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O
echo "== sha1 tests" && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sha1.py > $O/sha1_tests.log 2>&1 || { tail -30 $O/sha1_tests.log; exit 1; }
tail -1 $O/sha1_tests.log
echo "== study" && timeout -k 10 300 python -u tools/sha1_study.py storb_amd/lib/libstorbec_base.so > $O/sha1_study.jsonl 2>&1 && timeout -k 10 300 python -u tools/sha1_study.py >> $O/sha1_study.jsonl 2>&1 || { tail -20 $O/sha1_study.jsonl; exit 1; }
grep '^{' $O/sha1_study.jsonl
