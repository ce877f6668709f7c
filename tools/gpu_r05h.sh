#!/bin/bash
# Round 5: phase 2 of the wide decode persistent + double-buffered (SEC_SOLVE_PIPE=1 variant
# library) against the shipped one-workgroup-per-span kernel, tools/syn_ab.py, and the syndrome
# GPU tests on the variant (bit-exactness of the new kernel).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== syndrome tests on the pipe variant" && STORB_EC_LIB=$R/storb_amd/lib/libstorbec_pipe.so timeout -k 10 300 python -u -m pytest tests/test_gpu_syndrome.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/syn_tests_pipe.log 2>&1 || { tail -30 $O/syn_tests_pipe.log; exit 1; }
tail -2 $O/syn_tests_pipe.log
echo "== syn A/B" && timeout -k 10 600 python3 -u tools/syn_ab.py --rounds 3 --reps 5 --modes reassemble --variants "auto,pipe/pipe" --cases "32 lost;24 lost (random;16 lost (random;30 % of blocks lost, first;zfec(32,48) 1MiB x1024, 16 lost (every;12 lost (random" > $O/syn_ab_pipe.jsonl 2> $O/syn_ab_pipe.err || { tail -20 $O/syn_ab_pipe.err; exit 1; }
cat $O/syn_ab_pipe.jsonl
