#!/bin/bash
# Syndrome decode with per-row skips in the solve: tests + A/B (fixed and random patterns).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== syndrome tests" && timeout -k 10 400 python3 -u -m pytest tests/test_gpu_syndrome.py -x -v --timeout 120 --timeout-method thread > $O/pt_syn.log 2>&1 || { tail -40 $O/pt_syn.log; exit 1; }
tail -1 $O/pt_syn.log
echo "== syn A/B" && timeout -k 10 700 python3 -u tools/syn_ab.py --rounds 2 --variants "direct@SEC_SYN=0,two@SEC_SYN=1+SEC_SYN_FUSED=0,fused@SEC_SYN=1" > $O/syn_ab.jsonl 2> $O/syn_ab.err || { tail -20 $O/syn_ab.err; exit 1; }
cat $O/syn_ab.jsonl
