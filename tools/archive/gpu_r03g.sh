#!/bin/bash
# Syndrome decode: tests, then the ring-depth A/B (fused ring 6: libstorbec_fr6.so; two-kernel
# rings 4: libstorbec_synr4.so) against the default build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== syndrome tests" && timeout -k 10 400 python3 -u -m pytest tests/test_gpu_syndrome.py -x -v --timeout 120 --timeout-method thread > $O/pt_syn.log 2>&1 || { tail -40 $O/pt_syn.log; exit 1; }
tail -1 $O/pt_syn.log
echo "== syn A/B" && timeout -k 10 800 python3 -u tools/syn_ab.py --rounds 2 --variants "direct@SEC_SYN=0,two@SEC_SYN=1+SEC_SYN_FUSED=0,fused@SEC_SYN=1,two_r4@SEC_SYN=1+SEC_SYN_FUSED=0/synr4,fused_r6@SEC_SYN=1/fr6" > $O/syn_ab.jsonl 2> $O/syn_ab.err || { tail -20 $O/syn_ab.err; exit 1; }
cat $O/syn_ab.jsonl
