#!/bin/bash
# Fused syndrome decode with the LDS-DMA ring: syndrome tests (default build), then the A/B
# against the register ring (libstorbec_nolds.so) on the cases where the fused kernel runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== syndrome tests" && timeout -k 10 400 python3 -u -m pytest tests/test_gpu_syndrome.py -x -v --timeout 120 --timeout-method thread > $O/pt_syn.log 2>&1 || { tail -40 $O/pt_syn.log; exit 1; }
tail -1 $O/pt_syn.log
echo "== syn A/B" && timeout -k 10 700 python3 -u tools/syn_ab.py --rounds 3 --variants "direct@SEC_SYN=0,fused@SEC_SYN=1,fused_regring@SEC_SYN=1/nolds" > $O/syn_ab_lds.jsonl 2> $O/syn_ab_lds.err || { tail -20 $O/syn_ab_lds.err; exit 1; }
cat $O/syn_ab_lds.jsonl
