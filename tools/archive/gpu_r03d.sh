#!/bin/bash
# Cauchy-solve syndrome decode: its GPU parity tests, then the in-process A/B against the direct
# decode (tools/syn_ab.py) and a kernel-time profile of the 16-lost (64,96) case.  Each step
# under its own timeout; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== syndrome tests" && timeout -k 10 400 python3 -u -m pytest tests/test_gpu_syndrome.py -x -v --timeout 120 --timeout-method thread > $O/pt_syn.log 2>&1 || { tail -40 $O/pt_syn.log; exit 1; }
tail -1 $O/pt_syn.log
echo "== syn A/B" && timeout -k 10 500 python3 -u tools/syn_ab.py --rounds 2 --variants "direct@SEC_SYN=0,two@SEC_SYN=1+SEC_SYN_FUSED=0,fused@SEC_SYN=1,auto" > $O/syn_ab.jsonl 2> $O/syn_ab.err || { tail -20 $O/syn_ab.err; exit 1; }
cat $O/syn_ab.jsonl
echo "== rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_syn -o run -- python3 tools/syn_ab.py --cases "1MiB x1024" --variants "two@SEC_SYN=1+SEC_SYN_FUSED=0,fused@SEC_SYN=1" --rounds 1 > $O/prof_syn.log 2>&1 || { tail -10 $O/prof_syn.log; exit 1; }
cut -d, -f1-5 $O/prof_syn/run_kernel_stats.csv | head -8
