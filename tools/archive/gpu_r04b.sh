set -o pipefail
# Round 4: the two-wave syndrome decode (SEC_SYN_PAIR) on the GPU -- its parity tests, then its
# A/B against the cost rule without it and the plain two-kernel decode, on the zfec(64,96) cases
# whose present parity rows lie in both groups (tools/syn_ab.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== tests" && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_syndrome.py tests/test_gpu_choose.py tests/test_gpu_bs.py tests/test_gpu_decode_ex.py > $O/pt_pair.log 2>&1 || { tail -30 $O/pt_pair.log; exit 1; }
tail -2 $O/pt_pair.log
echo "== syn A/B" && timeout -k 10 600 python3 -u tools/syn_ab.py --rounds 3 --variants "auto,nopair@SEC_SYN_PAIR=0,two@SEC_SYN=1+SEC_SYN_FUSED=0+SEC_SYN_PAIR=0" --cases "16 lost (random;24 lost (random;15 %;20 %;30 %;rows 64..73;32 lost" > $O/syn_ab_pair.jsonl 2> $O/syn_ab_pair.err || { tail -20 $O/syn_ab_pair.err; exit 1; }
cat $O/syn_ab_pair.jsonl
