set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/gpu_c4_lds.sh || exit 1
echo "== syn A/B" && timeout -k 10 600 python3 -u tools/syn_ab.py --rounds 3 --variants "two@SEC_SYN=1+SEC_SYN_FUSED=0,two8@SEC_SYN=1+SEC_SYN_FUSED=0/snr8,two8w4@SEC_SYN=1+SEC_SYN_FUSED=0/snr8w4,auto" --cases "32 lost;24 lost;30 %;rows 64..73" > $O/syn_ab_r04a.jsonl 2> $O/syn_ab_r04a.err || { tail -20 $O/syn_ab_r04a.err; exit 1; }
cat $O/syn_ab_r04a.jsonl
