set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== tests" && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_syndrome.py > $O/pt_split.log 2>&1 || { tail -30 $O/pt_split.log; exit 1; }
tail -1 $O/pt_split.log
echo "== syn A/B" && timeout -k 10 600 python3 -u tools/syn_ab.py --rounds 5 --variants "auto,nosplit/nosplit,auto2,nosplit2/nosplit" --cases "32 lost;24 lost (random;30 %;16 lost (random" > $O/syn_ab_split.jsonl 2> $O/syn_ab_split.err || { tail -20 $O/syn_ab_split.err; exit 1; }
cat $O/syn_ab_split.jsonl
