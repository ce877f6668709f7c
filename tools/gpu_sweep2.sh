set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O
echo "== sweep c2" && timeout -k 10 400 python -u tools/sweep.py --variants base,dst2,dst0,est2,xcd,xcd_dst0,xcd_dst2 --us 4,1 --rounds 3 > $O/sweep2_c2.jsonl 2>&1 || { tail -20 $O/sweep2_c2.jsonl; exit 1; }
cat $O/sweep2_c2.jsonl
echo "== sweep c4" && timeout -k 10 400 python -u tools/sweep.py --workload c4 --variants base,dst2,xcd,xcd_dst2 --us 1 --rounds 3 > $O/sweep2_c4.jsonl 2>&1 || { tail -20 $O/sweep2_c4.jsonl; exit 1; }
cat $O/sweep2_c4.jsonl
echo "== e2e 15 copy threads" && SEC_COPY_THREADS=15 timeout -k 10 300 python -u tools/e2e_study.py > $O/e2e_study15.json 2>&1 || { tail -20 $O/e2e_study15.json; exit 1; }
tail -1 $O/e2e_study15.json
