# decode batching A/B: base vs decb8 vs decb16 on C2, C4 and an RS(8,3) 1 MiB shape
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
: > $O/sweep_dec.jsonl
for w in c2 c4 1024,1048576,8,11; do
  timeout -k 10 300 python tools/sweep.py --variants ${VARS:-base,decb8,decb16} --us ${US:-1,2,4} --rounds 4 --workload $w >> $O/sweep_dec.jsonl 2>&1 || exit $?
done
grep variant $O/sweep_dec.jsonl
