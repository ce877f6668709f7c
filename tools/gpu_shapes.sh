set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O
for w in c4 8192,65600,10,14 1024,655360,10,14 8192,65536,4,6 16384,32768,4,6 1024,1048576,8,11 1024,1048576,10,14; do
  echo "== $w"; timeout -k 10 200 python tools/sweep.py --variants base --us 1,2 --rounds 3 --workload $w 2>&1 | grep variant || exit 1
done
