set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/sweep.py --variants base --us 1,2 --rounds 2 --workload ${W:-1024,1048576,10,14} 2>&1 | tail -25
