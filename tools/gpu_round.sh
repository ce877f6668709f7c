#!/bin/bash
# Round evidence in one GPU call: gpu tests -> smoke -> bench -> rocprofv3 kernel stats of the
# bench (after the PMC traffic of c2 / c4 / c5, tools/gpu_pmc.sh, which the bench lines then carry)
# -> bench --workload c4 / c5 -> the --gpus 2 rehearsal
# -> every BASELINE config (tools/bench_configs.py).  Each step
# under its own timeout; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== pytest gpu" && timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
echo "== smoke" && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -z "$SKIP_PMC" ]; then  # first, so the bench lines below carry this build's traffic
  for W in c2 c4 c5; do echo "== pmc $W" && bash tools/gpu_pmc.sh $W > $O/pmc_$W.log 2>&1 || { tail -30 $O/pmc_$W.log; exit 1; }
    cp $O/pmc_$W.json $R/profiles/pmc_$W.json; done
fi
echo "== bench" && timeout -k 10 300 python3 -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
echo "== rocprofv3 stats" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-recover --no-c4 --no-c5 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
echo "== bench c4" && timeout -k 10 300 python3 -u bench.py --workload c4 > $O/bench_c4.log 2>&1 || { tail -30 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log
echo "== bench c5" && timeout -k 10 300 python3 -u bench.py --workload c5 > $O/bench_c5.log 2>&1 || { tail -30 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log
echo "== rehearse --gpus 2 (two ranks on one GPU, gloo)" && bash tools/gpu_rehearse_n2.sh > $O/rehearse.log 2>&1 || { tail -30 $O/rehearse.log; exit 1; }
cat $O/rehearse.log
[ -n "$SKIP_CONFIGS" ] && exit 0
echo "== configs" && timeout -k 10 600 python3 -u tools/bench_configs.py > $O/configs.json 2> $O/configs.err || { tail -30 $O/configs.err; exit 1; }
cat $O/configs.json
