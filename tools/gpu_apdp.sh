# F4 APDP: GPU parity tests, then the throughput bench.  Run via gpurun from the repo root.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_apdp_gpu.py -x -q > gpurun_out/apdp_tests.log 2>&1 && \
timeout -k 10 300 python tools/bench_apdp.py > gpurun_out/apdp.json 2> gpurun_out/apdp.err
rc=$?
tail -5 gpurun_out/apdp_tests.log
cat gpurun_out/apdp.json
tail -5 gpurun_out/apdp.err
exit $rc
