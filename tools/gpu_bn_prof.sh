# Integer-multiply ceilings + rocprofv3 kernel stats of the APDP kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/mad_ceiling > gpurun_out/mad_ceiling.json 2>&1 && cat gpurun_out/mad_ceiling.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_apdp -o apdp -- python3 tools/bench_apdp.py --quick > gpurun_out/apdp_prof_run.json 2> gpurun_out/apdp_prof.err
rc=$?
find gpurun_out/prof_apdp -name "*stats*" | head
exit $rc
