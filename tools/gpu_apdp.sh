# F4 APDP: GPU parity tests, then the throughput bench (VARIANTS: A/B build tags).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_apdp_gpu.py -x -q > gpurun_out/apdp_tests.log 2>&1
rc=$?
tail -15 gpurun_out/apdp_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/bn_variants.jsonl
for v in ${VARIANTS:-}; do
  STORB_EC_LIB=storb_amd/lib/libstorbec_$v.so timeout -k 10 120 python tools/bench_apdp.py --quick > gpurun_out/bn_$v.json 2>> gpurun_out/bn_variants.err || exit $?
  echo "{\"variant\": \"$v\", \"res\": $(cat gpurun_out/bn_$v.json)}" >> gpurun_out/bn_variants.jsonl
done
cat gpurun_out/bn_variants.jsonl
if [ -n "${FULL:-}" ]; then
  timeout -k 10 300 python tools/bench_apdp.py > gpurun_out/apdp.json 2> gpurun_out/apdp.err || exit $?
  cat gpurun_out/apdp.json
fi
