# A/B of bignum.hip build variants (storb_amd/lib/libstorbec_bn_*.so) on the APDP kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/bn_variants.jsonl
for v in ${VARIANTS:-bn_perm bn_dpp bn_dpp_u64 bn_dpp_u16}; do
  STORB_EC_LIB=storb_amd/lib/libstorbec_$v.so timeout -k 10 120 python tools/bench_apdp.py --quick > gpurun_out/bn_$v.json 2>> gpurun_out/bn_variants.err || exit $?
  echo "{\"variant\": \"$v\", \"res\": $(cat gpurun_out/bn_$v.json)}" >> gpurun_out/bn_variants.jsonl
done
cat gpurun_out/bn_variants.jsonl
