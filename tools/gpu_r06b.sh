#!/bin/bash
# Round 6: the GPU suite on the new kernels (pair encode, rank-ordered phase-1 ring, pipelined
# solve), then the A/Bs: wide encodes (pair / interleaved / planes-only pair) and wide decodes
# (this build / the round-5 kernels, build/variants/libstorbec_r05.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
[ -n "$NO_TESTS" ] || bash tools/gpu_tests.sh || exit 1
echo "== enc A/B" && timeout -k 10 400 python3 -u tools/enc_ab.py --rounds 3 --reps 5 --variants "pair,bs2@SEC_BS_PAIR=0,planes/planes" > $O/r06_enc_ab.jsonl 2> $O/r06_enc_ab.err || { tail -20 $O/r06_enc_ab.err; exit 1; }
cat $O/r06_enc_ab.jsonl
echo "== syn A/B" && timeout -k 10 500 python3 -u tools/syn_ab.py --rounds 3 --variants "auto,r05/r05,snr16/snr16" --cases "32 lost;24 lost (random;16 lost (random;x1024, 16 lost;30 %;14 data" > $O/r06_syn_ab.jsonl 2> $O/r06_syn_ab.err || { tail -20 $O/r06_syn_ab.err; exit 1; }
cat $O/r06_syn_ab.jsonl
