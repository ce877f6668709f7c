#!/bin/bash
# Round 6 evidence, part 2: every BASELINE config (tools/bench_configs.py), the in-process form on
# two contexts of the one GPU, the wide-decode A/B of the final build, the per-call profile, the
# C1 loopback and the 1 GiB object's upload / download loops.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== configs" && timeout -k 10 600 python3 -u tools/bench_configs.py > $O/configs.json 2> $O/configs.err || { tail -30 $O/configs.err; exit 1; }
echo "== in-process 0,0" && timeout -k 10 300 python3 -u bench.py --gpus 2 --in-process --inproc-devices 0,0 --steps 20 --warmup 3 --c5-steps 5 > $O/inproc00.log 2>&1 || { tail -30 $O/inproc00.log; exit 1; }
grep '^{' $O/inproc00.log
echo "== syn A/B" && timeout -k 10 600 python3 -u tools/syn_ab.py --rounds 3 --variants "auto,direct@SEC_SYN=0" --cases "32 lost;24 lost (random;30 %;16 lost (random;20 %;rows 64..73" > $O/syn_ab_final.jsonl 2> $O/syn_ab_final.err || { tail -20 $O/syn_ab_final.err; exit 1; }
echo "== small calls" && timeout -k 10 300 python3 -u tools/small_call_profile.py --reps 100 > $O/small_calls.json 2> $O/small_calls.err || { tail -20 $O/small_calls.err; exit 1; }
echo "== c1" && timeout -k 10 300 python3 -u tools/c1_loopback.py --reps 20 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
cat $O/c1.json
echo "== stream rate" && timeout -k 10 600 python3 -u tools/stream_rate.py --mib 1024 --reps 3 > $O/stream_rate.json 2> $O/stream_rate.err || { tail -20 $O/stream_rate.err; exit 1; }
cat $O/stream_rate.json
