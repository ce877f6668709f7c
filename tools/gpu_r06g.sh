#!/bin/bash
# Round 6 (VAR=pinkeep, the default): per-call staging returned to the process pool (this build) against contexts that keep
# their staging between calls (build/variants/libstorbec_pinkeep.so, SEC_PIN_RETURN=0): the
# small-call profile and the 1 GiB stream rates, each library twice, alternating.  VAR=pool14: the
# library task pool at 14 threads (SEC_POOL_THREADS_MAX=14, _DIV=1) against 7.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
V=$R/build/variants/libstorbec_${VAR:-pinkeep}.so
for i in 1 2; do
  for L in pool keep; do
    if [ $L = keep ]; then export STORB_EC_LIB=$V; else unset STORB_EC_LIB; fi
    echo "== $L $i small" && timeout -k 10 300 python3 -u tools/small_call_profile.py --reps 100 > $O/pin_${L}_${i}_small.json 2> $O/pin_${L}_${i}_small.err || { tail -20 $O/pin_${L}_${i}_small.err; exit 1; }
    echo "== $L $i stream" && timeout -k 10 400 python3 -u tools/stream_rate.py --mib 1024 --reps 3 > $O/pin_${L}_${i}_stream.json 2> $O/pin_${L}_${i}_stream.err || { tail -20 $O/pin_${L}_${i}_stream.err; exit 1; }
  done
done
unset STORB_EC_LIB
python3 - <<PY
import json
for i in (1, 2):
    for L in ("pool", "keep"):
        s = json.load(open(f"$O/pin_{L}_{i}_small.json")); t = json.load(open(f"$O/pin_{L}_{i}_stream.json"))
        print(L, i, {k: (v.get("encode_chunk"), v.get("encode_chunk_plus_ids"), v.get("lib_call")) for k, v in s.items() if isinstance(v, dict)},
              {k: v for k, v in t.items() if k.startswith(("upload", "download_stream"))})
PY
