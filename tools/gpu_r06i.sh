#!/bin/bash
# Round 6: library task pool A/Bs (VAR=p12: pool size; VAR=hashpool / joinpool: the second pool for piece copies + ids / host-only joins, measured as variants before they became the product) on what they move: the C5 end-to-end line (pinned host
# memory, the host joins beside the zero-copy kernels) and the 1 GiB piece streams.  This build
# against build/variants/libstorbec_${VAR}.so, alternating, twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
V=$R/build/variants/libstorbec_${VAR:-p12}.so
for i in 1 2; do
  for L in base var; do
    if [ $L = var ]; then export STORB_EC_LIB=$V; else unset STORB_EC_LIB; fi
    echo "== $L $i c5" && timeout -k 10 300 python3 -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu > $O/pt_${L}_${i}_c5.log 2>&1 || { tail -20 $O/pt_${L}_${i}_c5.log; exit 1; }
    echo "== $L $i stream" && timeout -k 10 400 python3 -u tools/stream_rate.py --mib 1024 --reps 2 > $O/pt_${L}_${i}_stream.json 2> $O/pt_${L}_${i}_stream.err || { tail -20 $O/pt_${L}_${i}_stream.err; exit 1; }
    echo "== $L $i small" && timeout -k 10 300 python3 -u tools/small_call_profile.py --reps 100 > $O/pt_${L}_${i}_small.json 2> $O/pt_${L}_${i}_small.err || { tail -20 $O/pt_${L}_${i}_small.err; exit 1; }
  done
done
unset STORB_EC_LIB
python3 - <<PY
import json
for i in (1, 2):
    for L in ("base", "var"):
        c5 = [json.loads(l) for l in open(f"$O/pt_{L}_{i}_c5.log") if l.startswith("{")][-1]
        t = json.load(open(f"$O/pt_{L}_{i}_stream.json"))
        sm = json.load(open(f"$O/pt_{L}_{i}_small.json"))
        print(L, i, "c5", c5["value"], (c5.get("staged") or {}).get("decode_gibs"), {k: v for k, v in t.items() if k in ("upload_per_chunk", "upload_stream", "download_stream_all_data_present", "download_stream_data_piece_0_lost")},
              {k: (v.get("encode_chunk"), v.get("encode_chunk_plus_ids")) for k, v in sm.items() if isinstance(v, dict)})
PY
