#!/bin/bash
# Round 6: the GPU suite on the build that faults in unbacked output pages before locking them,
# then the host paths it touches (small calls, 1 GiB streams, the e2e configs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
echo "== small calls" && timeout -k 10 300 python3 -u tools/small_call_profile.py --reps 100 > $O/h_small.json 2> $O/h_small.err || { tail -20 $O/h_small.err; exit 1; }
echo "== stream" && timeout -k 10 400 python3 -u tools/stream_rate.py --mib 1024 --reps 3 > $O/h_stream.json 2> $O/h_stream.err || { tail -20 $O/h_stream.err; exit 1; }
python3 -c "
import json
t=json.load(open('$O/h_stream.json')); print({k:v for k,v in t.items() if k.startswith(('upload','download'))})
s=json.load(open('$O/h_small.json')); print({k:(v.get('encode_chunk'),v.get('decode_chunk_lost0'),v.get('lib_call')) for k,v in s.items() if isinstance(v,dict)})"
