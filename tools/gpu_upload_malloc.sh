#!/bin/bash
# Host allocator: the library no longer calls mallopt.  Per-chunk upload
# timeline, stream rates and the C1 loopback, each with glibc's defaults and with the launch
# environment INTEGRATION.md documents for the validator (MALLOC_MMAP_THRESHOLD_ /
# MALLOC_TRIM_THRESHOLD_); one JSON line per run, the env in its "malloc_env" field.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
ENVS=("" "MALLOC_MMAP_THRESHOLD_=33554432 MALLOC_TRIM_THRESHOLD_=268435456")
: > $O/upload_malloc.jsonl
for E in "${ENVS[@]}"; do
  echo "== upload timeline [$E]" && env $E timeout -k 10 200 python3 -u tools/upload_timeline.py --mib 512 > $O/ut.json 2> $O/ut.err || { tail -20 $O/ut.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('$O/ut.json')); j['malloc_env']='$E'; j['tool']='upload_timeline'; print(json.dumps(j))" >> $O/upload_malloc.jsonl
  echo "== stream rate [$E]" && env $E timeout -k 10 300 python3 -u tools/stream_rate.py --mib 1024 > $O/sr.json 2> $O/sr.err || { tail -10 $O/sr.err; exit 1; }
  python3 -c "import json; j=json.load(open('$O/sr.json')); j['malloc_env']='$E'; j['tool']='stream_rate'; print(json.dumps(j))" >> $O/upload_malloc.jsonl
  echo "== c1 loopback [$E]" && env $E timeout -k 10 300 python3 -u tools/c1_loopback.py > $O/c1.json 2> $O/c1.err || { tail -10 $O/c1.err; exit 1; }
  python3 -c "import json; j=json.load(open('$O/c1.json')); j['malloc_env']='$E'; j['tool']='c1_loopback'; print(json.dumps(j))" >> $O/upload_malloc.jsonl
done
cat $O/upload_malloc.jsonl
