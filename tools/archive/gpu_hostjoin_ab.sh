#!/bin/bash
# Host-join reassembly A/B (api.cpp SEC_HOST_JOIN): bench.py's end-to-end legs (pageable locked
# per call, staged, pinned) with the host copying the present primaries (default) and with the
# GPU writing every output byte (SEC_HOST_JOIN=0), alternated twice; one JSON line per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
: > $O/hostjoin_ab.jsonl
for rep in 1 2; do
  for j in 1 0; do
    SEC_HOST_JOIN=$j timeout -k 10 300 python3 -u bench.py --no-cpu --steps 5 > $O/hj.log 2>&1 || { tail -20 $O/hj.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/hj.log').read().strip().splitlines()[-1]); print(json.dumps({'host_join': $j, **d['e2e']}))" >> $O/hostjoin_ab.jsonl
  done
done
cat $O/hostjoin_ab.jsonl
