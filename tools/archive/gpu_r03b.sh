#!/bin/bash
# Round-3 evidence, second batch: the whole -m gpu suite, the C4 line at several parity
# alignments, C4's PMC traffic, the upload / download streams and the C1 loopback.  Each step
# under its own timeout; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== pytest gpu" && timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
: > $O/c4_palign.jsonl
for A in 128 256 1 512 128 256; do
  timeout -k 10 120 python3 -u bench.py --workload c4 --no-cpu --steps 30 --warmup 3 --c4-palign $A >> $O/c4_palign.jsonl 2> $O/c4_palign.err || { tail -20 $O/c4_palign.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/c4_palign.jsonl'):
    j = json.loads(l); print(j['config']['parity_stride'], j['value'], j['roofline']['frac'])"
echo "== pmc c4" && bash tools/gpu_pmc.sh c4 > $O/pmc_c4.log 2>&1 || { tail -30 $O/pmc_c4.log; exit 1; }
tail -20 $O/pmc_c4.log
echo "== stream rate" && timeout -k 10 400 python3 -u tools/stream_rate.py --mib 1024 > $O/stream_rate.json 2> $O/stream_rate.err || { tail -20 $O/stream_rate.err; exit 1; }
cat $O/stream_rate.json
echo "== c1 loopback" && timeout -k 10 400 python3 -u tools/c1_loopback.py > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
cat $O/c1.json
