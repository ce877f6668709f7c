#!/bin/bash
# Per-chunk upload timeline: glibc's default heap trimming (STORB_AMD_MALLOC_TUNE=0) against the
# piece API's mallopt (the default), and the env form; then the stream rates and piece tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
: > $O/upload_malloc.jsonl
STORB_AMD_MALLOC_TUNE=0 timeout -k 10 200 python3 -u tools/upload_timeline.py --mib 512 >> $O/upload_malloc.jsonl 2> $O/upload_malloc.err || { tail -20 $O/upload_malloc.err; exit 1; }
timeout -k 10 200 python3 -u tools/upload_timeline.py --mib 512 >> $O/upload_malloc.jsonl 2> $O/upload_malloc.err || { tail -20 $O/upload_malloc.err; exit 1; }
STORB_AMD_MALLOC_TUNE=0 MALLOC_TRIM_THRESHOLD_=4294967296 MALLOC_MMAP_THRESHOLD_=134217728 timeout -k 10 200 python3 -u tools/upload_timeline.py --mib 512 >> $O/upload_malloc.jsonl 2> $O/upload_malloc.err || { tail -20 $O/upload_malloc.err; exit 1; }
cat $O/upload_malloc.jsonl
echo "== stream rate" && timeout -k 10 300 python3 -u tools/stream_rate.py --mib 1024 > $O/stream_rate.json 2> $O/stream_rate.err || { tail -10 $O/stream_rate.err; exit 1; }
cat $O/stream_rate.json
echo "== c1 loopback" && timeout -k 10 300 python3 -u tools/c1_loopback.py > $O/c1_loopback.json 2> $O/c1_loopback.err || { tail -10 $O/c1_loopback.err; exit 1; }
cat $O/c1_loopback.json
echo "== tests" && timeout -k 10 400 python3 -u -m pytest tests/test_piece_gpu.py tests/test_stream_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pt_host.log 2>&1 || { tail -40 $O/pt_host.log; exit 1; }
tail -1 $O/pt_host.log
