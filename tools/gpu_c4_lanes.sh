#!/bin/bash
# C4 tile-shape A/B: 256-lane tiles (2 per 64 KiB chunk) against one tile
# per chunk (448 / 512 lanes) and 1024-lane tiles, plus decode copies stored early; one process.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 tools/sweep.py --workload c4 --us 1 --rounds 7 \
  --variants base,base@SEC_FULL_LANES=448,base@SEC_FULL_LANES=512,base@SEC_FULL_LANES=1024,decearly \
  > $O/c4_lanes.jsonl 2> $O/c4_lanes.err || { tail -30 $O/c4_lanes.err; exit 1; }
cat $O/c4_lanes.jsonl
