#!/bin/bash
# Round 5, first GPU call: the headline-decode gap (tools/decode_gap.py, plain and under a kernel
# trace) and C5's decode by size class (tools/c5_classes.py, plain and with SQ counters).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== decode gap" && timeout -k 10 240 python3 -u tools/decode_gap.py --rounds 5 --reps 10 > $O/decode_gap.json 2> $O/decode_gap.err || { tail -20 $O/decode_gap.err; exit 1; }
cat $O/decode_gap.json
rm -rf $O/gap_trace
echo "== decode gap, kernel trace" && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gap_trace -o run -- python3 tools/decode_gap.py --rounds 3 --reps 10 > $O/gap_trace.log 2>&1 || { tail -20 $O/gap_trace.log; exit 1; }
echo "== c5 classes" && timeout -k 10 240 python3 -u tools/c5_classes.py run --reps 10 > $O/c5_classes.json 2> $O/c5_classes.err || { tail -20 $O/c5_classes.err; exit 1; }
cat $O/c5_classes.json
SQ="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
rm -rf $O/c5c_sq
echo "== c5 classes, SQ" && timeout -s KILL 150 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $O/c5c_sq -o run -- python3 tools/c5_classes.py run --reps 5 > $O/c5c_sq_plan.json 2> $O/c5c_sq.log || { tail -20 $O/c5c_sq.log; exit 1; }
python3 tools/c5_classes.py summarize $O/c5c_sq $O/c5c_sq_plan.json > $O/c5_classes_sq.json && cat $O/c5_classes_sq.json
