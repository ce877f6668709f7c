#!/bin/bash
# Round 6: sector-whole decode stores for k <= 8 chunks with B >= 128 KiB
# and unaligned rows (this build) against none (build/variants/libstorbec_nosect.so): the decode
# GPU tests, then the C5 / C4 / headline bench lines of both libraries, alternating, twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode_ex.py tests/test_gpu_bench_c5.py tests/test_gpu_bench_c4.py tests/test_gpu_pieces.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_sect.log 2>&1 || { tail -40 $O/pytest_sect.log; exit 1; }
tail -1 $O/pytest_sect.log
V=$R/build/variants/libstorbec_nosect.so
for i in 1 2; do
  for L in sect base; do
    if [ $L = base ]; then export STORB_EC_LIB=$V; else unset STORB_EC_LIB; fi
    for W in c5 c4 c2c3; do
      X=""; [ $W = c2c3 ] && X="--no-c4 --no-c5"
      timeout -k 10 300 python3 -u bench.py --workload $W --steps 30 --warmup 5 --no-cpu --no-e2e $X > $O/sect_${L}_${i}_$W.log 2>&1 || { tail -20 $O/sect_${L}_${i}_$W.log; exit 1; }
    done
  done
done
unset STORB_EC_LIB
python3 - <<PY
import json
def line(f):
    return [json.loads(l) for l in open(f) if l.startswith("{")][-1]
for i in (1, 2):
    for L in ("sect", "base"):
        c5 = line(f"$O/sect_{L}_{i}_c5.log"); c4 = line(f"$O/sect_{L}_{i}_c4.log"); c2 = line(f"$O/sect_{L}_{i}_c2c3.log")
        print(L, i, "c5 dev enc/dec ms", c5["device_resident"]["encode_ms"], c5["device_resident"]["decode_ms"], "c5", c5["value"],
              "| c4 enc/dec ms", c4["roofline"]["avg_launch_ms"], c4["decode_kernel"]["avg_launch_ms"],
              "| c3 dec ms", c2["roofline"]["avg_launch_ms"], "c2 enc", c2["encode_kernel"]["avg_launch_ms"])
PY
