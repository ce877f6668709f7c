#!/usr/bin/env python3
"""HBM traffic and SQ wave-state fractions of one syndrome-decode case from rocprofv3 --pmc
passes over tools/syn_ab.py (tools/gpu_pmc_syn.sh): for each variant, the first 3 dispatches of
its decode kernel are the case's reassembling calls and the next 3 its recover-only calls
(syn_ab's order with --rounds 1 --reps 2).  gfx950 correction as tools/pmc_summary.py: read =
2 x FETCH_SIZE KiB, written = WRITE_SIZE KiB.

    python tools/pmc_syn_summary.py gpurun_out > profiles/r03_pmc_syn.json
"""

from __future__ import annotations

import collections
import csv
import glob
import json
import sys

VARIANTS = {"fused": "sec_decode_bs_kernel<64", "direct": "sec_decode_kernel<8"}
K, B, NCH, E, N = 64, 16384, 1024, 16, 1 << 20


def load(d, counters=None):
    v = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if counters is None or r["Counter_Name"] in counters:
                i = int(r["Dispatch_Id"])
                v[i][r["Counter_Name"]] += float(r["Counter_Value"])
                name[i] = r["Kernel_Name"]
    return v, name


def main():
    o = sys.argv[1]
    alg = {"reassemble": NCH * (K * B + N), "recover_only": NCH * (K * B + E * B)}
    out = {"case": "zfec(64,96) 1024 x 1 MiB, 16 data blocks lost (0, 2, .., 30), parity rows 64..79 (one group)",
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ counters in separate passes over tools/syn_ab.py "
                     "(tools/gpu_pmc_syn.sh); read = 2 x FETCH_SIZE KiB (gfx950), write = WRITE_SIZE KiB; per "
                     "dispatch, the case's 3 reassembling then 3 recover-only calls",
           "algorithmic_bytes": alg}
    for var, pat in VARIANTS.items():
        f, nm = load(f"{o}/pmc_syn_{var}_FETCH_SIZE", {"FETCH_SIZE"})
        w, _ = load(f"{o}/pmc_syn_{var}_WRITE_SIZE", {"WRITE_SIZE"})
        ids = [i for i in sorted(f) if pat in nm[i]][:6]
        res = {"kernel": pat}
        for mode, sl in (("reassemble", ids[:3]), ("recover_only", ids[3:6])):
            rd = sum(2 * 1024 * f[i]["FETCH_SIZE"] for i in sl) / len(sl)
            wr = sum(1024 * w[i]["WRITE_SIZE"] for i in sl) / len(sl)
            res[mode] = {"read_bytes": round(rd), "write_bytes": round(wr),
                         "traffic_over_algorithmic": round((rd + wr) / alg[mode], 4)}
        q, qn = load(f"{o}/pmc_sq_{var}")
        qids = [i for i in sorted(q) if pat in qn[i]][:6]
        if qids:
            tot = {c: sum(q[i][c] for i in qids) / len(qids) for c in q[qids[0]]}
            wc = tot.get("SQ_WAVE_CYCLES") or 1
            res["sq_per_dispatch"] = {c: round(v) for c, v in sorted(tot.items())}
            res["sq_frac_of_wave_cycles"] = {c: round(tot[c] / wc, 3) for c in
                                             ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                              "SQ_ACTIVE_INST_VALU") if c in tot}
        out[var] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
