#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (separate passes).

Usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json

Counter values are KB per dispatch (profiles/gfx950_counters.txt).  On gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced read (MI355X_MICROARCH.md, HBM section), so it is doubled;
WRITE_SIZE is taken as is.  Infinity-Cache hits are counted by these counters (they sit on the
L2's fabric side), so "hbm" here means "left the XCD's L2".
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

# bench.py kernel classes -> predicate on the demangled kernel name
CLASSES = {
    "gemm": lambda n: "gemm_kernel<" in n or "gemm16_kernel<" in n or "gemm16f_kernel<" in n,
    "lstm_step_fwd": lambda n: "lstm_split_step_kernel<" in n or re.search(r"lstm_step_kernel<\d+, false", n) is not None,
    "lstm_step_bwd": lambda n: re.search(r"lstm_step_kernel<\d+, true", n) is not None,
    "lstm32": lambda n: "lstm32_" in n,
    # the persistent recurrences share one kernel template, told apart by NCH = H / 128: decoder
    # lstm2 (H = 1024) instantiates NCH = 8, decoder lstm1 (H = 512) NCH = 4
    "lstm2_persist": lambda n: "lstm_persist_kernel<8," in n,
    "lstm1_persist": lambda n: "lstm_persist_kernel<4," in n,
    "bptt_persist": lambda n: "bptt_persist_kernel<" in n or "bptt_xl_kernel" in n,
}


def collect(d, counter):
    per = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter:
                    per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch, write = collect(fdir, "FETCH_SIZE"), collect(wdir, "WRITE_SIZE")
    res = {"units": "bytes per dispatch; fetch = 2 x FETCH_SIZE(KB) x 1024 (gfx950 correction), "
                    "write = WRITE_SIZE(KB) x 1024", "classes": {}, "kernels": {}}
    for cls, pred in CLASSES.items():
        fs = [v for n, vs in fetch.items() if pred(n) for v in vs]
        ws = [v for n, vs in write.items() if pred(n) for v in vs]
        if not fs:
            continue
        fb = 2 * 1024 * sum(fs) / len(fs)
        wb = 1024 * sum(ws) / len(ws) if ws else 0.0
        res["classes"][cls] = {"dispatches": len(fs), "fetch_bytes": round(fb), "write_bytes": round(wb),
                               "traffic_bytes": round(fb + wb)}
    for n, vs in fetch.items():
        short = re.sub(r"\((?!anonymous).*$", "", n.replace("(anonymous namespace)", "anon"))[-90:]
        ws = write.get(n, [])
        res["kernels"][short] = {"dispatches": len(vs), "fetch_bytes": round(2 * 1024 * sum(vs) / len(vs)),
                                 "write_bytes": round(1024 * sum(ws) / len(ws)) if ws else None}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res["classes"], indent=1))


if __name__ == "__main__":
    main()
