"""Summarise rocprofv3 PMC passes into HBM bytes per kernel launch.

    python tools/pmc_traffic.py FETCH_CSV WRITE_CSV STATS_CSV OUT_JSON [--alg NAME=BYTES ...]

FETCH_CSV / WRITE_CSV: the *_counter_collection.csv of two SEPARATE
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` runs (TCC slots cannot hold
both, MI355X_MICROARCH.md §rocprofv3 PMC slots).  Both counters are in KiB.
gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half
the bytes of a wide (16 B/lane) coalesced streaming read, so the read side is
doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.
STATS_CSV: the kernel_stats.csv of the un-instrumented --kernel-trace run, for
the average duration of the same kernels.
"""
from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(gf_\w+)(?:<([^>]*)>)?", name)
    if not m:
        return name[:80]
    if m.group(2) is None:
        return m.group(1)
    args = [a.strip() for a in m.group(2).split(",")]
    two = m.group(1) in ("gf_apply_kernel", "gf_apply_tri")  # <K, R, ...>
    return f"{m.group(1)}<{','.join(args[:2])}>" if two else f"{m.group(1)}<{args[0]}>"


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            vals[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


def main():
    fetch_csv, write_csv, stats_csv, out = sys.argv[1:5]
    alg = {}
    workload = "encdec"
    for a in sys.argv[5:]:
        if a.startswith("--workload="):
            workload = a.split("=", 1)[1]
            continue
        if a.startswith("--alg"):
            continue
        k, v = a.split("=")
        alg[k] = int(v)
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    dur = {}
    with open(stats_csv) as f:
        for row in csv.DictReader(f):
            dur[short(row["Name"])] = float(row["AverageNs"])
    res = {}
    for k in fetch:
        if not k.startswith("gf_"):
            continue
        fkib, n = fetch[k]
        wkib = write.get(k, (0.0, 0))[0]
        rd = 2.0 * fkib * 1024
        wr = wkib * 1024
        d = {"dispatches": n, "FETCH_SIZE_KiB": round(fkib, 1), "WRITE_SIZE_KiB": round(wkib, 1),
             "read_bytes_corrected": int(rd), "write_bytes": int(wr),
             "hbm_bytes_per_launch": int(rd + wr)}
        if k in dur:
            d["avg_duration_ns"] = dur[k]
            d["hbm_GBps"] = round((rd + wr) / dur[k], 1)
        if k in alg:
            d["algorithmic_bytes_per_launch"] = alg[k]
            d["traffic_over_algorithmic"] = round((rd + wr) / alg[k], 4)
        res[k] = d
    json.dump({"note": __doc__.strip().splitlines()[0], "workload": workload,
               "correction": "read = 2 x FETCH_SIZE KiB x 1024", "kernels": res}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
