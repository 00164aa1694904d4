"""Summarise one rocprofv3 --pmc pass of SQ / GRBM counters per kernel: where a
kernel's waves spend their cycles (issuing, parked on s_waitcnt, stalled at
issue), how busy the SIMDs' vector ALUs are, and the clock the chip held.

    python tools/pmc_sq.py COUNTER_CSV STATS_CSV OUT_JSON [--workload=NAME]

COUNTER_CSV: the *_counter_collection.csv of one pass with SQ_WAVES,
SQ_WAVE_CYCLES, SQ_ACTIVE_INST_ANY, SQ_ACTIVE_INST_VALU, SQ_WAIT_ANY,
SQ_WAIT_INST_ANY, SQ_INSTS_VALU, SQ_INSTS_SALU, GRBM_GUI_ACTIVE, GRBM_COUNT.
STATS_CSV: the kernel_stats.csv of an UN-instrumented --kernel-trace run of the
same command (the kernel's duration; a profiled pass runs at another clock,
MI355X_MICROARCH.md §DVFS give-back (2)); the pass's own dispatch times are
used when the CSV carries them.

Units (MI355X_MICROARCH.md §Per-instruction cycle constants, §PMC slots):
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over
waves; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES.
GRBM_GUI_ACTIVE is the sum over the 8 XCDs of the cycles the GPU was busy, so
the held clock ~= GRBM_GUI_ACTIVE / 8 / kernel time.
"""
from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import short  # noqa: E402

SIMDS = 256 * 4  # MI355X: 256 CUs x 4 SIMDs


def per_dispatch(path):
    """{kernel: [ {counter: value, '_ns': duration or None}, ... ]} per dispatch"""
    disp = defaultdict(dict)
    names = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            names[key] = short(row["Kernel_Name"])
            d = disp[key]
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            s, e = row.get("Start_Timestamp"), row.get("End_Timestamp")
            if s and e and "_ns" not in d:
                d["_ns"] = float(e) - float(s)
    out = defaultdict(list)
    for key, d in disp.items():
        out[names[key]].append(d)
    return out


def summarise(dispatches, stats_ns=None):
    n = len(dispatches)
    avg = {c: sum(d.get(c, 0.0) for d in dispatches) / n for c in dispatches[0] if c != "_ns"}
    pass_ns = [d["_ns"] for d in dispatches if d.get("_ns")]
    res = {"dispatches": n, "counters_avg": {c: round(v, 1) for c, v in sorted(avg.items())}}
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
            if c in avg:
                res[f"{c[3:].lower()}_over_wave_cycles"] = round(avg[c] / wc, 4)
    if avg.get("SQ_WAVES"):
        res["valu_insts_per_wave"] = round(avg.get("SQ_INSTS_VALU", 0.0) / avg["SQ_WAVES"], 1)
        res["salu_insts_per_wave"] = round(avg.get("SQ_INSTS_SALU", 0.0) / avg["SQ_WAVES"], 1)
    gui = avg.get("GRBM_GUI_ACTIVE")
    if gui:
        kcyc = gui / 8.0  # busy cycles of one XCD ~ the kernel's cycles at the held clock
        res["kernel_cycles_per_xcd"] = round(kcyc, 0)
        # SIMD-cycle shares: VALU-active cycles (quad-cycles x 4) over every
        # SIMD's cycles, and VALU instructions issued per SIMD per cycle
        if "SQ_ACTIVE_INST_VALU" in avg:
            res["valu_active_share_of_simd_cycles"] = round(4.0 * avg["SQ_ACTIVE_INST_VALU"] / (SIMDS * kcyc), 4)
        if "SQ_INSTS_VALU" in avg:
            res["valu_insts_per_simd_cycle"] = round(avg["SQ_INSTS_VALU"] / (SIMDS * kcyc), 4)
        if wc:
            res["resident_waves_per_simd_avg"] = round(4.0 * wc / (SIMDS * kcyc), 2)
        for src, ns in (("stats", stats_ns), ("pass", sum(pass_ns) / len(pass_ns) if pass_ns else None)):
            if ns:
                res[f"clock_GHz_{src}_duration"] = round(kcyc / ns, 3)
                res[f"duration_ns_{src}"] = round(ns, 0)
    return res


def main():
    ctr, stats, out = sys.argv[1:4]
    workload = "?"
    for a in sys.argv[4:]:
        if a.startswith("--workload="):
            workload = a.split("=", 1)[1]
    dur = {}
    if stats and stats != "-":
        with open(stats) as f:
            for row in csv.DictReader(f):
                dur[short(row["Name"])] = float(row["AverageNs"])
    res = {}
    for k, ds in per_dispatch(ctr).items():
        if not re.match(r"gf_", k):
            continue
        res[k] = summarise(ds, dur.get(k))
    json.dump({"note": __doc__.strip().splitlines()[0], "workload": workload, "kernels": res}, open(out, "w"),
              indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
