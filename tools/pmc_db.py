"""Summarise a rocprofv3 --pmc run (rocpd database run_results.db, or the counter_collection.csv
of --output-format csv): per kernel (short name),
dispatch count, mean of each counter per dispatch, and the derived MFMA busy fraction
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs) when both were collected.

python tools/pmc_db.py gpurun_out/<dir>/run_results.db|run_counter_collection.csv [substr ...]
"""
import csv
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[a-z_0-9]+)", name)
    if not m:
        return name[:40]
    t = re.search(r"ILi(\d+)ELi(\d+)E(?:Li(\d+)ELi(\d+)E)?", name)
    return m.group(1) + ("<%s>" % ",".join(g for g in t.groups() if g) if t else "")


def summarise(path, filt=()):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    if path.endswith(".csv"):
        with open(path) as f:
            rows = [(r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]),
                     r["Dispatch_Id"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                    for r in csv.DictReader(f)]
    else:
        rows = sqlite3.connect(path).execute(
            "select kernel_name, counter_name, value, dispatch_id, duration "
            "from counters_collection")
    for name, counter, value, disp, d in rows:
        k = short(name)
        if filt and not any(s in k for s in filt):
            continue
        acc[k][counter].append(value)
        dur[k][disp] = d
    out = {}
    for k, cs in sorted(acc.items()):
        row = {c: sum(v) / len(v) for c, v in cs.items()}
        row["dispatches"] = len(dur[k])
        row["duration_us"] = sum(dur[k].values()) / max(1, len(dur[k])) / 1e3
        g, m = row.get("GRBM_GUI_ACTIVE"), row.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if g and m is not None:
            row["mfma_busy"] = m / (g / 8 * 1024)
        out[k] = row
    return out


def main():
    res = summarise(sys.argv[1], sys.argv[2:])
    for k, row in res.items():
        parts = " ".join("%s=%.4g" % (c, v) for c, v in sorted(row.items()))
        print("%-36s %s" % (k, parts))


if __name__ == "__main__":
    main()
