"""Summarise a rocprofv3 --pmc counter_collection.csv: per kernel (name prefix), the mean of each
counter per dispatch, and dispatch counts.

python tools/pmc_summary.py gpurun_out/pmc_micro/run_counter_collection.csv [name-substring ...]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[a-z_0-9]+)", name)
    if not m:
        return name[:40]
    t = re.search(r"ILi(\d+)ELi(\d+)E(?:Li(\d+)ELi(\d+)E)?", name)
    return m.group(1) + ("<%s>" % ",".join(g for g in t.groups() if g) if t else "")


def main():
    path = sys.argv[1]
    filt = sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if filt and not any(s in k for s in filt):
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        n = max(len(v) for v in cs.values())
        parts = ["%s=%.4g" % (c, sum(v) / len(v)) for c, v in sorted(cs.items())]
        print("%-36s n=%-4d %s" % (k, n, " ".join(parts)))


if __name__ == "__main__":
    main()
