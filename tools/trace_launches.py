"""Median duration per (kernel, grid size) of a rocprofv3 kernel trace, for the kernels whose
name contains one of the given substrings.

python tools/trace_launches.py run_kernel_trace.csv [substring ...]
"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if pats and not any(p in n for p in pats):
            continue
        m = re.search(r"(k_[a-z_0-9]+(<[\w, ]+>)?)", n)
        key = (m.group(1) if m else n[:40], r["Grid_Size_X"])
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for (k, g), v in sorted(d.items()):
        print("%-34s grid %8s  n=%4d  median %8.2f us  mean %8.2f us" % (
            k, g, len(v), statistics.median(v), statistics.mean(v)))


if __name__ == "__main__":
    main()
