"""Average rocprofv3 PMC counters per kernel (library kernels by short name).

usage: python tools/pmc_summary.py DIR [DIR ...]   (each DIR holds a *counter_collection.csv)
FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB per dispatch.
"""
import collections
import csv
import json
import re
import sys
from pathlib import Path


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?)\(", name)
    return m.group(1) if m else None


def summarize(dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        f = next(Path(d).glob("*counter_collection.csv"))
        for r in csv.DictReader(open(f)):
            n = short(r["Kernel_Name"])
            if n:
                agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {n: {c: sum(v) / len(v) for c, v in dd.items()} for n, dd in agg.items()}


if __name__ == "__main__":
    print(json.dumps({k: {c: round(v, 1) for c, v in d.items()} for k, d in summarize(sys.argv[1:]).items()}, indent=1))
