"""Per-dispatch PMC values of one kernel from a rocprofv3 counter_collection CSV.
usage: python tools/pmc_raw.py DIR KERNEL_SUBSTRING"""
import collections
import csv
import sys
from pathlib import Path

f = next(Path(sys.argv[1]).glob("*counter_collection.csv"))
rows = collections.OrderedDict()
for r in csv.DictReader(open(f)):
    if sys.argv[2] in r["Kernel_Name"]:
        rows.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
for d, c in list(rows.items())[:12]:
    print(d, " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))
