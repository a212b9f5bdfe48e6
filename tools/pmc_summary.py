"""Average PMC counters per kernel from a rocprofv3 --pmc CSV directory."""
import collections
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
f = next(d.glob("*counter_collection.csv"))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    name = k.split("(")[0].split("::")[-1] if "anonymous" in k else k[:40]
    agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, dd in agg.items():
    if "anonymous" not in n and not n.startswith("k_"):
        pass
    print(n, {c: round(sum(v) / len(v)) for c, v in dd.items()})
