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


def summarize(dirs, idle_frac=0.1):
    """Per kernel (short name) and counter, the average over its dispatches. Dispatches that
    ran shorter than idle_frac x the longest dispatch of the same kernel in the same pass are
    left out: launches that return at once (the depth cut's tail passes when no tile is
    flagged) share the kernel's name but not its work, and bench.py times the working launch."""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        f = next(Path(d).glob("*counter_collection.csv"))
        rows = [r for r in csv.DictReader(open(f)) if short(r["Kernel_Name"])]
        longest = collections.defaultdict(float)
        for r in rows:
            dur = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            longest[short(r["Kernel_Name"])] = max(longest[short(r["Kernel_Name"])], dur)
        for r in rows:
            n = short(r["Kernel_Name"])
            if float(r["End_Timestamp"]) - float(r["Start_Timestamp"]) < idle_frac * longest[n]:
                continue
            agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {n: {c: sum(v) / len(v) for c, v in dd.items()} for n, dd in agg.items()}


def traffic(summary):
    """Per-kernel HBM bytes per launch: FETCH_SIZE (KiB) x 2 (gfx950 reports half of a wide
    streaming read, MI355X_MICROARCH.md HBM section) + WRITE_SIZE (KiB); plus the SQ
    instruction / wave counters per launch when a pass collected them."""
    out = {}
    for k, d in summary.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            fb, wb = 2 * 1024 * d["FETCH_SIZE"], 1024 * d["WRITE_SIZE"]
            out[k] = {"fetch_bytes_corrected": int(fb), "write_bytes": int(wb), "hbm_bytes": int(fb + wb)}
            out[k].update({c: round(v, 1) for c, v in d.items() if c.startswith("SQ_")})
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "--json":  # --json OUT WORKLOAD SOURCE DIR...
        out, workload, source, dirs = args[1], args[2], args[3], args[4:]
        Path(out).write_text(json.dumps({"workload": workload, "source": source,
                                         "kernels": traffic(summarize(dirs))}, indent=1) + "\n")
    else:
        print(json.dumps({k: {c: round(v, 1) for c, v in d.items()} for k, d in summarize(args).items()}, indent=1))
