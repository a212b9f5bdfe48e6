"""profiles/pmc_costvol.json from tools/prof_cv.sh output dirs (one per bench shape).

usage: python tools/cv_pmc_json.py OUT SOURCE TAG=DIR [TAG=DIR ...]
Per shape, the forward's matrix-core kernel (k_cost_band on small grids, else k_cost_epi): busy_frac = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) (median over its dispatches), LDS bank conflicts per
LDS instruction, and the HBM bytes of the channel-last copies (k_to_hwc)."""
import csv
import json
import re
import statistics
import sys
from pathlib import Path


def rows(d):
    f = next(Path(d).glob("*counter_collection.csv"))
    out = {}
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+(?:<[^>]*>)?)\(", r["Kernel_Name"])
        if m:
            out.setdefault((r["Dispatch_Id"], m.group(1)), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    return out


def main():
    out_path, source, specs = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = {}
    for spec in specs:
        tag, d = spec.split("=", 1)
        sq, gr = rows(Path(d) / "pmc_sq"), rows(Path(d) / "pmc_grbm")
        ks = sorted({k for _, k in sq if k.startswith("k_cost_band")}) or \
            sorted({k for _, k in sq if k.startswith("k_cost_epi") and not k.startswith("k_cost_epi_bwd")})
        if not ks:
            continue
        k = ks[0]
        busy = [v["SQ_VALU_MFMA_BUSY_CYCLES"] for (_, kk), v in sq.items() if kk == k]
        gui = [v["GRBM_GUI_ACTIVE"] for (_, kk), v in gr.items() if kk == k]
        lds = [v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_INSTS_LDS"], 1.0) for (_, kk), v in sq.items() if kk == k]
        b, g = statistics.median(busy), statistics.median(gui)
        res[tag] = {"kernel": k, "busy_frac": round(b / (g / 8 * 1024), 4), "SQ_VALU_MFMA_BUSY_CYCLES": b,
                    "GRBM_GUI_ACTIVE": g, "lds_conflict_per_lds_instr": round(statistics.median(lds), 3),
                    "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), median dispatch",
                    "source": source}
    Path(out_path).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
