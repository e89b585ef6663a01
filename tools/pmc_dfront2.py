"""Summarise tools/gpu_pmc_dfront2.sh: per kernel (dfront2_fwd / bwd variants / part_reduce) average
duration, HBM bytes per launch (FETCH_SIZE x2 for 16-byte loads per MI355X_MICROARCH.md, WRITE_SIZE),
MFMA-busy and VALU-active fractions.  usage: python tools/pmc_dfront2.py <dir> <out.json>"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def kname(full):
    m = re.search(r"dfront2_\w+(<[^>]*>)?", full)
    return m.group(0) if m else full


def rows(d, counter):
    out = defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and "dfront2" in r["Kernel_Name"]:
                out[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return out


def main():
    d, out = sys.argv[1], sys.argv[2]
    dur = {}
    for f in glob.glob(d + "/kt/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "dfront2" in r["Name"]:
                dur[kname(r["Name"])] = float(r["AverageNs"]) / 1e3
    fetch, write = rows(d + "/fetch", "FETCH_SIZE"), rows(d + "/write", "WRITE_SIZE")
    mfma, valu, gui = (rows(d + "/busy", c) for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"))
    res = {}
    for k in sorted(set(fetch) | set(dur)):
        n = max(len(fetch.get(k, [])), 1)
        e = {"avg_us": round(dur.get(k, 0.0), 1),
             "fetch_bytes": round(2 * 1024 * sum(fetch.get(k, [0])) / n),
             "write_bytes": round(1024 * sum(write.get(k, [0])) / max(len(write.get(k, [])), 1))}
        g = sum(gui.get(k, [0]))
        if g:
            e["mfma_busy_frac"] = round(sum(mfma.get(k, [0])) / (1024.0 * g / 8.0), 4)
            e["valu_active_frac"] = round(4 * sum(valu.get(k, [0])) / (1024.0 * g / 8.0) / 16, 4)
        res[k] = e
    res["method"] = ("rocprofv3 separate passes over tools/mb_dfront2.py 1024 (N = 1024 images, 44 x 44): FETCH_SIZE x2 "
                     "(gfx950), WRITE_SIZE, SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8); "
                     "valu_active_frac approximate (SQ_ACTIVE_INST_VALU quad-cycles)")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
