"""Summarise tools/gpu_pmc_ab.sh output: per kernel (name filter), the counters per dispatch.
usage: python tools/pmc_ab_summary.py <dir> <name substrings...>"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    d, names = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(float))
    ndisp = defaultdict(set)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = next((n for n in names if n in r["Kernel_Name"]), None)
            if k is None:
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            ndisp[(k, r["Counter_Name"])].add((f, r.get("Dispatch_Id")))
    for k in names:
        c = acc[k]
        if not c:
            continue
        per = {n: v / max(1, len(ndisp[(k, n)])) for n, v in c.items()}
        g = per.get("GRBM_GUI_ACTIVE", 0)
        print(f"== {k}")
        for n in sorted(per):
            print(f"  {n:32s} {per[n]:.4g}")
        if g:
            print(f"  mfma busy (/(1024 SIMD x GRBM/8)): {per.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (1024 * g / 8):.3f}")
    for f in glob.glob(d + "/kt/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if any(n in r["Name"] for n in names):
                print(f"{float(r['AverageNs']) / 1e3:9.1f} us avg x {r['Calls']}  {r['Name'][:100]}")


if __name__ == "__main__":
    main()
