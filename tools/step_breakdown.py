"""Per-category breakdown of ONE train step from a rocprofv3 kernel trace.

usage: python tools/step_breakdown.py <run_kernel_trace.csv> [--top N]
A step is delimited by the last Adam launch of the previous step (4 Adam launches per step)."""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", n)
    return n.split("(")[0][:70]


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
    s, e = adam[-5] + 1, adam[-1] + 1
    step = rows[s:e]
    tot = 0.0
    cat = collections.Counter()
    launches = []
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        cat[short(r["Kernel_Name"])] += d
        launches.append((d, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], short(r["Kernel_Name"])))
    span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    print(f"one step: {len(step)} launches, kernel time {tot / 1e3:.2f} ms, wall span {span / 1e3:.2f} ms")
    print("\n| kernel | ms/step | % |\n|---|---|---|")
    for k, v in cat.most_common():
        print(f"| `{k}` | {v / 1e3:.3f} | {100 * v / tot:.1f} |")
    print(f"\ntop {top} launches (us, grid x*y*z work-items):")
    for d, x, y, z, n in sorted(launches, reverse=True)[:top]:
        print(f"{d:9.1f}  {x:>8}x{y:>5}x{z:>5}  {n}")


if __name__ == "__main__":
    main()
