"""Summarise rocprofv3 --kernel-trace --stats output into markdown.

usage: python tools/prof_summary.py <run_kernel_stats.csv> <steps | marker kernel> [<run_kernel_trace.csv>]

<steps> is an integer, or the name (substring) of a kernel launched once per step (bench.py:
step_metrics_kernel), whose launch count in the stats is then the step count.

Table 1 is rocprofv3's own per-kernel-name statistics (kernel_stats.csv) divided per step.
Table 2 (needs the trace) splits each kernel name by launch grid, so that one layer's launches
can be told apart from other layers that share the kernel instantiation: bench.py's roofline
kernel (e.g. the generator conv_layers.5 weight gradient) is one (name, grid) row there, and its
average must agree with the bench's live HIP-event average.
"""
import collections
import csv
import re
import sys


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", n)
    return n.split("(")[0][:90]


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    arg = sys.argv[2] if len(sys.argv) > 2 else "1"
    if arg.isdigit():
        steps, how = int(arg), "given"
    else:
        steps = sum(int(r["Calls"]) for r in rows if arg in r["Name"])
        how = f"launches of {arg}"
        if steps == 0:
            sys.exit(f"no launches of {arg} in {path}")
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time {tot/1e6:.2f} ms over {steps} steps ({how}) = {tot/1e6/steps:.2f} ms/step\n")
    print("| kernel | calls/step | ms/step | avg us | % |")
    print("|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
        t = float(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {int(r['Calls'])/steps:.1f} | {t/1e6/steps:.3f} | "
              f"{float(r['AverageNs'])/1e3:.1f} | {100*t/tot:.1f} |")
    if len(sys.argv) > 3:
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(sys.argv[3])):
            grid = f"{r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
            agg[(short(r["Kernel_Name"]), grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        print("\nPer launch grid (work-items x*y*z), top 30 by total time:\n")
        print("| kernel | grid | launches | avg us | min us | max us | total ms |")
        print("|---|---|---|---|---|---|---|")
        for (k, g), d in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:30]:
            print(f"| `{k}` | {g} | {len(d)} | {sum(d)/len(d)/1e3:.1f} | {min(d)/1e3:.1f} | {max(d)/1e3:.1f} | "
                  f"{sum(d)/1e6:.3f} |")


if __name__ == "__main__":
    main()
