"""Summarise a rocprofv3 kernel_stats.csv (+ per-step division) into a markdown table."""
import csv
import re
import sys


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = n.replace("_ZN12_GLOBAL__N_117conv_igemm_kernelI", "conv_igemm<")
    return n[:100]


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time {tot/1e6:.2f} ms over {steps} steps = {tot/1e6/steps:.2f} ms/step\n")
    print("| kernel | calls/step | ms/step | avg us | % |")
    print("|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
        t = float(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {int(r['Calls'])/steps:.1f} | {t/1e6/steps:.3f} | "
              f"{float(r['AverageNs'])/1e3:.1f} | {100*t/tot:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
