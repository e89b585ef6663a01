"""Per-kernel HBM traffic and MFMA-busy of a whole train step (tools/gpu_pmc_step.sh output).

usage: python tools/pmc_step.py <dir> <steps> > summary.md

<dir>/kt: kernel-trace pass; <dir>/fetch, <dir>/write, <dir>/mfma: one rocprofv3 --pmc pass each
(FETCH_SIZE; WRITE_SIZE; SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE), all csv.  Per kernel name: launches
per step, average duration, FETCH_SIZE x 2 (gfx950 counts half the bytes of 16-byte-per-lane reads,
MI355X_MICROARCH.md; other widths uncalibrated) and WRITE_SIZE per launch, the implied GB/s, and the MFMA-busy
fraction (busy cycles over the 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs)).  Per step: summed kernel time,
bytes and MFMA-busy cycles.  <steps>: the number of train steps the profiled command ran (warm-up and
capture included), to normalise the per-step columns."""
import csv
import glob
import sys
from collections import defaultdict


def rows(d, pat):
    for f in glob.glob(f"{d}/**/{pat}", recursive=True):
        yield from csv.DictReader(open(f))


def counters(d, name):
    out = defaultdict(list)
    for r in rows(d, "*counter_collection.csv"):
        if r["Counter_Name"] == name:
            out[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return out


def main(d, steps):
    dur = defaultdict(list)
    for r in rows(d + "/kt", "*kernel_trace.csv"):
        dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    fetch, write = counters(d + "/fetch", "FETCH_SIZE"), counters(d + "/write", "WRITE_SIZE")
    mfma, gui = counters(d + "/mfma", "SQ_VALU_MFMA_BUSY_CYCLES"), counters(d + "/mfma", "GRBM_GUI_ACTIVE")
    avg = lambda v: sum(v) / len(v) if v else float("nan")
    tab = []
    for k, v in dur.items():
        fb = 2 * 1024 * avg(fetch.get(k, []))
        wb = 1024 * avg(write.get(k, []))
        m, g = avg(mfma.get(k, [])), avg(gui.get(k, []))
        busy = m / (1024.0 * g / 8.0) if g == g and g > 0 else float("nan")
        tab.append((sum(v) / steps, len(v) / steps, avg(v), fb, wb, busy, m * len(v) / steps, k))
    tab.sort(reverse=True)
    tot_t = sum(t[0] for t in tab)
    tot_b = sum((t[3] + t[4]) * t[1] for t in tab if t[3] == t[3] and t[4] == t[4])
    tot_m = sum(t[6] for t in tab if t[6] == t[6])
    print(f"# Train-step PMC summary ({steps} steps)\n")
    print(f"kernel time per step {tot_t / 1e3:.3f} ms; HBM bytes per step (FETCHx2 + WRITE) {tot_b / 1e9:.3f} GB "
          f"= {tot_b / tot_t / 1e6:.2f} TB/s over the kernel time; MFMA-busy cycles per step {tot_m:.3e} "
          f"(= {tot_m / 1024 / (tot_t * 1e-6) / 1e9:.3f} GHz-equivalent busy per SIMD)\n")
    print("| us/step | launches/step | avg us | FETCHx2 MB | WRITE MB | GB/s | MFMA busy | kernel |")
    print("|---|---|---|---|---|---|---|---|")
    for t_, n, a, fb, wb, busy, _, k in tab:
        gbs = (fb + wb) / (a * 1e3) if a > 0 else float("nan")
        print(f"| {t_:.1f} | {n:.2f} | {a:.1f} | {fb / 1e6:.1f} | {wb / 1e6:.1f} | {gbs:.0f} | {busy:.3f} | "
              f"`{k[:110]}` |")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]))
