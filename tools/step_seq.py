"""One train step's kernel sequence from a rocprofv3 kernel trace (durations, gaps, grid sizes).
usage: python tools/step_seq.py <run_kernel_trace.csv> [step index] > out.txt"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
idx = [i for i, r in enumerate(rows) if "rand_exp_kernel" in r["Kernel_Name"]]
s, e = idx[k], idx[k + 1]
t0 = int(rows[s]["Start_Timestamp"])
prev_end, tot_gap, tot_k, small = t0, 0, 0, 0


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("_ZN12_GLOBAL__N_1", "")[:72]


for r in rows[s:e]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = st - prev_end
    tot_gap += max(gap, 0)
    tot_k += en - st
    small += (en - st) if en - st < 8000 else 0
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // int(r["Workgroup_Size_X"])
    print(f"{(st - t0) / 1e3:9.1f} gap {gap / 1e3:6.1f} dur {(en - st) / 1e3:7.1f}  wg {g:6d}  {short(r['Kernel_Name'])}")
    prev_end = max(prev_end, en)
print(f"kernels {e - s} ktime {tot_k / 1e6:.3f} ms gaps {tot_gap / 1e6:.3f} ms small(<8us) {small / 1e6:.3f} ms "
      f"span {(int(rows[e]['Start_Timestamp']) - t0) / 1e6:.3f} ms")
