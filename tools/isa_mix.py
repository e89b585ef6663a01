"""Instruction mix between the first and last MFMA of one kernel in a hipcc -S listing, and the
distribution of non-MFMA vector instructions between consecutive MFMAs (diagnostic).

usage: python tools/isa_mix.py <file.s> <mangled kernel name>"""
import re
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
for blk in re.split(r"\n  - ", s[s.find("amdhsa.kernels"):]):
    n = re.search(r"\.name:\s+(\S+)", blk)
    if n and n.group(1) == name:
        print(re.findall(r"\.(agpr_count|vgpr_count|vgpr_spill_count|sgpr_spill_count|group_segment_fixed_size):\s*(\d+)", blk))
i = s.index(name + ":")
body = s[i:s.index(".Lfunc_end", i)].split("\n")
idx = [k for k, l in enumerate(body) if "v_mfma" in l]
seg = body[idx[0]:idx[-1] + 1]
ops = {}
runs, cur = [], 0
for l in seg:
    t = l.strip().split()
    if not t or t[0].startswith((".", ";")):
        continue
    ops[t[0]] = ops.get(t[0], 0) + 1
    if "mfma" in t[0]:
        runs.append(cur)
        cur = 0
    elif t[0].startswith("v_") or t[0].startswith("s_nop"):
        cur += 1
print(sorted(ops.items(), key=lambda x: -x[1])[:30])
print("VALU between MFMAs:", {k: runs.count(k) for k in sorted(set(runs))})
