"""Instruction mix of the loops of one kernel in a hipcc -S listing (diagnostic).

usage: python tools/isa_loops.py <file.s> <mangled kernel name substring> [min loop lines]"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    pat, minl = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 200
    names = [m.group(1) for m in re.finditer(r"^(\S+):\s*;\s*@\1", s, re.M) if pat in m.group(1)]
    for name in names:
        i = s.index(name + ":")
        body = s[i:s.index(".Lfunc_end", i)].split("\n")
        labels = {}
        for k, l in enumerate(body):
            m = re.match(r"^(\.LBB\S+):", l)
            if m:
                labels[m.group(1)] = k
        meta = re.findall(r"\.(vgpr_count|agpr_count|sgpr_count|vgpr_spill_count):\s*(\d+)", s[s.index(".name:           " + name) - 4000:s.index(".name:           " + name) + 200]) if (".name:           " + name) in s else []
        print(name, meta)
        for k, l in enumerate(body):
            m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)", l)
            if m and m.group(1) in labels and labels[m.group(1)] < k and k - labels[m.group(1)] >= minl:
                cnt = {}
                for x in body[labels[m.group(1)]:k + 1]:
                    t = x.strip().split()
                    if not t or t[0].startswith((".", ";")):
                        continue
                    op = t[0]
                    for key in ("mfma", "accvgpr", "ds_read", "ds_write", "buffer_load", "s_waitcnt", "s_nop", "v_cvt", "v_sub", "v_add"):
                        if key in op:
                            op = key
                            break
                    else:
                        op = "v_other" if op.startswith("v_") else ("s_other" if op.startswith("s_") else op)
                    cnt[op] = cnt.get(op, 0) + 1
                print("  loop", m.group(1), "lines", k - labels[m.group(1)], dict(sorted(cnt.items())))


if __name__ == "__main__":
    main()
