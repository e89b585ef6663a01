"""Summarise a rocprofv3 rocpd database: per-kernel totals, summed vs wall (interval union) time.

usage: python tools/prof_summary.py RESULTS.db [top]"""
import sqlite3
import sys


def main(path, top=25):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    tot = {}
    for n, s, e in rows:
        k = tot.setdefault(n, [0, 0.0])
        k[0] += 1
        k[1] += (e - s) / 1e3
    busy, cur_s, cur_e = 0.0, None, None
    for _, s, e in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = (rows[-1][2] - rows[0][1]) / 1e3 if rows else 0.0
    summed = sum(v[1] for v in tot.values())
    print(f"kernels {len(rows)}  summed {summed / 1e3:.1f} ms  busy(union) {busy / 1e6:.1f} ms  span {span / 1e3:.1f} ms")
    for n, (cnt, us) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{us / 1e3:9.2f} ms {cnt:6d} x {us / cnt:8.1f} us  {n[:150]}")
    # one template instance can serve several layers (e.g. conv_layers.0 and .5 FWD): the top kernels
    # split by launch grid
    cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
    grid = [k for k in cols if k.startswith("grid_size")] or [k for k in cols if "grid" in k]
    if grid:
        print("\nby launch grid (" + ", ".join(grid) + "):")
        for n, _ in sorted(tot.items(), key=lambda kv: -kv[1][1])[:min(top, 12)]:
            q = f"select {', '.join(grid)}, count(*), sum(end - start) from kernels where name = ? group by {', '.join(grid)}"
            for row in c.execute(q, (n,)).fetchall():
                g, cnt, ns = row[:-2], row[-2], row[-1]
                print(f"{ns / 1e6:9.2f} ms {cnt:6d} x {ns / 1e3 / cnt:8.1f} us  grid {tuple(g)}  {n[:110]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
