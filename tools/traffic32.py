"""Per-OP HBM traffic / MFMA-busy of one neutron generator conv in the fp32 parity mode, from the
rocprofv3 passes of tools/gpu_traffic32.sh (an op may be several dispatches: image chunks of the
1 GiB ring limit, plus the deterministic WGRAD's ordered reduce).

usage: python tools/traffic32.py <dir> <out.json> <layer> <mode> <batch> <ops> [split 0|1]
FETCH_SIZE (KiB, x2 on gfx950 for 16-byte-per-lane streaming reads) + WRITE_SIZE (KiB) summed over
the op's dispatches / ops (MI355X_MICROARCH.md HBM / rocprofv3 section); MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) over the op's conv dispatches."""
import csv
import glob
import json
import sys

LAYERS = {"c0": (128, 13, 13, 256, 24, 24, 3), "c5": (256, 24, 24, 128, 46, 46, 3),
          "c9": (128, 46, 46, 64, 45, 45, 2),
          "p1": (512, 18, 10, 256, 35, 19, 4), "p5": (256, 35, 19, 128, 55, 29, 4)}
NAMES = {"fwd": ("conv_ring_kernel<0", "upsample_fwd_nhwc"), "dgrad": ("conv_ring_kernel<1", "upsample_bwd_nhwc"),
         "wgrad": ("wgrad_f32_kernel", "wgrad_f32_col_kernel", "wgrad_f32_col2_kernel", "wgrad_coop_kernel", "wgrad_ws_kernel",
                   "wgrad_reduce_kernel")}


def rows(d, counter, names):
    out = []
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and any(n in r["Kernel_Name"] for n in names):
                out.append((r["Kernel_Name"], float(r["Counter_Value"])))
    return out


def main():
    d, out, layer, mode, batch, ops = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]), int(sys.argv[6])
    split = len(sys.argv) > 7 and sys.argv[7] == "1"
    names = NAMES[mode]
    fetch = rows(d + "/fetch", "FETCH_SIZE", names)
    write = rows(d + "/write", "WRITE_SIZE", names)
    conv = tuple(n for n in names if "reduce" not in n and "upsample" not in n)
    mfma = rows(d + "/mfma", "SQ_VALU_MFMA_BUSY_CYCLES", conv)
    gui = rows(d + "/mfma", "GRBM_GUI_ACTIVE", conv)
    dur = {}
    for f in glob.glob(d + "/kt/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if any(n in r["Name"] for n in names):
                dur[r["Name"]] = float(r["TotalDurationNs"]) / 1e3 / ops
    cin, hi, wi, cout, ho, wo, k = LAYERS[layer]
    alg = 4 * batch * (hi * wi * cin + ho * wo * cout) + 4 * cout * cin * k * k
    fb = 2.0 * 1024 * sum(v for _, v in fetch) / ops
    wb = 1024.0 * sum(v for _, v in write) / ops
    res = {"layer": layer, "mode": mode, "batch": batch, "dtype": "fp32", "ops": ops,
           "fp32_mfma": "split" if split else "exact",
           "dispatches_per_op": len(fetch) / ops, "us_per_op": round(sum(dur.values()), 1), "kernels": dur,
           "fetch_bytes": round(fb), "write_bytes": round(wb), "traffic_bytes": round(fb + wb),
           "algorithmic_bytes": alg,
           "method": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_VALU_MFMA_BUSY_CYCLES+GRBM_GUI_ACTIVE in "
                     f"separate passes over ES_MB_DTYPE=fp32{' ES_MB_SPLIT=1' if split else ''} tools/mb_one.py "
                     f"{layer} {mode} (B={batch}); "
                     f"FETCH_SIZE x2 (gfx950); per op = sum over its dispatches / {ops} ops"}
    if mfma and gui:
        m = sum(v for _, v in mfma)
        g = sum(v for _, v in gui)
        res["mfma_busy_frac"] = round(m / (1024.0 * g / 8.0), 4)
        if split:
            res["mfma_note"] = "split-fp32: busy cycles of the bf16 MFMA pipe (6 plane products per fp32 product)"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
