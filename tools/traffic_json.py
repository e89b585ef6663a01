"""Summarise tools/gpu_traffic.sh output into a JSON file
(profiles/traffic_<arch>_<layer>_<mode>_b<B>.json, which bench.py reports as roofline.traffic).

usage: python tools/traffic_json.py <dir> <out.json> [layer c5] [mode fwd] [batch 512]

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB per dispatch.  On gfx950 FETCH_SIZE counts
half the bytes of 16-byte-per-lane streaming reads (global_load_dwordx4 and buffer_load ... lds
alike), so it is doubled; WRITE_SIZE is exact for 16-byte stores (MI355X_MICROARCH.md).
SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8) (when that pass exists) is the MFMA-busy fraction."""
import csv
import glob
import json
import sys

# neutron generator conv shapes (Cin, Hin, Win, Cout, Hout, Wout, k) -- generator.py:41-47
LAYERS = {"c0": (128, 13, 13, 256, 24, 24, 3), "c5": (256, 24, 24, 128, 46, 46, 3),
          "c9": (128, 46, 46, 64, 45, 45, 2)}
KERNEL = ("conv_ring_kernel", "wgrad_ring_kernel", "conv_igemm_kernel", "conv_persist_kernel", "conv_p256_kernel")


def _match(name):
    return any(k in name for k in KERNEL)


def per_dispatch(d, counter):
    vals = []
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if _match(r["Kernel_Name"]) and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def algorithmic_bytes(layer, mode, batch):
    """bf16 operands read once + result written once (weights / weight grads in their dtype)."""
    cin, hi, wi, cout, ho, wo, k = LAYERS[layer]
    x = batch * hi * wi * cin * 2
    y = batch * ho * wo * cout * 2
    w = cout * cin * k * k * 2
    if mode == "fwd":
        return x + y + w
    if mode == "dgrad":
        return y + x + w
    return x + y + cout * cin * k * k * 4     # wgrad: fp32 gradient out


def main():
    d, out = sys.argv[1], sys.argv[2]
    layer = sys.argv[3] if len(sys.argv) > 3 else "c5"
    mode = sys.argv[4] if len(sys.argv) > 4 else "fwd"
    batch = int(sys.argv[5]) if len(sys.argv) > 5 else 512
    fetch = per_dispatch(d + "/fetch", "FETCH_SIZE")
    write = per_dispatch(d + "/write", "WRITE_SIZE")
    mfma = per_dispatch(d + "/mfma", "SQ_VALU_MFMA_BUSY_CYCLES")
    gui = per_dispatch(d + "/mfma", "GRBM_GUI_ACTIVE")
    dur = []
    for f in glob.glob(d + "/kt/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if _match(r["Name"]):
                dur.append((r["Name"], float(r["AverageNs"]) / 1e3, int(r["Calls"])))
    fb = 2.0 * 1024 * sum(fetch) / len(fetch)
    wb = 1024.0 * sum(write) / len(write)
    res = {"kernel": dur[0][0] if dur else None, "avg_us": dur[0][1] if dur else None,
           "layer": layer, "mode": mode, "batch": batch,
           "dispatches": len(fetch), "fetch_bytes": round(fb), "write_bytes": round(wb),
           "traffic_bytes": round(fb + wb), "algorithmic_bytes": algorithmic_bytes(layer, mode, batch),
           "method": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     f"tools/mb_one.py {layer} {mode} (neutron generator, B={batch}); FETCH_SIZE x2 (gfx950)"}
    if mfma and gui:
        # SQ_VALU_MFMA_BUSY_CYCLES: MFMA-busy cycles summed over the chip's 1024 SIMDs;
        # GRBM_GUI_ACTIVE: busy clocks summed over the 8 XCDs (MI355X_MICROARCH.md) -> /8 = kernel clocks
        m, g = sum(mfma) / len(mfma), sum(gui) / len(gui)
        res["mfma_busy_cycles"] = m
        res["grbm_gui_active"] = g
        res["mfma_busy_frac"] = round(m / (1024.0 * g / 8.0), 4)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
