"""Summarise tools/gpu_traffic.sh output into a JSON file (profiles/<tag>_c5_fwd_traffic.json).

usage: python tools/traffic_json.py gpurun_out/traffic profiles/<tag>_c5_fwd_traffic.json

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB per dispatch.  On gfx950 FETCH_SIZE counts
half the bytes of 16-byte-per-lane streaming reads (global_load_dwordx4 and buffer_load ... lds
alike), so it is doubled; WRITE_SIZE is exact for 16-byte stores (MI355X_MICROARCH.md)."""
import csv
import glob
import json
import sys

KERNEL = "conv_ring_kernel"


def per_dispatch(d, counter):
    vals = []
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    d, out = sys.argv[1], sys.argv[2]
    fetch = per_dispatch(d + "/fetch", "FETCH_SIZE")
    write = per_dispatch(d + "/write", "WRITE_SIZE")
    dur = []
    for f in glob.glob(d + "/kt/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Name"]:
                dur.append((r["Name"], float(r["AverageNs"]) / 1e3, int(r["Calls"])))
    fb = 2.0 * 1024 * sum(fetch) / len(fetch)
    wb = 1024.0 * sum(write) / len(write)
    res = {"kernel": dur[0][0] if dur else KERNEL, "avg_us": dur[0][1] if dur else None,
           "dispatches": len(fetch), "fetch_bytes": round(fb), "write_bytes": round(wb),
           "traffic_bytes": round(fb + wb),
           "algorithmic_bytes": 512 * 24 * 24 * 256 * 2 + 512 * 46 * 46 * 128 * 2 + 128 * 256 * 16 * 2,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "tools/mb_one.py c5 fwd (neutron G conv_layers.5, B=512); FETCH_SIZE x2 (gfx950)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
