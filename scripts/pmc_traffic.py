#!/usr/bin/env python3
"""Per-launch HBM traffic of pass 1 from rocprofv3 PMC passes (scripts/gpu_session.sh pmc).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  gfx950 correction (MI355X_MICROARCH.md,
HBM section): FETCH_SIZE counts wide coalesced 16-B/lane streaming reads at half their bytes
(128-B requests tallied as 64 B), so it is doubled; WRITE_SIZE is exact for such stores.
Writes profiles/<tag>/<file> and profiles/<file> (read by bench.py), where <file> is
pass1_traffic.json for config2 (kernel k_pass1s) and pass1_traffic_config3.json for config3
(the wide-map kernel k_pass1w).

usage: pmc_traffic.py <gpurun_out dir> <tag> [config2|config3]
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"config2": "k_pass1s", "config3": "k_pass1w"}
KERNEL = KERNELS["config2"]


def per_dispatch(pattern, counter):
    vals = []
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    global KERNEL
    out, tag = sys.argv[1], sys.argv[2]
    workload = sys.argv[3] if len(sys.argv) > 3 else "config2"
    KERNEL = KERNELS[workload]
    fname = "pass1_traffic.json" if workload == "config2" else f"pass1_traffic_{workload}.json"
    fetch = per_dispatch(os.path.join(out, "pmc1", "**", "*counter_collection.csv"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(out, "pmc2", "**", "*counter_collection.csv"), "WRITE_SIZE")
    if not fetch:
        sys.exit("no FETCH_SIZE rows for " + KERNEL)
    # Steady state: the bench cycles 2 pooled batches, and pass 1 stores chunk aggregates only
    # for still-virgin bits, so the first 2 dispatches (fresh virgin maps) write ~100 MB more.
    # Dispatches are in launch order in the CSV; the median of the later ones is reported.
    first_w = write[:2]
    fetch, write = (fetch[2:] or fetch), (write[2:] or write)
    f_kib = sorted(fetch)[len(fetch) // 2]
    w_kib = sorted(write)[len(write) // 2] if write else 0.0
    read_bytes = 2.0 * f_kib * 1024.0
    write_bytes = w_kib * 1024.0
    res = {"workload": workload, "kernel": KERNEL, "dispatches": len(fetch),
           "fetch_size_kib_raw_median": f_kib, "write_size_kib_median": w_kib,
           "hbm_read_bytes_per_launch": read_bytes, "hbm_write_bytes_per_launch": write_bytes,
           "hbm_bytes_per_launch": read_bytes + write_bytes,
           "first_two_dispatches_write_kib": first_w,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read tally), WRITE_SIZE as is"}
    os.makedirs(os.path.join(ROOT, "profiles", tag), exist_ok=True)
    for p in (os.path.join(ROOT, "profiles", tag, fname), os.path.join(ROOT, "profiles", fname)):
        json.dump(res, open(p, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
