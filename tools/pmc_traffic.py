"""Turn rocprofv3 --pmc CSV output into per-launch HBM bytes per kernel.

Usage: python tools/pmc_traffic.py PROF_DIR OUT_JSON
  PROF_DIR holds the rocprofv3 -d directories of tools/profile_bench.sh:
    calib_fetch, calib_dram   tools/calib_fetch under --pmc FETCH_SIZE / the DRAM counters
    fetch, write, dram        the bench command under --pmc FETCH_SIZE / WRITE_SIZE / the DRAM counters
The DRAM counters are gfx950's size-aware TCC_EA0_RDREQ_DRAM_32B and
TCC_EA0_WRREQ_WRITE_DRAM_32B (32-B units: a 64-B request counts 2, a 128-B one
4), so their bytes do not depend on the request width.  FETCH_SIZE (KiB) tallies
128-B requests at 64 B on gfx950 (MI355X_MICROARCH.md §HBM): exactly 1/2 of a
wide stream, but a different fraction for scattered single-dword gathers.  Both
are calibrated here on known byte counts (tools/calib_fetch.hip: coalesced
streams and one dword per 128-B line), and the per-launch HBM bytes are taken
from the DRAM counters when their stream calibration reads 1.00 +- 3%.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

GIB = 1 << 30
CALIB_KNOWN = {  # known bytes (streams) / lines touched (gather_lines) per launch
    "stream4": ("bytes", GIB),
    "stream16": ("bytes", GIB),
    "gather_lines": ("lines", (4 * GIB) // 128),
    "gather_random": ("loads", 1 << 25),
}


def short(name):
    for k in ("k_conj", "k_disj", "k_scan", "k_fmask", "k_final", "k_merge", "k_dense", "stream16", "stream4",
              "gather_lines", "gather_random"):
        if k in name:
            return k
    return name[:40]


def read_counters(d):
    """{kernel: {counter: [per-dispatch value]}} (rows of one dispatch summed)."""
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                per[short(row.get("Kernel_Name", ""))][row["Counter_Name"]][row["Dispatch_Id"]] += float(
                    row["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in per.items()}


def mean(v):
    return sum(v) / len(v) if v else 0.0


def main():
    prof, out = sys.argv[1:3]
    cf = read_counters(os.path.join(prof, "calib_fetch"))
    cd = read_counters(os.path.join(prof, "calib_dram"))
    calib = {}
    for k, (kind, known) in CALIB_KNOWN.items():
        e = {"known": kind, "count": known}
        if k in cf:
            e["fetch_size_bytes"] = mean(cf[k].get("FETCH_SIZE", [])) * 1024.0
        if k in cd:
            e["dram_rd_bytes"] = 32.0 * mean(cd[k].get("TCC_EA0_RDREQ_DRAM_32B", []))
        if kind == "bytes":
            for key in ("fetch_size_bytes", "dram_rd_bytes"):
                if e.get(key):
                    e[key.replace("_bytes", "") + "_over_known"] = round(e[key] / known, 4)
        else:
            for key in ("fetch_size_bytes", "dram_rd_bytes"):
                if e.get(key):
                    e[key.replace("_bytes", "") + "_per_" + kind[:-1]] = round(e[key] / known, 2)
        calib[k] = e
    dram_ok = all(abs(calib[s].get("dram_rd_over_known", 0) - 1.0) <= 0.03 for s in ("stream4", "stream16"))
    fetch_factor = 1.0 / calib["stream4"]["fetch_size_over_known"] if calib["stream4"].get("fetch_size_over_known") else None

    fetch = read_counters(os.path.join(prof, "fetch"))
    write = read_counters(os.path.join(prof, "write"))
    dram = read_counters(os.path.join(prof, "dram"))
    kernels = {}
    for k in set(fetch) | set(dram):
        e = {}
        if k in fetch:
            e["fetch_size_bytes"] = mean(fetch[k].get("FETCH_SIZE", [])) * 1024.0
            e["dispatches"] = len(fetch[k].get("FETCH_SIZE", []))
        if k in write:
            e["write_size_bytes"] = mean(write[k].get("WRITE_SIZE", [])) * 1024.0
        if k in dram:
            e["dram_rd_bytes"] = 32.0 * mean(dram[k].get("TCC_EA0_RDREQ_DRAM_32B", []))
            e["dram_wr_bytes"] = 32.0 * mean(dram[k].get("TCC_EA0_WRREQ_WRITE_DRAM_32B", []))
        if dram_ok and "dram_rd_bytes" in e:
            e["hbm_bytes_per_launch"] = e["dram_rd_bytes"] + e["dram_wr_bytes"]
            e["hbm_source"] = "32 B x (TCC_EA0_RDREQ_DRAM_32B + TCC_EA0_WRREQ_WRITE_DRAM_32B)"
        elif fetch_factor and "fetch_size_bytes" in e:
            e["hbm_bytes_per_launch"] = e["fetch_size_bytes"] * fetch_factor + e.get("write_size_bytes", 0.0)
            e["hbm_source"] = f"FETCH_SIZE x {fetch_factor:.3f} (stream calibration) + WRITE_SIZE"
        kernels[k] = e
    res = {"calibration": calib, "dram_counter_calibrated": dram_ok, "kernels": kernels}
    for k in ("k_conj", "k_disj"):
        if k in kernels and "hbm_bytes_per_launch" in kernels[k]:
            res[f"{k}_hbm_bytes_per_launch"] = kernels[k]["hbm_bytes_per_launch"]
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from lib_id import lib_id
    res["lib_id"] = lib_id()
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
