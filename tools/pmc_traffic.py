"""Turn rocprofv3 --pmc CSV output into per-launch HBM bytes per kernel.

Usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR CALIB_DIR OUT_JSON
  FETCH_DIR / WRITE_DIR: rocprofv3 -d dirs of the bench run with --pmc FETCH_SIZE / WRITE_SIZE
  CALIB_DIR: rocprofv3 -d dir of tools/calib_fetch under --pmc FETCH_SIZE (known 1 GiB per launch)
FETCH_SIZE / WRITE_SIZE are in KiB (MI355X_MICROARCH.md §HBM).  The read side is
corrected by the measured calibration factor of 4-byte-per-lane streams (the
search kernels' load width); the raw and corrected values are both written.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def read_counters(d, counter):
    per = defaultdict(list)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                per[name].append(float(row["Counter_Value"]))
    return per


def short(name):
    for k in ("k_conj", "k_disj", "k_scan", "k_fmask", "k_final", "k_merge", "stream16", "stream4"):
        if k in name:
            return k
    return name[:40]


def main():
    fetch_dir, write_dir, calib_dir, out = sys.argv[1:5]
    calib = read_counters(calib_dir, "FETCH_SIZE")
    factor = {}
    for name, vals in calib.items():
        kb = sum(vals) / len(vals)
        factor[short(name)] = (1 << 30) / (kb * 1024.0)
    f4 = factor.get("stream4", 1.0)
    res = {"calibration": {k: round(v, 4) for k, v in factor.items()}, "kernels": {}}
    fetch = read_counters(fetch_dir, "FETCH_SIZE")
    write = read_counters(write_dir, "WRITE_SIZE")
    for name, vals in fetch.items():
        k = short(name)
        raw = sum(vals) / len(vals) * 1024.0
        w = write.get(name, [0.0])
        wb = sum(w) / len(w) * 1024.0
        res["kernels"][k] = {"fetch_bytes_raw": raw, "fetch_bytes_corrected": raw * f4, "write_bytes": wb,
                             "dispatches": len(vals)}
    kc = res["kernels"].get("k_conj")
    if kc:
        res["k_conj_hbm_bytes_per_launch"] = kc["fetch_bytes_corrected"] + kc["write_bytes"]
    # the library the counters were taken on: bench.py only quotes this traffic
    # for the same build (tools/lib_id.py)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from lib_id import lib_id
    res["lib_id"] = lib_id()
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
