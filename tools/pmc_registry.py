"""File a tools/profile_workloads.sh run into the committed profile registry.

  python tools/pmc_registry.py TAG ROUND      e.g.  r04a r04

For every workload directory W of gpurun_out/prof_TAG/ (trace + DRAM-counter
passes of one `bench.py` command):
  * the bench line under trace gives the workload_key and the dominant kernel;
  * kernel_stats.csv gives the kernel's average duration per execute (the sum
    over its template instantiations: a C3 batch launches k_conj's single-list
    and general instantiations once each per execute);
  * the DRAM pass gives 32 B x (TCC_EA0_RDREQ_DRAM_32B + TCC_EA0_WRREQ_WRITE_DRAM_32B)
    per dispatch, averaged per instantiation and summed the same way -- HBM
    bytes per execute of the kernel (MI355X_MICROARCH.md: gfx950's size-aware
    request counters; calibrated on tools/calib_fetch's known streams and
    gathers, which must read 1.00 +- 3% on the streams).
Copies the evidence to profiles/ROUND/W/ and writes profiles/latest.json:
{"workloads": {workload_key: {hbm_bytes_per_launch, lib_id, source, ...}}},
which bench.py quotes as `roofline.traffic` for the same build.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lib_id import lib_id  # noqa: E402
from pmc_traffic import CALIB_KNOWN, read_counters  # noqa: E402

DRAM = ("TCC_EA0_RDREQ_DRAM_32B", "TCC_EA0_WRREQ_WRITE_DRAM_32B")


def family(name, kname):
    return name.startswith(f"void fg::(anonymous namespace)::{kname}<") or name.startswith(f"fg::{kname}") or \
        f"::{kname}<" in name or f"::{kname}(" in name


def trace_ms(path, kname):
    per = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if family(row["Name"], kname):
                per[row["Name"]] = (float(row["AverageNs"]) * 1e-6, int(row["Calls"]))
    return sum(v[0] for v in per.values()), per


def dram_bytes(d, kname):
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] in DRAM and family(row["Kernel_Name"], kname):
                    acc[row["Kernel_Name"]][row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    per = {}
    for name, disp in acc.items():
        vals = [32.0 * sum(c.values()) for c in disp.values()]
        per[name] = (sum(vals) / len(vals), len(vals))
    return sum(v[0] for v in per.values()), per


def calibration(prof):
    cd = read_counters(os.path.join(prof, "calib_dram"))
    out = {}
    for k, (kind, known) in CALIB_KNOWN.items():
        if k in cd:
            b = 32.0 * sum(cd[k].get("TCC_EA0_RDREQ_DRAM_32B", [])) / max(len(cd[k].get("TCC_EA0_RDREQ_DRAM_32B", [])), 1)
            out[k] = {"known": kind, "count": known, "dram_rd_bytes": b,
                      ("dram_rd_over_known" if kind == "bytes" else f"dram_rd_per_{kind[:-1]}"): round(b / known, 4)}
    ok = all(abs(out.get(s, {}).get("dram_rd_over_known", 0) - 1.0) <= 0.03 for s in ("stream4", "stream16"))
    return out, ok


def main():
    tag, rnd = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    calib, ok = calibration(prof)
    if not ok:
        raise SystemExit(f"DRAM counter calibration off: {json.dumps(calib)}")
    reg_path = os.path.join(ROOT, "profiles", "latest.json")
    reg = {"workloads": {}}
    if os.path.exists(reg_path):
        with open(reg_path) as f:
            old = json.load(f)
        reg["workloads"] = old.get("workloads", {})
    lid = lib_id()
    for w in sorted(os.listdir(prof)):
        d = os.path.join(prof, w)
        if not os.path.isfile(os.path.join(d, "trace_bench.json")):
            continue
        with open(os.path.join(d, "trace_bench.json")) as f:
            lines = [x for x in f.read().strip().splitlines() if x.startswith("{")]
        if not lines:
            print(f"{w}: no bench line, skipped")
            continue
        line = json.loads(lines[-1])
        roof = line["roofline"]
        kname, key = roof["kernel"], roof["workload_key"]
        t_ms, t_per = trace_ms(os.path.join(d, "kernel_stats.csv"), kname)
        b, b_per = dram_bytes(os.path.join(d, "dram"), kname)
        dst = os.path.join(ROOT, "profiles", rnd, w)
        os.makedirs(dst, exist_ok=True)
        shutil.copy(os.path.join(d, "kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
        shutil.copy(os.path.join(d, "trace_bench.json"), os.path.join(dst, "bench_under_trace.json"))
        for f in glob.glob(os.path.join(d, "dram", "**", "*counter_collection.csv"), recursive=True):
            shutil.copy(f, os.path.join(dst, "dram_counter_collection.csv"))
        with open(os.path.join(d, "bench_args.txt")) as f:
            args = f.read().strip()
        ent = {"workload_key": key, "kernel": kname, "lib_id": lid, "hbm_bytes_per_launch": b,
               "hbm_source": "32 B x (TCC_EA0_RDREQ_DRAM_32B + TCC_EA0_WRREQ_WRITE_DRAM_32B), per dispatch, "
                             "summed over the kernel's instantiations",
               "per_instantiation_bytes": {k: v[0] for k, v in b_per.items()},
               "dispatches": {k: v[1] for k, v in b_per.items()},
               "trace_avg_ms": t_ms, "trace_per_instantiation_ms": {k: v[0] for k, v in t_per.items()},
               "bench_kernel_ms_under_trace": roof["kernel_ms"],
               "command": f"bash tools/profile_workloads.sh {tag} {w}  (python3 bench.py --steps 5 --warmup 1 "
                          f"--no-cpu --p50-queries 0 --no-extra --no-model {args})",
               "source": os.path.relpath(os.path.join(dst, "pmc.json"), ROOT), "calibration": calib}
        with open(os.path.join(dst, "pmc.json"), "w") as f:
            json.dump(ent, f, indent=1)
        reg["workloads"][key] = ent
        print(f"{w}: {key} {kname} {b / 1e9:.3f} GB/launch, trace {t_ms:.4f} ms, bench {roof['kernel_ms']} ms")
    with open(reg_path, "w") as f:
        json.dump(reg, f, indent=1)


if __name__ == "__main__":
    main()
