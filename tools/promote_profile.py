"""Copy a tools/profile_bench.sh result (gpurun_out/prof_<tag>) into the
committed profiles/<round>/ and point profiles/latest.json at it (the per-launch
k_conj HBM bytes bench.py quotes as roofline.traffic for the same build).

  python tools/promote_profile.py <tag> <round>          e.g.  r02a r02
  python tools/promote_profile.py <tag> <round> or       an OR profile (profile_bench.sh <tag> --disj --k 1000)
                                                         -> profiles/<round>/disj/ and profiles/latest_or.json
"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, rnd = sys.argv[1], sys.argv[2]
    is_or = len(sys.argv) > 3 and sys.argv[3] == "or"
    kname = "k_disj" if is_or else "k_conj"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", rnd, "disj") if is_or else os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    shutil.copy(os.path.join(src, "pmc.json"), os.path.join(dst, "pmc.json"))
    for sub in ("calib_fetch", "calib_dram"):
        for f in glob.glob(os.path.join(src, sub, "**", "*counter_collection.csv"), recursive=True):
            shutil.copy(f, os.path.join(dst, f"{sub}_counter_collection.csv"))
    shutil.copy(os.path.join(src, "trace_bench.json"), os.path.join(dst, "bench_under_trace.json"))
    with open(os.path.join(src, "pmc.json")) as f:
        pmc = json.load(f)
    with open(os.path.join(src, "trace_bench.json")) as f:
        bench = json.loads(f.read().strip().splitlines()[-1])
    cfg = bench["config"]
    kc = pmc["kernels"].get(kname, {})
    extra = " --disj --k 1000" if is_or else ""
    rel = os.path.relpath(dst, ROOT)
    latest = {
        "source": f"{rel}/pmc.json",
        "command": f"bash tools/profile_bench.sh {tag}{extra}  (= rocprofv3 --kernel-trace --stats, then separate --pmc "
                   "passes (FETCH_SIZE / WRITE_SIZE / TCC_EA0_RDREQ_DRAM_32B + TCC_EA0_WRREQ_WRITE_DRAM_32B) of python3 "
                   f"bench.py --steps 5 --warmup 1 --no-cpu --p50-queries 0 --no-extra{extra})",
        "workload": {"n_docs": cfg["n_docs"], "batch": cfg["batch"], "k": cfg["k"], "terms": cfg["terms"]},
        "lib_id": pmc.get("lib_id"),
        f"{kname}_hbm_bytes_per_launch": pmc.get(f"{kname}_hbm_bytes_per_launch"),
        "hbm_source": kc.get("hbm_source"),
        "calibration": pmc.get("calibration"),
    }
    out = os.path.join(ROOT, "profiles", "latest_or.json" if is_or else "latest.json")
    with open(out, "w") as f:
        json.dump(latest, f, indent=1)
    print(json.dumps(latest, indent=1))


if __name__ == "__main__":
    main()
