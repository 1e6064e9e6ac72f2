"""Where the slow GET /search calls during commits wait: the db_api bench's
reader searches (start, latency on the steady clock) lined up with the native
commit / build / free phases (FUGU_COMMIT_TRACE, FUGU_BUILD_TRACE: each phase
line ends with its end time "@<ms>").

  python tools/stall_trace.py run [--docs N] [--out DIR]     # bench + traces into DIR
  python tools/stall_trace.py analyze DIR [--slow MS]         # the report (JSON)

For every phase name: how much of the commits' wall time it covers, and how
often it overlaps a slow search (latency >= --slow ms, default the p99) --
a phase that overlaps most slow searches while covering little of the time is
what they wait behind.
"""
import argparse
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINE = re.compile(r"\[fg (\w[\w ]*)\]\s+(.+?)\s+([\d.]+) ms @([\d.]+)")


def run(args):
    os.makedirs(args.out, exist_ok=True)
    env = dict(os.environ, FUGU_COMMIT_TRACE="1", FUGU_BUILD_TRACE="1",
               FUGU_STALL_TRACE=os.path.join(args.out, "searches.json"))
    with open(os.path.join(args.out, "bench.json"), "w") as fo, open(os.path.join(args.out, "trace.err"), "w") as fe:
        rc = subprocess.call([sys.executable, "-u", os.path.join(ROOT, "tools", "db_api_bench.py"), "--docs",
                              str(args.docs), "--no-ref"], stdout=fo, stderr=fe, env=env)
    if rc:
        sys.exit(rc)
    analyze(argparse.Namespace(dir=args.out, slow=None))


def analyze(args):
    import numpy as np
    searches = json.load(open(os.path.join(args.dir, "searches.json")))
    spans = []
    for line in open(os.path.join(args.dir, "trace.err")):
        m = LINE.search(line)
        if m:
            tag, phase, ms, end = m.group(1), m.group(2).strip(), float(m.group(3)), float(m.group(4))
            spans.append((f"{tag}: {phase}", end - ms, end))
    if not searches or not spans:
        sys.exit("no searches or no traced phases")
    lat = np.array([s[1] for s in searches])
    cut = args.slow if args.slow is not None else float(np.percentile(lat, 99))
    t_lo, t_hi = searches[0][0], searches[-1][0] + searches[-1][1]
    wall = t_hi - t_lo
    slow = [(s, s + l) for s, l in searches if l >= cut]
    rep = {}
    for name, a, b in spans:
        r = rep.setdefault(name, {"n": 0, "ms": 0.0, "slow_overlaps": 0})
        r["n"] += 1
        r["ms"] += max(0.0, min(b, t_hi) - max(a, t_lo))
    for name in rep:
        iv = [(a, b) for n, a, b in spans if n == name]
        rep[name]["slow_overlaps"] = sum(1 for s0, s1 in slow if any(a < s1 and b > s0 for a, b in iv))
    out = {"searches": len(searches), "slow_cut_ms": round(cut, 3), "slow": len(slow), "wall_ms": round(wall, 1),
           "phases": {k: {"count": v["n"], "time_frac": round(v["ms"] / wall, 4),
                          "slow_frac": round(v["slow_overlaps"] / max(len(slow), 1), 3)}
                      for k, v in sorted(rep.items(), key=lambda kv: -kv[1]["slow_overlaps"])},
           "slowest": [{"start_ms": round(s0 - t_lo, 3), "lat_ms": round(s1 - s0, 3),
                        "overlapping": sorted({n for n, a, b in spans if a < s1 and b > s0})}
                       for s0, s1 in sorted(slow, key=lambda x: x[0] - x[1])[:10]]}
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--docs", type=int, default=10_000_000)
    r.add_argument("--out", default="gpurun_out/stall")
    a = sub.add_parser("analyze")
    a.add_argument("dir")
    a.add_argument("--slow", type=float, default=None)
    args = ap.parse_args()
    run(args) if args.cmd == "run" else analyze(args)


if __name__ == "__main__":
    main()
