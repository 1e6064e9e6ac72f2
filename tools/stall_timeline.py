"""What ran on the GPU while a GET /search kernel waited to start.

Reads a rocprofv3 run's CSV output (--kernel-trace --hip-trace
--memory-copy-trace --output-format csv) of tools/db_api_bench.py: every kernel
dispatch's submit time is the end of the HIP API call that launched it (same
correlation id); its queue delay is its start minus that.  For the search
thread's dispatches (the thread that launched the most k_final / k_merge
kernels outside the commits) it reports the delay distribution and, for the
slowest, the other threads' kernels and copies that were running between submit
and start, by name: total overlap time, count, largest grid.

  python tools/stall_timeline.py <rocprofv3 output dir> [--top 30] > summary.json
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f, newline="") as fh:
            out.extend(csv.DictReader(fh))
    return out


def col(r, *names):
    for n in names:
        if n in r and r[n] != "":
            return r[n]
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--delay-ms", type=float, default=0.5)
    args = ap.parse_args()
    kern = rows(os.path.join(args.dir, "**", "*kernel_trace.csv"))
    api = rows(os.path.join(args.dir, "**", "*hip_api_trace.csv"))
    cps = rows(os.path.join(args.dir, "**", "*memory_copy_trace.csv"))
    if not kern:
        sys.exit("no kernel_trace.csv under " + args.dir)
    sub = {}  # correlation id -> (api end, api name, thread)
    for r in api:
        cid = col(r, "Correlation_Id")
        if cid is None:
            continue
        sub[cid] = (int(col(r, "End_Timestamp")), col(r, "Function", "Operation") or "", col(r, "Thread_Id"))
    K = []
    for r in kern:
        cid = col(r, "Correlation_Id")
        s, e = int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp"))
        name = col(r, "Kernel_Name") or ""
        t = sub.get(cid, (None, "", col(r, "Thread_Id")))
        grid = col(r, "Grid_Size_X", "Grid_Size", "Grid_X") or "?"
        wg = col(r, "Workgroup_Size_X", "Workgroup_Size", "Workgroup_X") or "?"
        K.append({"name": name, "start": s, "end": e, "submit": t[0], "thread": t[2] or col(r, "Thread_Id"),
                  "grid": grid, "wg": wg, "queue": col(r, "Queue_Id"), "stream": col(r, "Stream_Id")})
    C = [{"name": "copy " + (col(r, "Direction", "Operation") or ""), "start": int(col(r, "Start_Timestamp")),
          "end": int(col(r, "End_Timestamp")), "thread": col(r, "Thread_Id"),
          "bytes": col(r, "Bytes", "Size")} for r in cps]
    # the search thread: most k_final launches with a tiny grid (a batch of one)
    per_thread = collections.Counter(k["thread"] for k in K if "k_final" in k["name"] and str(k["grid"]).isdigit()
                                     and int(k["grid"]) <= 64 * 256)
    if not per_thread:
        sys.exit("no search-shaped k_final dispatches found")
    sth = per_thread.most_common(1)[0][0]
    mine = [k for k in K if k["thread"] == sth and k["submit"] is not None]
    others = [k for k in K if k["thread"] != sth] + C
    others.sort(key=lambda x: x["start"])
    delays = sorted((k["start"] - k["submit"]) / 1e6 for k in mine)
    q = lambda p: delays[min(len(delays) - 1, int(p * len(delays)))] if delays else 0
    slow = sorted(mine, key=lambda k: k["start"] - k["submit"], reverse=True)[:args.top]
    blame = collections.defaultdict(lambda: {"overlap_ms": 0.0, "count": 0, "max_grid": 0, "max_dur_ms": 0.0})
    detail = []
    for k in slow:
        a, b = k["submit"], k["start"]
        if (b - a) / 1e6 < args.delay_ms:
            continue
        ov = []
        for o in others:
            if o["start"] >= b:
                break
            if o["end"] <= a:
                continue
            t = (min(b, o["end"]) - max(a, o["start"])) / 1e6
            nm = o["name"].split("(")[0][:80]
            e = blame[nm]
            e["overlap_ms"] += t
            e["count"] += 1
            e["max_dur_ms"] = max(e["max_dur_ms"], (o["end"] - o["start"]) / 1e6)
            try:
                e["max_grid"] = max(e["max_grid"], int(o.get("grid", 0)))
            except (TypeError, ValueError):
                pass
            ov.append((round(t, 3), nm, round((o["end"] - o["start"]) / 1e6, 3), o.get("grid"), o.get("thread")))
        ov.sort(reverse=True)
        detail.append({"kernel": k["name"].split("(")[0][:80], "delay_ms": round((b - a) / 1e6, 3),
                       "ran_ms": round((k["end"] - k["start"]) / 1e6, 3), "overlapping": ov[:8]})
    out = {"search_thread": sth, "search_dispatches": len(mine),
           "queue_delay_ms": {"p50": round(q(0.5), 4), "p90": round(q(0.9), 4), "p99": round(q(0.99), 4),
                              "max": round(delays[-1], 3) if delays else 0},
           "blame_over_slowest": dict(sorted(((n, {kk: round(v, 3) if isinstance(v, float) else v
                                                    for kk, v in e.items()}) for n, e in blame.items()),
                                             key=lambda x: -x[1]["overlap_ms"])),
           "slowest": detail}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
