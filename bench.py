"""fugu query hot path on MI355X: queries/sec + p50 latency on a synthetic
10M-doc Zipf corpus, 3-term AND, BM25 top-100 (BASELINE.json `metric`).

A step = one batch of 1024 planned queries through the gfx950 pipeline
(k_conj -> k_final) with the plan and the index resident in HBM.
N > 1 (torchrun, one rank per GPU): rank r holds namespace r (its own 10M-doc
corpus, weak scaling); every step also all-gathers the per-shard top-100 over
RCCL and merges them on the device (fan-out query over all namespaces).

Prints ONE JSON line on rank 0.  See DESIGN.md §Measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "queries/sec + p50 latency, 10M-doc Zipf corpus, 3-term AND, top-100"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def workload_key(kname, n_docs, batch, k, terms, extra=""):
    """The key a committed rocprofv3 profile of a bench workload is filed under
    (profiles/latest.json "workloads"), e.g. "k_conj|n10000000|b1024|k100|t3"."""
    return f"{kname}|n{n_docs}|b{batch}|k{k}|t{terms}" + (f"|{extra}" if extra else "")


def measured_traffic(key):
    """(HBM bytes per launch of the workload's dominant kernel, source) from the
    committed profile registry when its lib_id is this build's, else (None, reason)."""
    reg = os.environ.get("FUGU_PMC_BYTES") or os.path.join(ROOT, "profiles", "latest.json")
    if not os.path.exists(reg):
        return None, "no profiles/latest.json"
    with open(reg) as f:
        pmc = json.load(f)
    e = pmc.get("workloads", {}).get(key)
    if e is None:
        return None, f"no profile of {key}"
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from lib_id import lib_id
    if e.get("lib_id") != lib_id():
        return None, f"profile of {key} is of lib {e.get('lib_id')}, this build is {lib_id()}"
    return e.get("hbm_bytes_per_launch"), e.get("source")


def roofline(kname, kernel_ms, model, key, alg_model, pruned=None):
    """The roofline object of one bench line: algorithmic bytes (fg_model_batch)
    over the kernel's HIP-event time vs the HBM peak, the 128-B line floor of the
    same loads, and the measured DRAM bytes of the same workload and build
    (rocprofv3 PMC, committed under profiles/) when there is a profile."""
    t = kernel_ms * 1e-3
    if model is None:  # --no-model (profiling passes): the kernel and its workload only
        return {"bound": "hbm", "kernel": kname, "kernel_ms": round(kernel_ms, 4), "workload_key": key}
    alg = model["alg_bytes"]
    r = {"bound": "hbm", "kernel": kname, "kernel_ms": round(kernel_ms, 4), "alg_bytes_per_launch": alg,
         "achieved": round(alg / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4), "alg_model": alg_model,
         "alg_bytes_split": {"stream": model["stream_bytes"], "probe": model["probe_bytes"],
                             "output": model["output_bytes"]},
         "line_floor_bytes": model["line_bytes"], "query_line_bytes": model["query_line_bytes"],
         "line_floor_gbs": round(model["line_bytes"] / t / 1e9, 1), "workload_key": key}
    # three fractions of the HBM peak side by side: the line's
    # model (k_conj: the exhaustive cascade; k_disj: already at the final threshold),
    # the same model replayed at each query's final threshold (the work an exact
    # pruned kernel must do), and the measured DRAM bytes
    r["frac_model"] = r["frac"]
    pruned_alg = pruned["alg_bytes"] if pruned is not None else (alg if "final" in alg_model else None)
    r["frac_pruned"] = round(pruned_alg / t / 1e9 / HBM_PEAK_GBS, 4) if pruned_alg else None
    if pruned is not None:
        r["at_final_threshold"] = {"alg_bytes": pruned["alg_bytes"], "line_floor_bytes": pruned["line_bytes"],
                                   "query_line_bytes": pruned["query_line_bytes"]}
    traffic, src = measured_traffic(key)
    r["traffic"] = traffic
    r["frac_rule"] = "the model's bytes (no measured traffic at this build)"
    if traffic:
        r.update({"traffic_source": src, "traffic_over_alg": round(traffic / alg, 3),
                  "traffic_over_line_floor": round(traffic / model["line_bytes"], 3),
                  "hbm_gbs_measured": round(traffic / t / 1e9, 1),
                  "hbm_frac_measured": round(traffic / t / 1e9 / HBM_PEAK_GBS, 4)})
        # a model more than 1.5x the bytes the kernel measurably moved (C3's
        # exhaustive cascade: 7.5 vs 3.2 GB) overstates its work: frac is then the
        # measured DRAM fraction
        if alg > 1.5 * traffic:
            r["frac"] = r["hbm_frac_measured"]
            r["achieved"] = r["hbm_gbs_measured"]
            r["frac_rule"] = "measured DRAM bytes (the model exceeds them by more than 1.5x)"
        else:
            r["frac_rule"] = "the model's bytes (within 1.5x of the measured DRAM bytes)"
    else:
        log(f"[bench] {key}: roofline.traffic = null ({src})")
    return r


NO_MODEL = False  # --no-model: profiling passes skip the host replays
# C5 over N GPUs, opt-in: the fraction of each rank's k_disj sweep run before the
# ranks' score histograms are summed (shard.exchange_hist).  Default 0 (none):
# the sweep's first items are its longest (no threshold yet), so a launch split
# after 1/16 / 1/4 / 1/2 of them idles the GPU through their tail -- one shard
# 5.96 ms whole, 8.08 / 7.52 / 7.04 ms in two parts with the summed histogram
# (tools/c5_parts.py, profiles/r05/ab/c5_parts_r05r.json)
C5_XFRAC = float(os.environ.get("FUGU_C5_XFRAC", "0"))


def model_sum(ixs, q_off, terms, k, thr, mode):
    """fg_model_batch over the snapshots of one multi-snapshot plan (their arrays
    are disjoint, so bytes and lines add up)."""
    if NO_MODEL:
        return None
    tot = None
    for ix in ixs:
        m, _ = ix.model(q_off, terms, k, thr=thr, mode=mode)
        tot = m if tot is None else {n: tot[n] + m[n] for n in tot}
    return tot


def final_thresholds(s, n, k):
    """Each query's final k-th best score (0 when it has fewer than k hits)."""
    s = np.asarray(s).reshape(len(n), k)
    return np.where(np.asarray(n) >= k, s[:, k - 1], 0.0).astype(np.float32)


def host_cores():
    """The host CPU share this process may use (T = nproc on the box).
    nproc honours OMP_NUM_THREADS (16 on the GPU box = its CPU share per GPU);
    the affinity mask and the cgroup quota are reported beside it."""
    import subprocess
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True, check=True).stdout.strip())
    except Exception:
        nproc = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except Exception:
        pass
    return {"nproc": nproc, "affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
            "cgroup_cpus": quota}


def host_threads(cores):
    """Host threads of this rank: FUGU_THREADS, else nproc -- except under a
    launcher that sets OMP_NUM_THREADS=1 for every rank (torchrun), where the
    CPU share (cgroup quota or affinity) is split over the node's ranks."""
    if os.environ.get("FUGU_THREADS"):
        return int(os.environ["FUGU_THREADS"])
    if os.environ.get("OMP_NUM_THREADS") == "1" and "LOCAL_WORLD_SIZE" in os.environ:
        share = cores["cgroup_cpus"] or cores["affinity"]
        return max(1, int(share) // max(1, int(os.environ["LOCAL_WORLD_SIZE"])))
    return cores["nproc"]


def native_oracle():
    """Compile the CPU baseline (oracle/fugu_oracle.c) for THIS host with
    -march=native and point oracle.py at it; returns the flags."""
    import subprocess
    import tempfile
    d = tempfile.mkdtemp(prefix="fugu_oracle_")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native", f"OUT={d}"],
                       capture_output=True, text=True)
    lib = os.path.join(d, "libfugu_oracle_native.so")
    if r.returncode == 0 and os.path.exists(lib):
        os.environ["FUGU_ORACLE_LIB"] = lib
        from oracle import oracle as orc
        return orc.NATIVE_FLAGS
    log(f"[bench] native oracle build failed ({r.stderr[-300:]}); using the portable build")
    return "-O3 -ffp-contract=off -march=x86-64-v2 (portable build: native compile failed)"


def throughput_fields(nq, world, steps, elapsed_s):
    """The headline's throughput at N ranks: a step is ONE fan-out batch of nq
    queries (each answered once, from the N namespaces' merged lists), so `value`
    counts nq per step whatever N is; the (query, namespace) pairs the ranks
    searched are reported beside it, never as `value`."""
    return {"value": round(nq * steps / elapsed_s, 1),
            "namespace_queries_per_s": round(nq * world * steps / elapsed_s, 1),
            "queries_per_step": nq}


def timed_steps(step, steps, warmup, torch):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def e2e_pipeline(ix, native, synth, torch, dev, nq, K, steps, workers):
    """End-to-end batch throughput: every step plans a DIFFERENT 1024-query batch
    on the host (fg_plan_create: cost order, work items, H2D), executes it and
    copies the hits back (D2H), with `workers` batches in flight on their own
    streams so host planning overlaps the kernels of the other batches."""
    import threading
    batches = [synth.queries(nq, 3, 3, seed_q=1000 + i) for i in range(steps + workers)]
    streams = [torch.cuda.Stream(dev) for _ in range(workers)]
    plan_ms, run_ms, close_ms, errors = [], [], [], []

    def work(w, idxs):
        try:
            for i in idxs:
                t1 = time.perf_counter()
                p = ix.plan(batches[i][0], batches[i][1], K)
                t2 = time.perf_counter()
                p.execute(streams[w].cuda_stream)
                p.results()
                t3 = time.perf_counter()
                p.close()
                plan_ms.append((t2 - t1) * 1e3)
                run_ms.append((t3 - t2) * 1e3)
                close_ms.append((time.perf_counter() - t3) * 1e3)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    def run(idxs_all):
        th = [threading.Thread(target=work, args=(w, idxs_all[w::workers])) for w in range(workers)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    run(list(range(steps, steps + workers)))  # warm the workspace pool and the streams
    plan_ms.clear()
    run_ms.clear()
    close_ms.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(list(range(steps)))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if errors:
        raise RuntimeError(errors[0])
    return {"value": round(nq * steps / el, 1), "unit": "queries/s", "ms_per_batch": round(el * 1e3 / steps, 3),
            "batches": steps, "batch": nq, "k": K, "workers": workers,
            "plan_ms_per_batch_p50": round(float(np.median(plan_ms)), 3),
            "breakdown_ms_p50": {"plan_host": round(float(np.median(plan_ms)), 3),
                                 "execute_to_hits_on_host": round(float(np.median(run_ms)), 3),
                                 "plan_destroy": round(float(np.median(close_ms)), 3)},
            "breakdown_ms_p90": {"plan_host": round(float(np.percentile(plan_ms, 90)), 3),
                                 "execute_to_hits_on_host": round(float(np.percentile(run_ms, 90)), 3)},
            "note": "each step = a different 3-term AND batch: host planning + H2D + k_conj + k_final + D2H of the "
                    "hits, pipelined over the workers' streams (planning overlaps other batches' kernels); "
                    "execute_to_hits_on_host includes waiting behind the other workers' kernels on the GPU"}


def bench_db_api(ctx, corp, native, synth, ref, threads, nq=200, n_seg=8):
    """The default API shape end to end through the host mirror: a 10M-doc
    namespace ingested by n_seg POST /batch/upsert calls (one commit, one
    segment each: src/db/document.rs:65), then batch-of-one GET /search?q=a b
    (bare terms = Should, limit 20: src/server/handlers/search.rs:36, 370-374;
    src/db/search.rs:112) through fg_db_search: parse, dictionary, ONE
    fg_search_sharded over the 8 segments (shared thresholds, device merge),
    hits out; and the same query through the full handler (JSON with the 20
    docs fetched).  Parity sample: the oracle's top-20 (an OR does not depend
    on the segmentation)."""
    from fugu_amd import db as fdb
    # LogMergePolicy::set_max_docs_before_merge(2^20): the 8 bulk segments of
    # 1.25M docs stay 8 (tantivy's default 10M would merge them into one in the
    # background), so this line keeps measuring the segmented search path
    os.environ.setdefault("FUGU_MERGE_MAX_DOCS", str(1 << 20))
    t0 = time.time()
    d = fdb.Database(ctx)
    d.create_namespace("api")
    tb, to = synth.render_text(corp, threads)
    ib, io = synth.render_ids(corp.n_docs)
    bounds = [corp.n_docs * i // n_seg for i in range(n_seg + 1)]
    for a, b in zip(bounds[:-1], bounds[1:]):
        d.upsert_batch("api", id_buf=ib[int(io[a]):int(io[b])], id_off=io[a:b + 1] - io[a],
                       text_buf=tb[int(to[a]):int(to[b])], text_off=to[a:b + 1] - to[a])
    del tb, ib
    ingest_s = time.time() - t0
    q_off, terms = synth.queries(nq, 2, 5, seed_q=333)
    qs = [" ".join(f"t{t}" for t in terms[q_off[i]:q_off[i + 1]]) for i in range(nq)]
    # the JSON handler on queries of its own (not a warm repeat of a query just run)
    qj_off, qj_terms = synth.queries(nq, 2, 5, seed_q=334)
    qjs = [" ".join(f"t{t}" for t in qj_terms[qj_off[i]:qj_off[i + 1]]) for i in range(nq)]
    for q in qs[:8]:
        d.search("api", q, 0, 20)
    lat, lat_json, mism = [], [], 0
    got_all = []
    for i, q in enumerate(qs):
        t1 = time.perf_counter()
        got_all.append(d.search("api", q, 0, 20))
        lat.append(time.perf_counter() - t1)
    for q in qjs:
        t1 = time.perf_counter()
        d.search_json("api", q, 0, 20)
        lat_json.append(time.perf_counter() - t1)
    # the same queries again with the phase trace on (fg_search_trace): where a
    # GET /search batch of one spends its time
    fdb.search_trace(1)
    fdb.search_trace()
    for q in qs:
        d.search("api", q, 0, 20)
    ph = fdb.search_trace(0)
    phases = {k: round(v / max(ph["calls"], 1), 4) for k, v in ph.items() if k not in ("calls", "json_fetch")}
    fdb.search_trace(1)
    fdb.search_trace()
    for q in qjs:
        d.search_json("api", q, 0, 20)
    phj = fdb.search_trace(0)
    phases["json_fetch"] = round(phj["json_fetch"] / max(phj["calls"], 1), 4)
    if ref is not None:
        for i, got in enumerate(got_all):
            rs, rd = ref.search(terms[q_off[i]:q_off[i + 1]], 20, mode=1)
            if [g[1] for g in got] != rd.tolist() or not np.allclose([g[0] for g in got], rs, rtol=1e-5, atol=0):
                mism += 1
    pct = lambda v, p: round(float(np.percentile(v, p) * 1e3), 4)  # noqa: E731
    out = {"p50_ms": pct(lat, 50), "p90_ms": pct(lat, 90), "p99_ms": pct(lat, 99),
           "json_p50_ms": pct(lat_json, 50), "json_p99_ms": pct(lat_json, 99), "queries": nq, "segments": n_seg,
           "k": 20, "mode": "OR (bare terms)", "ingest_s": round(ingest_s, 1), "n_docs": corp.n_docs,
           "phases_ms_mean": phases,
           "note": "batch of one through fg_db_search (parse + dictionary + fg_search_sharded over the namespace's "
                   "8 commit segments + device merge + hits out); json_*: the GET /search handler shape with the "
                   "20 docs fetched from the host doc store, on queries of its own; phases_ms_mean: fg_search_trace "
                   "means per call (a second pass over the same queries with the trace on)"}
    if ref is not None:
        out["parity"] = {"queries_checked": nq, "mismatches": mism}
    # ---- commits on the 10M namespace: 16 consecutive POST
    # /batch/upsert calls of 1000 new docs, each one fg_db_commit (a new segment;
    # the older ones take the new statistics on the host, scored at query time:
    # src/db/document.rs:65);
    # past 8 segments the background merger folds the small ones together
    # (IndexWriter merge threads, src/db/core.rs:247-249), off the commit path
    n_new, n_commits = 1000, 16
    new = synth.corpus(n_new * n_commits, doc_begin=corp.n_docs, threads=threads)
    tb2, to2 = synth.render_text(new, threads)
    ib2, io2 = synth.render_ids(n_new * n_commits, doc_begin=corp.n_docs)
    lat_c = []
    # GET /search from a reader thread the whole time the commits (and the
    # merges they queue) run: ctypes drops the GIL inside both calls, so the
    # reader searches while the writer gathers, builds and swaps
    import threading
    stop = threading.Event()
    lat_r, err_r, ph_r, t_r = [], [], [], []
    fdb.search_trace(1)

    warm = threading.Event()

    def reader():
        i = 0
        try:
            # the thread's first HIP calls set up its per-thread runtime state (a
            # server's worker threads are warm): untimed, before the commits start
            for j in range(3):
                d.search("api", qs[j % nq], 0, 20)
            warm.set()
            fdb.search_trace()
            while not stop.is_set():
                t0 = time.monotonic()  # the steady clock of the native traces' @ stamps
                t1 = time.perf_counter()
                d.search("api", qs[i % nq], 0, 20)
                lat_r.append(time.perf_counter() - t1)
                t_r.append(t0)
                ph_r.append(fdb.search_trace())  # this search's phases (only this thread searches)
                i += 1
        except Exception as e:  # noqa: BLE001
            err_r.append(repr(e))
            warm.set()

    th = threading.Thread(target=reader)
    th.start()
    warm.wait()
    t_all = time.perf_counter()
    for c in range(n_commits):
        a, b = c * n_new, (c + 1) * n_new
        t1 = time.perf_counter()
        d.upsert_batch("api", id_buf=ib2[int(io2[a]):int(io2[b])], id_off=io2[a:b + 1] - io2[a],
                       text_buf=tb2[int(to2[a]):int(to2[b])], text_off=to2[a:b + 1] - to2[a])
        lat_c.append(time.perf_counter() - t1)
    t_commits = time.perf_counter() - t_all
    stop.set()
    th.join()
    fdb.search_trace(0)
    if err_r:
        raise RuntimeError(err_r[0])
    # where the slowest 1% of the searches during commits spent their time
    cut = float(np.percentile(lat_r, 99))
    slow = [p for l, p in zip(lat_r, ph_r) if l >= cut]
    slow_ph = {k: round(float(np.mean([p[k] for p in slow])), 4) for k in fdb.SEARCH_PHASES if k != "json_fetch"}
    d.merge_wait("api")
    t_done = time.perf_counter() - t_all
    if os.environ.get("FUGU_STALL_TRACE"):  # tools/stall_trace.py: every reader search (start ms, latency ms)
        with open(os.environ["FUGU_STALL_TRACE"], "w") as f:
            json.dump([[round(t * 1e3, 3), round(l * 1e3, 4)] for t, l in zip(t_r, lat_r)], f)
    out["during_commits"] = {"p50_ms": pct(lat_r, 50), "p90_ms": pct(lat_r, 90), "p99_ms": pct(lat_r, 99),
                             "max_ms": round(max(lat_r) * 1e3, 3), "searches": len(lat_r),
                             "p99_over_idle_p99": round(pct(lat_r, 99) / max(out["p99_ms"], 1e-9), 3),
                             "slowest_1pct_phases_ms_mean": slow_ph,
                             "note": "GET /search (fg_db_search, OR limit 20) back to back from a second thread while "
                                     "the 16 commits of commit_10M run; the read path takes no writer lock"}
    mi = d.merge_info("api")
    ms = [x * 1e3 for x in lat_c]
    commits = {"commits": n_commits, "docs_per_commit": n_new, "base_docs": corp.n_docs,
               "commit_ms": [round(x, 1) for x in ms],
               "p50_ms": round(float(np.percentile(ms, 50)), 1), "p99_ms": round(float(np.percentile(ms, 99)), 1),
               "max_ms": round(max(ms), 1), "wall_16_commits_ms": round(t_commits * 1e3, 1),
               "wall_incl_background_merges_ms": round(t_done * 1e3, 1),
               "merges": mi["merges"], "merge_ms_max": round(mi["merge_ms_max"], 1),
               "merge_ms_total": round(mi["merge_ms_total"], 1), "segments_after": mi["segments"],
               "note": "each commit = POST /batch/upsert of 1000 docs through fg_db_upsert_batch (analyzer, dictionary, "
                       "raw-id deletes, a new segment built with the namespace statistics over its own term "
                       "dictionary, the older segments given the new statistics on the host: no device work, scores "
                       "formed at query time); merges run on the background merger and are waited for at the end"}
    d.close()
    return out, commits


def fanout(plans, gs, gd, gn, streams, torch, dev):
    """One fan-out step's shard executes: every shard's plan on its own stream
    (the shards are independent, so one shard's tail overlaps the next one's
    start), joined back into torch's current stream before the merge."""
    main = torch.cuda.current_stream(dev)
    ev = torch.cuda.Event()
    ev.record(main)
    for r, p in enumerate(plans):
        s = streams[r % len(streams)]
        s.wait_event(ev)
        p.execute(s.cuda_stream, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
    for s in streams:
        main.wait_stream(s)


def merge_ms(gs, gd, gn, nq, K, torch, reps=20):
    """Device time of one fg_merge_shards call on the gathered lists (torch's
    current stream, where merge_on_device launches it)."""
    from fugu_amd.shard import merge_on_device
    st = torch.cuda.current_stream(gs.device)
    merge_on_device(gs, gd, gn, nq, K, st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        merge_on_device(gs, gd, gn, nq, K, st.cuda_stream)
    e1.record(st)
    e1.synchronize()
    return round(e0.elapsed_time(e1) / reps, 4)


def bench_c4(ctx, corp, native, synth, torch, dev, nq, K, steps, warmup, threads):
    """C4 (BASELINE configs[3]) on one GPU: the 10M docs as 8 namespaces x
    1.25M, each its own index and statistics; a step = one fan-out 3-term AND
    top-100 batch on all 8 namespaces + the device merge of the 8 top-100 lists
    (what each GPU of the 8-GPU run does for its namespace, then the RCCL
    gather's merge)."""
    from fugu_amd.shard import merge_on_device, shard_ranges
    q_off, terms = synth.queries(nq, 3, 3)
    ranges = shard_ranges(corp.n_docs, 8)
    ixs, plans = [], []
    t0 = time.time()
    for b, e in ranges:
        off = corp.off[b:e + 1] - corp.off[b]
        ix = native.Index.from_docs(ctx, off, corp.tok[corp.off[b]:corp.off[e]], synth.VOCAB, threads=threads,
                                    keep_host=True)
        ixs.append(ix)
        plans.append(ix.plan(q_off, terms, K))
    build_s = time.time() - t0
    gs = torch.empty((8, nq * K), dtype=torch.float32, device=dev)
    gd = torch.empty((8, nq * K), dtype=torch.int32, device=dev)
    gn = torch.empty((8, nq), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream

    streams = [torch.cuda.Stream(dev) for _ in range(8)]

    def step_seq():
        for r, p in enumerate(plans):
            p.execute(st, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        merge_on_device(gs, gd, gn, nq, K, st)

    def step_fan():
        fanout(plans, gs, gd, gn, streams, torch, dev)
        merge_on_device(gs, gd, gn, nq, K, st)

    # per-namespace kernel times from back-to-back launches; then the 8
    # namespaces on 8 streams; then the step: ONE multi-snapshot plan over the 8
    # namespaces (one launch per kernel, shared score-only thresholds), the plan
    # fg_search_sharded runs for a device's namespaces
    for p in plans:
        p.profile(True)
    el_seq = timed_steps(step_seq, steps, warmup, torch)
    kms = [p.kernel_ms() for p in plans]
    per_ns = [round(m[0][0] / max(m[1], 1), 4) for m in kms]
    for p in plans:
        p.profile(False)
    el_fan = timed_steps(step_fan, steps, warmup, torch)
    mp = native.Plan(ixs, q_off, terms, K)
    os_, od_, osh_ = (torch.empty(nq * K, dtype=t, device=dev) for t in (torch.float32, torch.int32, torch.int32))
    on_ = torch.empty(nq, dtype=torch.int32, device=dev)

    def step():  # the merged select: the merged lists straight from k_final
        mp.execute_merged(st, os_.data_ptr(), od_.data_ptr(), osh_.data_ptr(), on_.data_ptr())

    mp.profile(True)
    el = timed_steps(step, steps, warmup, torch)
    mk, mkn = mp.kernel_ms()
    # roofline of the multi-snapshot k_conj: every namespace's exhaustive cascade
    # (and pruned at the merged k-th score, the shared score-only threshold)
    t0 = time.time()
    thr = final_thresholds(os_.cpu().numpy(), on_.cpu().numpy(), K)
    roof = roofline("k_conj", mk[0] / max(mkn, 1), model_sum(ixs, q_off, terms, K, None, native.MODE_AND),
                    workload_key("k_conj", corp.n_docs, nq, K, 3, "c4 8ns"),
                    "fg_model_batch over the 8 namespaces: k_conj's exhaustive cascade (as the headline)",
                    model_sum(ixs, q_off, terms, K, thr, native.MODE_AND))
    log(f"[bench] C4 models in {time.time() - t0:.1f}s")
    mms = merge_ms(gs, gd, gn, nq, K, torch)
    # the same fan-out through the ABI call a host makes: fg_search_sharded
    # (host batch in, merged host hits out: 8 plans, 8 executes, merge, D2H)
    ms_, md, msh, mn = merge_on_device(gs, gd, gn, nq, K, st)
    torch.cuda.synchronize()
    for _ in range(3):  # (warms the plan-workspace and pinned pools for every part size)
        native.search_sharded(ixs, q_off, terms, K)
    t0 = time.perf_counter()
    for _ in range(steps):
        s2, d2, sh2, n2 = native.search_sharded(ixs, q_off, terms, K)
    sharded_ms = (time.perf_counter() - t0) * 1e3 / steps
    mn = mn.cpu().numpy()
    same = bool(np.array_equal(n2, mn))
    ms_, md, msh = (x.cpu().numpy().reshape(nq, K) for x in (ms_, md, msh))
    for i in range(nq):
        m = int(mn[i])
        same = same and np.array_equal(s2[i, :m], ms_[i, :m]) and np.array_equal(
            d2[i, :m], md[i, :m].view(np.uint32)) and np.array_equal(sh2[i, :m], msh[i, :m].astype(np.uint32))
    del plans, mp
    for ix in ixs:
        ix.close()
    return {"value": round(nq * steps / el, 1), "unit": "queries/s", "ms_per_step": round(el * 1e3 / steps, 4),
            "batch": nq, "k": K, "terms": 3, "mode": "AND", "namespaces": 8, "docs_per_namespace": ranges[0][1],
            "step": "one multi-snapshot plan over the 8 namespaces (fg_plan_create_multi) and its merged select "
                    "(fg_plan_execute_merged)",
            "multi_plan_kernels_ms": [round(mk[0] / max(mkn, 1), 4), round(mk[1] / max(mkn, 1), 4)],
            "roofline": roof,
            "k_conj_ms_per_namespace": per_ns, "merge_ms": mms, "snapshot_build_s": round(build_s, 1),
            "ms_per_step_8_plans_8_streams": round(el_fan * 1e3 / steps, 4),
            "ms_per_step_8_plans_one_stream": round(el_seq * 1e3 / steps, 4),
            "fg_search_sharded": {"value": round(nq / sharded_ms * 1e3, 1), "ms_per_batch": round(sharded_ms, 4),
                                  "same_hits_as_step": same,
                                  "note": "one synchronous ABI call per batch: host planning of 8 namespaces "
                                          "(in parallel), one multi-snapshot plan, device merge, D2H"},
            "workload": "C4: 10M docs as 8 namespaces x 1.25M (own statistics each), fan-out 3-term AND top-100 "
                        "on all 8 + device merge, all 8 namespaces on this one GPU",
            "projected_8gpu": "each GPU runs one namespace: step ~ max(k_conj_ms_per_namespace) + k_final + gather"}


def alone_kernel_ms(ixs, q_off, terms, K, mode, st, reps):
    """Every shard's plan run ALONE (no shared threshold word): each shard's
    kernel ms as one GPU of an 8-GPU doc-sharded run sees it (k_disj / k_conj,
    k_final), and the hash of the hits merged from the shards' lists."""
    from fugu_amd.shard import merge_on_device
    import torch
    nq = len(q_off) - 1
    dev = torch.device(f"cuda:{torch.cuda.current_device()}")
    gs = torch.empty((len(ixs), nq * K), dtype=torch.float32, device=dev)
    gd = torch.empty((len(ixs), nq * K), dtype=torch.int32, device=dev)
    gn = torch.empty((len(ixs), nq), dtype=torch.int32, device=dev)
    ms = []
    for r, ix in enumerate(ixs):
        p = ix.plan(q_off, terms, K, mode)
        p.execute(st, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        torch.cuda.synchronize()
        p.profile(True)
        for _ in range(reps):
            p.execute(st, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        torch.cuda.synchronize()
        m, n = p.kernel_ms()
        ms.append((round(m[0] / max(n, 1), 4), round(m[1] / max(n, 1), 4)))
        p.close()
    out = merge_on_device(gs, gd, gn, nq, K, st)
    torch.cuda.synchronize()
    return ms, hits_sha1(out[0], out[1], out[2], out[3], K)


def peers_rehearsal(ixs, q_off, terms, K, native, torch, gs, gd, gn, st, reps):
    """C5's 8-GPU threshold sharing rehearsed on one GPU: every shard's plan a
    PEER of the others' (fg_plan_set_peers: its thresholds and hit counts also
    published into theirs during the launch), the 8 plans on 8 streams at once.
    Sharing one GPU, each shard progresses at ~1/8 of its speed, so thresholds
    evolve per posting as on 8 GPUs: wall / 8 is the per-GPU time of the split."""
    from fugu_amd.shard import agree_hist_span, merge_on_device
    nq = len(q_off) - 1
    plans = [ix.plan(q_off, terms, K, native.MODE_OR) for ix in ixs]
    agree_hist_span(plans)
    for i, p in enumerate(plans):
        p.set_peers([x for j, x in enumerate(plans) if j != i])
    streams = [torch.cuda.Stream() for _ in plans]

    def rnd():
        for p in plans:
            p.reset(st)
        torch.cuda.synchronize()  # every reset before any peer's kernels
        t = time.perf_counter()
        for r, (p, s) in enumerate(zip(plans, streams)):
            p.execute(s.cuda_stream, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    rnd()
    walls = [rnd() for _ in range(reps)]
    out = merge_on_device(gs, gd, gn, nq, K, st)
    torch.cuda.synchronize()
    sha = hits_sha1(out[0], out[1], out[2], out[3], K)
    for p in plans:
        p.set_peers([])
        p.close()
    w = float(np.median(walls))
    return {"wall_ms": round(w, 4), "per_gpu_ms": round(w / len(plans), 4), "result_sha1": sha,
            "note": "8 shard plans, peers of each other (fg_plan_set_peers), on 8 streams of this GPU; per_gpu_ms = "
                    "wall / 8 (tools/c5_peers.py)"}


def hits_sha1(s, d, sh, n, K):
    """sha1 (16 hex) of merged (score, doc, shard) lists, each query's first n entries."""
    import hashlib
    s, d, n = s.cpu().numpy(), d.cpu().numpy(), n.cpu().numpy()
    sh = None if sh is None else sh.cpu().numpy()
    h = hashlib.sha1()
    for i in range(len(n)):
        m = int(n[i])
        h.update(s[i * K:i * K + m].tobytes() + d[i * K:i * K + m].tobytes())
        if sh is not None:
            h.update(sh[i * K:i * K + m].tobytes())
    return h.hexdigest()[:16]


def bench_c5(ctx, native, synth, torch, dev, nq, steps, warmup, threads, cpu_seconds, do_cpu):
    """C5 (BASELINE configs[4]) on one GPU: 100M docs, Zipf s=1.1, as 8
    contiguous doc shards scored with the GLOBAL statistics (tantivy's segment
    model); a step = one 2-5-term OR top-1000 batch on all 8 shards + the device
    merge by (score desc, shard asc, doc asc)."""
    from fugu_amd.shard import merge_on_device, shard_ranges
    K, N, S = 1000, 100_000_000, 1.1
    t0 = time.time()
    c = synth.corpus(N, synth.VOCAB, S, threads=threads)
    ranges = shard_ranges(N, 8)
    parts = [(c.off[b:e + 1] - c.off[b], c.tok[c.off[b]:c.off[e]]) for b, e in ranges]
    g = None
    for off, tok in parts:
        x = native.docs_stats(off, tok, synth.VOCAB, threads=threads)
        g = x if g is None else g + x
    ixs = [native.Index.from_docs(ctx, off, tok, synth.VOCAB, threads=threads, keep_host=True, global_stats=g)
           for off, tok in parts]
    del parts
    build_s = time.time() - t0
    log(f"[bench] C5: 100M docs as 8 shards built in {build_s:.1f}s")
    q_off, terms = synth.queries(nq, 2, 5)
    plans = [ix.plan(q_off, terms, K, native.MODE_OR) for ix in ixs]
    native.link_plans(plans)
    gs = torch.empty((8, nq * K), dtype=torch.float32, device=dev)
    gd = torch.empty((8, nq * K), dtype=torch.int32, device=dev)
    gn = torch.empty((8, nq), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    merged = {}

    # the round-2/3 step: 8 linked plans back to back on one stream (per-shard times)
    def step_linked():
        for r, p in enumerate(plans):
            p.execute(st, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        merge_on_device(gs, gd, gn, nq, K, st)

    for p in plans:
        p.profile(True)
    el_linked = timed_steps(step_linked, max(2, steps // 2), 1, torch)
    kms = [p.kernel_ms() for p in plans]
    per_shard = [round(m[0][0] / max(m[1], 1), 4) for m in kms]
    del plans
    # every shard ALONE (what each GPU of the 8-GPU split runs: no threshold word
    # shared across devices), from its own K-th scores, then from the
    # namespace-wide floor (ladders exchanged once at build: shard.seed_kth_floor)
    alone_un, sha_un = alone_kernel_ms(ixs, q_off, terms, K, native.MODE_OR, st, max(2, steps // 2))
    from fugu_amd.shard import seed_kth_floor
    t0 = time.time()
    seed_kth_floor(ixs)
    seed_s = time.time() - t0
    alone_se, sha_se = alone_kernel_ms(ixs, q_off, terms, K, native.MODE_OR, st, max(2, steps // 2))
    log(f"[bench] C5 shards alone: unseeded max {max(x[0] for x in alone_un)} ms, seeded max "
        f"{max(x[0] for x in alone_se)} ms (linked mean {np.mean(per_shard):.3f}); floor in {seed_s:.1f}s")
    peers = peers_rehearsal(ixs, q_off, terms, K, native, torch, gs, gd, gn, st, max(2, steps // 2))
    log(f"[bench] C5 peers on 8 streams: {peers['wall_ms']} ms wall, {peers['per_gpu_ms']} ms per shard")
    # the step: ONE multi-snapshot plan over the 8 shards (one launch per kernel),
    # planned with the floor; beside it the same plan without the floor
    outs = tuple(torch.empty(nq * K, dtype=t, device=dev) for t in (torch.float32, torch.int32, torch.int32)) + (
        torch.empty(nq, dtype=torch.int32, device=dev),)
    for ix in ixs:
        ix.set_kth_floor(None)
    mp0 = native.Plan(ixs, q_off, terms, K, native.MODE_OR)
    mp0.profile(True)
    el0 = timed_steps(lambda: mp0.execute_merged(st, *[x.data_ptr() for x in outs]), max(2, steps // 2), 1, torch)
    mk0, mkn0 = mp0.kernel_ms()
    sha_multi_un = hits_sha1(outs[0], outs[1], outs[2], outs[3], K)
    del mp0
    seed_kth_floor(ixs)
    mp = native.Plan(ixs, q_off, terms, K, native.MODE_OR)

    def step():  # the merged select: the merged lists straight from k_final
        mp.execute_merged(st, *[x.data_ptr() for x in outs])
        merged["out"] = outs

    mp.profile(True)
    el = timed_steps(step, steps, warmup, torch)
    mk, mkn = mp.kernel_ms()
    sha_multi = hits_sha1(outs[0], outs[1], outs[2], outs[3], K)
    # roofline of the multi-snapshot k_disj: every shard replayed at the merged
    # k-th score (the shards' shared score-only threshold)
    t0 = time.time()
    thr = final_thresholds(outs[0].cpu().numpy(), outs[3].cpu().numpy(), K)
    roof = roofline("k_disj", mk[0] / max(mkn, 1), model_sum(ixs, q_off, terms, K, thr, native.MODE_OR),
                    workload_key("k_disj", N, nq, K, "2-5 OR", "c5 s=1.1 8 shards"),
                    "fg_model_batch over the 8 shards: k_disj at each query's final (merged) k-th score")
    log(f"[bench] C5 models in {time.time() - t0:.1f}s")
    mms = merge_ms(gs, gd, gn, nq, K, torch)
    ent = {"value": round(nq * steps / el, 1), "unit": "queries/s", "ms_per_step": round(el * 1e3 / steps, 4),
           "batch": nq, "k": K, "terms": "2-5", "mode": "OR", "n_docs": N, "zipf_s": S, "shards": 8,
           "step": "one multi-snapshot plan over the 8 shards (fg_plan_create_multi) and its merged select "
                   "(fg_plan_execute_merged)",
           "multi_plan_kernels_ms": [round(mk[0] / max(mkn, 1), 4), round(mk[1] / max(mkn, 1), 4)],
           "roofline": roof,
           "ms_per_step_8_linked_plans": round(el_linked * 1e3 / max(2, steps // 2), 4),
           "k_disj_ms_per_shard_linked": per_shard, "k_disj_ms_per_shard_linked_mean": round(float(np.mean(per_shard)), 4),
           "k_disj_ms_per_shard_independent": {
               "unseeded": [x[0] for x in alone_un], "seeded": [x[0] for x in alone_se],
               "unseeded_max": max(x[0] for x in alone_un), "seeded_max": max(x[0] for x in alone_se),
               "k_final_ms_seeded": [x[1] for x in alone_se],
               "seeded_max_over_linked_mean": round(max(x[0] for x in alone_se) / float(np.mean(per_shard)), 3),
               "result_sha1_unseeded": sha_un, "result_sha1_seeded": sha_se, "same_hits": sha_un == sha_se,
               "floor_s": round(seed_s, 2),
               "note": "each shard's plan alone (no shared threshold word: one GPU of the 8-GPU split); seeded = "
                       "its starting thresholds floored by the namespace-wide per-term K-th score bounds "
                       "(fg_index_term_ladder of every shard, one all-gather at build, fg_kth_floor_combine)"},
           "peers_8_streams": {**peers, "per_gpu_over_linked_mean": round(peers["per_gpu_ms"] / float(np.mean(per_shard)), 3),
                               "same_hits": peers["result_sha1"] == sha_se},
           "multi_plan_unseeded": {"ms_per_step": round(el0 * 1e3 / max(2, steps // 2), 4),
                                   "kernels_ms": [round(mk0[0] / max(mkn0, 1), 4), round(mk0[1] / max(mkn0, 1), 4)],
                                   "result_sha1": sha_multi_un},
           "result_sha1": sha_multi, "same_hits_seeded_unseeded": sha_multi == sha_multi_un,
           "merge_ms": mms, "snapshot_build_s": round(build_s, 1),
           "workload": "C5: 100M docs s=1.1 as 8 doc shards with global BM25 statistics, 2-5-term OR top-1000 on "
                       "all 8 + device merge, all 8 shards on this one GPU (the step: one multi-snapshot plan, "
                       "seeded with the namespace-wide K-th floors)",
           "projected_8gpu": "each GPU runs one shard, its plan a peer of the others' (bench --config c5 over N "
                             "GPUs: shard.link_peers): step ~ peers_8_streams.per_gpu_ms + reset barrier + all-gather "
                             "+ merge; without peers max(k_disj_ms_per_shard_independent.seeded)"}
    del mp
    for ix in ixs:
        ix.close()
    if do_cpu:
        # CPU baseline + parity on a bounded sample: ONE 100M-doc oracle index
        from oracle import oracle as orc
        ms_, md, msh, mn = merged["out"]
        base = np.array([b for b, _ in ranges], np.uint64)
        ms_ = ms_.cpu().numpy().reshape(nq, K)
        gdoc = md.cpu().numpy().view(np.uint32).reshape(nq, K).astype(np.uint64) + base[
            msh.cpu().numpy().reshape(nq, K)]
        mn = mn.cpu().numpy()
        ref = orc.OracleIndex(synth.VOCAB, c.off, c.tok, threads=threads)
        done, wall, mism = 0, 0.0, 0
        while done < nq and wall < cpu_seconds:
            hi = min(nq, done + threads)
            so = (q_off[done:hi + 1] - q_off[done]).astype(np.uint32)
            rs, rd, rn, w, _ = ref.search_batch(so, terms[q_off[done]:q_off[hi]], K, mode=orc.OR, threads=threads)
            wall += w
            for j in range(hi - done):
                i, m = done + j, int(rn[j])
                if (int(mn[i]) != m or not np.array_equal(gdoc[i, :m], rd[j, :m].astype(np.uint64))
                        or not np.allclose(ms_[i, :m], rs[j, :m], rtol=1e-5, atol=0)):
                    mism += 1
            done = hi
        ent["cpu_baseline"] = {"value": round(done / wall, 2), "unit": "queries/s", "cores": threads, "kind": "port",
                               "sample": f"first {done} queries of the batch on ONE 100M-doc oracle index "
                                         "(exhaustive union, SumCombiner)"}
        ent["parity"] = {"queries_checked": done, "mismatches": mism}
        del ref
    return ent


def run_config(args, cfg, rank, world, local, dev, backend, threads, torch, dist):
    """BASELINE configs[3] (c4) / configs[4] (c5) across the job's GPUs (strong
    scaling: the corpus is fixed, its 8 units are split over the ranks):
      c4: the 10M-doc corpus as 8 namespaces x 1.25M (own statistics each), a
          fan-out 3-term AND top-100 batch;
      c5: 100M docs, Zipf s = 1.1, as 8 doc shards scored with the namespace's
          global statistics (one all-reduce of the shard statistics at build),
          a 2-5-term OR top-1000 batch.
    Rank r holds units [8r/N, 8(r+1)/N) on its GPU, their plans linked (one
    shared threshold per query); a step = every unit's kernels, the rank's
    device merge, ONE all-gather of the rank lists (RCCL over xGMI) and the
    final device merge by (score desc, unit asc, doc asc).  Every rank prints
    nothing; rank 0 prints the JSON line, with a hash of the merged hits (equal
    for every N)."""
    import hashlib

    from fugu_amd import native, synth
    from fugu_amd.shard import allreduce_stats, gather_packed, merge_on_device, shard_ranges
    c4 = cfg == "c4"
    N, S, K = (10_000_000, 1.0, 100) if c4 else (100_000_000, 1.1, 1000)
    mode = native.MODE_AND if c4 else native.MODE_OR
    nq = args.batch
    units = 8
    if units % world:
        raise SystemExit(f"--config {cfg}: {units} units do not split over {world} ranks")
    ranges = shard_ranges(N, units)
    per = units // world
    mine = list(range(rank * per, (rank + 1) * per))
    t0 = time.time()
    parts = []
    for u in mine:
        b, e = ranges[u]
        c = synth.corpus(e - b, synth.VOCAB, S, doc_begin=b, threads=threads)
        parts.append((c.off, c.tok))
    ctx = native.Context((local,))
    g = None
    if not c4:  # global statistics: the rank's shards summed, then one all-reduce over the ranks
        for off, tok in parts:
            x = native.docs_stats(off, tok, synth.VOCAB, threads=threads)
            g = x if g is None else g + x
        if world > 1:
            g = allreduce_stats(g, device=dev if backend == "nccl" else None)
    ixs = [native.Index.from_docs(ctx, off, tok, synth.VOCAB, threads=threads, keep_host=True, global_stats=g)
           for off, tok in parts]
    del parts
    build_s = time.time() - t0
    log(f"[bench] {cfg}: rank {rank} built units {mine} in {build_s:.1f}s")
    floor_info = None
    if not c4 and os.environ.get("FUGU_C5_SEED", "1") != "0":
        # the doc shards' ladders all-gathered once (RCCL), combined into the
        # namespace-wide floor of every term's K-th scores: each rank's shards start
        # their thresholds from it (no threshold word is shared across GPUs)
        from fugu_amd.shard import seed_kth_floor
        t1 = time.time()
        seed_kth_floor(ixs, device=dev if backend == "nccl" else None)
        floor_info = {"seconds": round(time.time() - t1, 2),
                      "all_gather_bytes_per_rank": 4 * len(ixs) * synth.VOCAB * len(native.LADDER_KS)}
    q_off, terms = synth.queries(nq, 3, 3) if c4 else synth.queries(nq, 2, 5)
    # a rank's units: ONE multi-snapshot plan (one launch per kernel, shared
    # score-only thresholds); FUGU_BENCH_LINKED=1: one linked plan per unit (A/B)
    if len(ixs) > 1 and os.environ.get("FUGU_BENCH_LINKED") != "1":
        plans = [native.Plan(ixs, q_off, terms, K, mode)]
    else:
        plans = [ix.plan(q_off, terms, K, mode) for ix in ixs]
        if len(plans) > 1:
            native.link_plans(plans)
    gs = torch.empty((len(ixs), nq * K), dtype=torch.float32, device=dev)
    gd = torch.empty((len(ixs), nq * K), dtype=torch.int32, device=dev)
    gn = torch.empty((len(ixs), nq), dtype=torch.int32, device=dev)
    # unit u's doc d as a global id: c5 the corpus doc id, c4 (namespace << 24) | doc
    off_u = torch.tensor([ranges[u][0] if not c4 else (u << 24) for u in mine], dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)
    out = {}

    merged_sel = len(plans) == 1 and len(ixs) > 1
    mouts = [torch.empty(nq * K, dtype=t, device=dev) for t in (torch.float32, torch.int32, torch.int32)] + [
        torch.empty(nq, dtype=torch.int32, device=dev)]
    # C5 over N ranks: the ranks' plans are PEERS -- each publishes its thresholds
    # and hit counts into every other rank's during the launch, over xGMI
    # (shard.link_peers; one-GPU rehearsal: tools/c5_peers.py); FUGU_C5_XFRAC > 0
    # instead runs the sweep in two parts with the histograms summed between them
    xfrac = C5_XFRAC if (not c4 and world > 1 and len(plans) == 1 and 0.0 < C5_XFRAC < 1.0) else 0.0
    peers = 0
    if not c4 and world > 1 and len(plans) == 1 and backend == "nccl":
        from fugu_amd.shard import agree_hist_span
        agree_hist_span(plans, device=dev)
        if not xfrac:
            from fugu_amd.shard import link_peers, reset_peers
            peers = link_peers(plans[0])
    if xfrac:
        from fugu_amd.shard import exchange_hist
        hbuf = torch.zeros(nq * native.HIST_BINS, dtype=torch.int32, device=dev)

    def step():
        if peers:
            reset_peers(plans[0], st.cuda_stream)
        if xfrac:
            p0 = plans[0]
            p0.execute_part(st.cuda_stream, 0.0, xfrac)
            exchange_hist(p0, st.cuda_stream, hbuf)
            if merged_sel:
                p0.execute_part(st.cuda_stream, xfrac, 1.0, *[x.data_ptr() for x in mouts])
                ms, md, msh, mn = mouts
            else:
                p0.execute_part(st.cuda_stream, xfrac, 1.0, gs[0].data_ptr(), gd[0].data_ptr(), None,
                                gn[0].data_ptr())
                ms, md, msh, mn = merge_on_device(gs, gd, gn, nq, K, st.cuda_stream)
        elif merged_sel:  # the rank's units merged by the plan's own final select
            plans[0].execute_merged(st.cuda_stream, *[x.data_ptr() for x in mouts])
            ms, md, msh, mn = mouts
        else:
            for r, p in enumerate(plans):  # plans[0] first: it zeroes the shared thresholds
                p.execute(st.cuda_stream, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
            ms, md, msh, mn = merge_on_device(gs, gd, gn, nq, K, st.cuda_stream)
        # slots past a query's count hold no hit (undefined shard / doc): clamp the
        # gather index so it stays inside off_u; those slots are never read
        gdoc = (md.to(torch.int64) + off_u[msh.to(torch.int64).clamp_(0, len(mine) - 1)]).to(torch.int32)
        if world > 1:
            s2, d2, c2 = gather_packed(ms, gdoc, mn)
            out["m"] = merge_on_device(s2, d2, c2, nq, K, st.cuda_stream)
        else:
            out["m"] = (ms, gdoc, None, mn)

    for p in plans:
        p.profile(True)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    for p in plans:
        p.kernel_ms()  # drop the warmup's events
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t1
    el_rank = el
    kms = [p.kernel_ms() for p in plans]
    n_ex = max(kms[0][1] // (2 if xfrac else 1), 1)  # executes per plan (two parts each when exchanging)
    kern = sum(m[0][0] for m in kms) / n_ex
    fin = sum(m[0][1] for m in kms) / n_ex
    if world > 1:
        t = torch.tensor([el, kern], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern = float(t[0].item()), float(t[1].item())
    ms, md, _, mn = out["m"]
    mn = mn.cpu().numpy()
    ms = ms.cpu().numpy().reshape(nq, K)
    md = md.cpu().numpy().view(np.uint32).reshape(nq, K)
    h = hashlib.sha1()
    for i in range(nq):
        h.update(md[i, :mn[i]].tobytes())
        h.update(ms[i, :mn[i]].tobytes())
    # this rank's roofline: its units replayed (fg_model_batch) at the merged
    # k-th score of the whole job (c4: also k_conj's exhaustive cascade)
    kname = "k_conj" if c4 else "k_disj"
    my_ms = sum(m[0][0] for m in kms) / n_ex
    thr = final_thresholds(ms, mn, K)
    key = workload_key(kname, N, nq, K, 3 if c4 else "2-5 OR", f"c4 {per}ns" if c4 else f"c5 s=1.1 {per} shards")
    if c4:
        roof = roofline(kname, my_ms, model_sum(ixs, q_off, terms, K, None, mode), key,
                        f"fg_model_batch over the rank's {per} namespaces: k_conj's exhaustive cascade",
                        model_sum(ixs, q_off, terms, K, thr, mode))
    else:
        roof = roofline(kname, my_ms, model_sum(ixs, q_off, terms, K, thr, mode), key,
                        f"fg_model_batch over the rank's {per} shards: k_disj at each query's final (merged) k-th score")
    per_rank = None
    if world > 1:
        allr = [None] * world
        alg = roof.get("alg_bytes_per_launch")
        dist.all_gather_object(allr, {"rank": rank, "kernel_ms": roof["kernel_ms"], "frac": roof.get("frac"),
                                      "step_ms": round(el_rank * 1e3 / args.steps, 4),
                                      "frac_step": round(alg / (el_rank / args.steps) / 1e9 / HBM_PEAK_GBS, 4)
                                      if alg else None,
                                      "alg_bytes_per_launch": alg, "units": mine})
        per_rank = {"ranks": allr, "kernel_ms_min": min(x["kernel_ms"] for x in allr),
                    "kernel_ms_max": max(x["kernel_ms"] for x in allr),
                    "frac_min": min(x["frac"] or 0 for x in allr), "frac_max": max(x["frac"] or 0 for x in allr),
                    "frac_step_min": min(x["frac_step"] or 0 for x in allr),
                    "frac_step_max": max(x["frac_step"] or 0 for x in allr)}
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(nq * args.steps / el, 1), "unit": "queries/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32+f32",
            "data": "synthetic",
            "config": {"workload": ("C4: 10M docs as 8 namespaces x 1.25M, fan-out 3-term AND top-100"
                                    if c4 else "C5: 100M docs Zipf s=1.1 as 8 doc shards (global BM25 statistics), "
                                               "2-5-term OR top-1000"),
                       "n_docs": N, "batch": nq, "k": K, "units": units, "units_per_gpu": per,
                       "parallelism": f"{'namespace' if c4 else 'doc'}-shard x{world}" + (
                           (" + RCCL all-gather top-k" if backend == "nccl" else f" + {backend} all-gather (rehearsal)")
                           if world > 1 else "")},
            "kernels_ms_per_step_max_rank": {kname: round(kern, 4), "k_final": round(fin, 4)},
            "roofline": roof,
            **({"per_rank": per_rank} if per_rank else {}),
            "rank_plan": ("one multi-snapshot plan over the rank's units, merged by its final select"
                          if merged_sel else f"{len(plans)} linked plan(s) + k_merge_rank"),
            "result_sha1": h.hexdigest()[:16],
            "hits": int(mn.sum()),
            **({"kth_floor": floor_info} if floor_info else {}),
            **({"peers": {"per_rank": peers, "note": "each rank's plan publishes its thresholds and hit counts into "
                                                       "every other rank's during the launch (device atomics over "
                                                       "xGMI on HIP-IPC-mapped words: shard.link_peers); a step "
                                                       "starts with reset_peers (reset + barrier)"}} if peers else {}),
            **({"hist_exchange": {"frac": xfrac, "all_reduce_bytes_per_rank": 4 * nq * native.HIST_BINS,
                                  "note": "each rank's k_disj sweep in two parts ([0, frac), [frac, 1)); between "
                                          "them ONE all-reduce sums the ranks' per-query score histograms "
                                          "(shard.exchange_hist), so the second part prunes with every shard's "
                                          "first-part counts"}} if xfrac else {}),
            "snapshot_build_s_rank0": round(build_s, 1),
            "cpu_baseline": None,
            "note": "strong scaling of one fixed corpus; roofline = rank 0's units (per_rank: every rank's); the "
                    "headline mode (no --config) carries the CPU baseline",
        }
        print(json.dumps(line), flush=True)
    del plans[1:]
    del plans


def spawn_ranks(n):
    """`--gpus N` (N > 1) without a launcher: run the N ranks (one process per GPU,
    torch.distributed.run on 127.0.0.1) as CHILD processes of this one, which
    has not touched the GPU, and return their exit code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"[bench] --gpus {n}: launching {n} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--terms", type=int, default=3)
    ap.add_argument("--mixed", action="store_true", help="1-5 terms per query (config C3) instead of 3")
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="bound on the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--p50-queries", type=int, default=200)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the secondary workloads (C3, OR top-1000, end-to-end, C4, C5)")
    ap.add_argument("--extra-steps", type=int, default=5)
    ap.add_argument("--no-c5", action="store_true", help="skip the 100M-doc C5 secondary line")
    ap.add_argument("--e2e-workers", type=int, default=4,
                    help="batches in flight in the end-to-end line (tools/e2e_workers.py, 96 batches: 2 -> 800-943K, "
                         "4 -> 991K-1.035M, 6 -> 1.035-1.055M, 8 -> 1.03M q/s)")
    ap.add_argument("--disj", action="store_true",
                    help="headline batch = 2-5-term OR (k_disj; profiling runs, pass --k 1000 --no-cpu)")
    ap.add_argument("--overlap", action="store_true",
                    help="N > 1: each step's gather + merge on a side stream behind the next batch (opt-in: a gloo "
                         "rehearsal on one GPU measured it slower, RCCL unmeasured)")
    ap.add_argument("--no-model", action="store_true",
                    help="skip the host traffic models (profiling passes: only kernel times and counters matter)")
    ap.add_argument("--config", choices=["headline", "c4", "c5"], default="headline",
                    help="c4 / c5: BASELINE configs[3] / [4] split over the job's GPUs (strong scaling)")
    args = ap.parse_args()
    global NO_MODEL
    NO_MODEL = args.no_model

    # one process per GPU: a launcher (torchrun) sets WORLD_SIZE; without one,
    # --gpus N > 1 starts the N ranks itself (before anything touches the GPU)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return spawn_ranks(args.gpus)
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} ranks but --gpus {args.gpus}: pass --gpus equal to the rank count",
              file=sys.stderr)
        return 2

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one rank per GPU; FUGU_DIST_BACKEND=gloo rehearses the N>1 flow with
    # several ranks on fewer GPUs (the driver's runs use RCCL, one GPU each)
    backend = os.environ.get("FUGU_DIST_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from fugu_amd import native, synth

    cores = host_cores()
    threads = args.threads or host_threads(cores)
    if args.config != "headline":
        run_config(args, args.config, rank, world, local, dev, backend, threads, torch, dist)
        if world > 1:
            dist.destroy_process_group()
        return
    t0 = time.time()
    # namespace r: its own corpus (seeds offset by rank); rank 0 is the standard corpus
    corp = synth.corpus(args.docs, synth.VOCAB, 1.0, synth.SEED_L + rank, synth.SEED_T + rank, threads=threads)
    log(f"[bench] corpus {args.docs} docs, {len(corp.tok)} tokens in {time.time() - t0:.1f}s")
    t0 = time.time()
    ctx = native.Context((local,))
    ix = native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, threads=threads, keep_host=True)
    st = ix.stats()
    log(f"[bench] index: {st.n_postings} postings, {st.device_bytes / 2**30:.2f} GiB in HBM, built in "
        f"{time.time() - t0:.1f}s")

    m_min, m_max = (1, 5) if args.mixed else (2, 5) if args.disj else (args.terms, args.terms)
    qmode = native.MODE_OR if args.disj else native.MODE_AND
    kname = "k_disj" if args.disj else "k_conj"
    wl_terms = "1-5" if args.mixed else "2-5 OR" if args.disj else args.terms
    q_off_all, terms_all = synth.queries(4096, m_min, m_max)
    nq = args.batch
    q_off = q_off_all[: nq + 1].copy()
    terms = terms_all[: q_off[-1]].copy()
    K = args.k
    plan = ix.plan(q_off, terms, K, qmode)
    info = plan.info()
    log(f"[bench] plan: {info.total_chunks} work items, workspace {info.workspace_bytes / 2**20:.1f} MiB")

    out_s = torch.empty(nq * K, dtype=torch.float32, device=dev)
    out_d = torch.empty(nq * K, dtype=torch.int32, device=dev)
    out_n = torch.empty(nq, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    merged = {}  # N > 1: the last step's merged lists (result_sha1)

    def step():
        plan.execute(stream.cuda_stream, out_s.data_ptr(), out_d.data_ptr(), out_n.data_ptr())
        if world > 1:
            from fugu_amd.shard import gather_packed, merge_on_device
            s, d, c = gather_packed(out_s, out_d, out_n)
            merged["m"] = merge_on_device(s, d, c, nq, K, stream.cuda_stream)

    if world > 1 and args.overlap:
        # N > 1: a step's all-gather + merge run on a side stream while the next
        # step's batch runs (two output buffers in turn; a buffer is reused only
        # after its gather has read it), so the collective hides behind the kernels
        from fugu_amd.shard import gather_packed, merge_on_device
        side = torch.cuda.Stream(dev)
        bufs = [(torch.empty(nq * K, dtype=torch.float32, device=dev), torch.empty(nq * K, dtype=torch.int32, device=dev),
                 torch.empty(nq, dtype=torch.int32, device=dev)) for _ in range(2)]
        gathered = [None, None]
        turn = [0]

        def step():  # noqa: F811
            b = turn[0] % 2
            turn[0] += 1
            s_, d_, n_ = bufs[b]
            if gathered[b] is not None:
                stream.wait_event(gathered[b])
            plan.execute(stream.cuda_stream, s_.data_ptr(), d_.data_ptr(), n_.data_ptr())
            ran = torch.cuda.Event()
            ran.record(stream)
            side.wait_event(ran)
            with torch.cuda.stream(side):
                s, d, c = gather_packed(s_, d_, n_)
                merged["m"] = merge_on_device(s, d, c, nq, K, side.cuda_stream)
                ev = torch.cuda.Event()
                ev.record(side)
                gathered[b] = ev

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    plan.profile(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    el_rank = elapsed
    plan.profile(False)
    ms_k, n_prof = plan.kernel_ms()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    tput = throughput_fields(nq, world, args.steps, elapsed)
    result_sha1 = None
    if world > 1 and "m" in merged:  # the merged lists of the last step (equal with and without --overlap)
        import hashlib
        ms_, md_, msh_, mn_ = (x.cpu().numpy() for x in merged["m"])
        h = hashlib.sha1()
        for i in range(nq):
            m = int(mn_[i])
            h.update(ms_[i * K:i * K + m].tobytes() + md_[i * K:i * K + m].tobytes() + msh_[i * K:i * K + m].tobytes())
        result_sha1 = h.hexdigest()[:16]
    qps = tput["value"]

    # ---- p50 latency at batch = 1 (host query in, host hits out: plan + PCIe + kernels)
    lat = []
    for i in range(min(args.p50_queries, nq)):
        a, b = int(q_off[i]), int(q_off[i + 1])
        one_off = np.array([0, b - a], np.uint32)
        t1 = time.perf_counter()
        ix.search_batch(one_off, terms[a:b], K)
        lat.append(time.perf_counter() - t1)
    p50_ms = float(np.median(lat) * 1e3) if lat else None
    tail_ms = {f"p{q}": round(float(np.percentile(lat, q) * 1e3), 4) for q in (90, 99)} if lat else None

    # ---- roofline of the dominant kernel: algorithmic bytes of the batch at the
    # HBM layout (fg_model_batch: the kernel's loads replayed on the host; k_conj:
    # its exhaustive cascade, beside it the same replay pruned at each query's
    # final k-th score; k_disj: MaxScore at the final k-th score) over the
    # kernel's HIP-event time on its launch stream, with the 128-B line floor of
    # those loads and the measured DRAM bytes of the same workload and build
    t0 = time.time()
    thr_h = final_thresholds(out_s.cpu().numpy(), out_n.cpu().numpy(), K)
    conj_ms = ms_k[0] / max(n_prof, 1)
    if NO_MODEL:
        mod = pruned = None
        alg_model = None
    elif args.disj:
        mod, _ = ix.model(q_off, terms, K, thr=thr_h, mode=qmode)
        pruned = None
        alg_model = ("fg_model_batch: k_disj at each query's final k-th score (per (tile, clause) directory bounds "
                     "+ tile maximum, 8 B per essential posting, per posting past bound 1 every other clause's rank "
                     "word (8 B) + posting score (4 B) or bucket maximum (4 B), directory probes of rescored "
                     "candidates, 8 B per kept key)")
    else:
        mod, _ = ix.model(q_off, terms, K)
        pruned, _ = ix.model(q_off, terms, K, thr=thr_h)
        alg_model = ("fg_model_batch: k_conj's exhaustive cascade at the HBM layout (8 B per lead posting; per probe "
                     "8 B rank word + 4 B score on a hit, or 8 B bucket bounds + 4 B per search step + 4 B compare + "
                     "4 B score on a hit; 8 B per kept key)")
    roof = roofline(kname, conj_ms, mod, workload_key(kname, args.docs, nq, K, wl_terms), alg_model, pruned)
    if not args.disj and not NO_MODEL:
        # SURVEY.md 8(d)'s tantivy model (1 KiB block decode per probed block): a
        # byte count of the CPU walk, not bytes this layout reads
        roof["tantivy_walk_bytes_per_launch"] = float(ix.bytes_model(q_off, terms, K)[:, 2].sum())
    if mod:
        log(f"[bench] models in {time.time() - t0:.1f}s: alg {mod['alg_bytes'] / 1e9:.3f} GB, line floor "
            f"{mod['line_bytes'] / 1e9:.3f} GB, frac {roof['frac']}")

    # N > 1: every rank's kernel time and roofline fraction (its own namespace)
    per_rank = None
    if world > 1:
        alg = roof.get("alg_bytes_per_launch")
        mine = {"rank": rank, "kernel_ms": roof["kernel_ms"], "frac": roof.get("frac"),
                "step_ms": round(el_rank * 1e3 / args.steps, 4),
                # the same bytes over the rank's whole step (kernels + all-gather + merge)
                "frac_step": round(alg / (el_rank / args.steps) / 1e9 / HBM_PEAK_GBS, 4) if alg else None,
                "alg_bytes_per_launch": alg, "line_floor_bytes": roof.get("line_floor_bytes"),
                "device": torch.cuda.get_device_name(dev), "local_rank": local}
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        per_rank = {"ranks": allr,
                    "kernel_ms_min": min(r["kernel_ms"] for r in allr), "kernel_ms_max": max(r["kernel_ms"] for r in allr),
                    "frac_min": min(r["frac"] or 0 for r in allr), "frac_max": max(r["frac"] or 0 for r in allr),
                    "frac_step_min": min(r["frac_step"] or 0 for r in allr),
                    "frac_step_max": max(r["frac_step"] or 0 for r in allr),
                    "note": "frac: the rank's algorithmic bytes over its kernel time; frac_step: over its step time "
                            "(north_star: the 1-GPU fraction held within 10% at 8 GPUs)"}

    # ---- CPU baseline: the oracle (tantivy's algorithm restated in C, compiled
    # -march=native on this host) on T = nproc host threads, each running whole
    # queries (a tokio worker per request, tantivy's single-threaded executor),
    # plus a T = 1 row; rank 0, N = 1 only, bounded samples of the same batch
    cpu = None
    parity = None
    ref = None
    s_gpu = out_s.cpu().numpy().reshape(nq, K)
    d_gpu = out_d.cpu().numpy().view(np.uint32).reshape(nq, K)
    n_gpu = out_n.cpu().numpy()
    if rank == 0 and world == 1 and not args.no_cpu:
        flags = native_oracle()
        from oracle import oracle as orc
        t0 = time.time()
        ref = orc.OracleIndex(synth.VOCAB, corp.off, corp.tok, threads=threads)
        log(f"[bench] oracle index built in {time.time() - t0:.1f}s ({flags})")

        def cpu_run(T, budget, step):
            done, wall, lats, mism = 0, 0.0, [], 0
            while done < nq and wall < budget:
                hi = min(nq, done + step)
                sub_off = (q_off[done:hi + 1] - q_off[done]).astype(np.uint32)
                rs, rd, rn, w, l = ref.search_batch(sub_off, terms[q_off[done]:q_off[hi]], K, threads=T,
                                                    latencies=True)
                wall += w
                lats.append(l)
                for j in range(hi - done):
                    i, m = done + j, int(rn[j])
                    if (int(n_gpu[i]) != m or not np.array_equal(d_gpu[i, :m], rd[j, :m])
                            or not np.allclose(s_gpu[i, :m], rs[j, :m], rtol=1e-5, atol=0)):
                        mism += 1
                done = hi
            return done, wall, float(np.median(np.concatenate(lats))) * 1e-6, mism

        done, wall, p50_cpu, mism = cpu_run(threads, args.cpu_seconds, 128)
        d1, w1, p1, m1 = cpu_run(1, args.cpu_seconds / 4, 16)
        cpu = {"value": round(done / wall, 2), "unit": "queries/s", "cores": threads, "kind": "port",
               "sample": f"first {done} queries of the same 1024-query batch, {threads} threads x whole queries, "
                         f"warm in-RAM index (tantivy 0.24.1 algorithm restated in C: oracle/fugu_oracle.c)",
               "p50_ms": round(p50_cpu, 4), "compile": f"gcc {flags}", "host": cores,
               "t1": {"value": round(d1 / w1, 2), "unit": "queries/s", "cores": 1, "p50_ms": round(p1, 4),
                      "sample": f"first {d1} queries of the batch, 1 thread"}}
        parity = {"queries_checked": done, "mismatches": mism + m1, "rule": "doc ids exact, scores rtol 1e-5"}

    # ---- secondary workloads on the same index (rank 0, N=1): SURVEY §8(d) C3 and the
    # disjunctive C5 query shape (k_disj), each timed the same way and parity-sampled
    extra = None
    if rank == 0 and world == 1 and not args.no_extra:
        extra = {}
        specs = [("C3_mixed_and", 1, 5, 100, native.MODE_AND), ("OR_top1000_10M", 2, 5, 1000, native.MODE_OR),
                 ("OR_top20_default_api", 2, 5, 20, native.MODE_OR)]
        for name, a_min, a_max, kk, mode in specs:
            qo_all, qt_all = synth.queries(4096, a_min, a_max)
            qo = qo_all[: nq + 1].copy()
            qt = qt_all[: qo[-1]].copy()
            pl2 = ix.plan(qo, qt, kk, mode=mode)
            os2 = torch.empty(nq * kk, dtype=torch.float32, device=dev)
            od2 = torch.empty(nq * kk, dtype=torch.int32, device=dev)
            on2 = torch.empty(nq, dtype=torch.int32, device=dev)
            for _ in range(2):
                pl2.execute(stream.cuda_stream, os2.data_ptr(), od2.data_ptr(), on2.data_ptr())
            torch.cuda.synchronize()
            pl2.profile(True)
            t1 = time.perf_counter()
            for _ in range(args.extra_steps):
                pl2.execute(stream.cuda_stream, os2.data_ptr(), od2.data_ptr(), on2.data_ptr())
            torch.cuda.synchronize()
            el = time.perf_counter() - t1
            pl2.profile(False)
            kms, kn = pl2.kernel_ms()
            s2 = os2.cpu().numpy().reshape(nq, kk)
            d2 = od2.cpu().numpy().view(np.uint32).reshape(nq, kk)
            n2 = on2.cpu().numpy()
            kname2 = "k_conj" if mode == native.MODE_AND else "k_disj"
            kms_ = kms[0] / max(kn, 1)
            ent = {"value": round(nq * args.extra_steps / el, 1), "unit": "queries/s",
                   "ms_per_step": round(el * 1e3 / args.extra_steps, 4), "batch": nq, "k": kk,
                   "terms": f"{a_min}-{a_max}", "mode": "AND" if mode == native.MODE_AND else "OR",
                   "kernel": kname2, "kernel_ms": round(kms_, 4), "k_final_ms": round(kms[1] / max(kn, 1), 4)}
            thr2 = final_thresholds(s2, n2, kk)
            t0 = time.time()
            if mode == native.MODE_AND:
                mod2, _ = ix.model(qo, qt, kk)
                pr2, _ = ix.model(qo, qt, kk, thr=thr2)
                am = "fg_model_batch: k_conj's exhaustive cascade at the HBM layout (as the headline)"
                wterms = f"{a_min}-{a_max}" if a_min != a_max else a_min
            else:
                mod2, _ = ix.model(qo, qt, kk, thr=thr2, mode=mode)
                pr2 = None
                am = "fg_model_batch: k_disj at each query's final k-th score (as the --disj headline)"
                wterms = f"{a_min}-{a_max} OR"
            ent["roofline"] = roofline(kname2, kms_, mod2, workload_key(kname2, args.docs, nq, kk, wterms), am, pr2)
            log(f"[bench] {name}: models in {time.time() - t0:.1f}s")
            if ref is not None:
                done, wall, mism = 0, 0.0, 0
                budget = args.cpu_seconds / 2
                while done < nq and wall < budget:
                    hi = min(nq, done + 32)
                    so = (qo[done:hi + 1] - qo[done]).astype(np.uint32)
                    rs, rd, rn, w, _ = ref.search_batch(so, qt[qo[done]:qo[hi]], kk, mode=mode, threads=threads)
                    wall += w
                    for j in range(hi - done):
                        i, m = done + j, int(rn[j])
                        if (int(n2[i]) != m or not np.array_equal(d2[i, :m], rd[j, :m])
                                or not np.allclose(s2[i, :m], rs[j, :m], rtol=1e-5, atol=0)):
                            mism += 1
                    done = hi
                ent["cpu_baseline"] = {"value": round(done / wall, 2), "unit": "queries/s", "cores": threads,
                                       "kind": "port",
                                       "sample": f"first {done} queries of the batch, oracle/fugu_oracle.c "
                                                 f"({'leapfrog intersection' if mode == native.MODE_AND else 'exhaustive union, SumCombiner'})"}
                ent["parity"] = {"queries_checked": done, "mismatches": mism}
            extra[name] = ent
            log(f"[bench] {name}: {ent['value']} q/s, {ent['kernel']} {ent['kernel_ms']} ms")
            del pl2

    # ---- the same batches right after a commit of 1000 docs elsewhere in the namespace:
    # the snapshot rescored to the new statistics (host work only), so its kernels
    # form every posting's score at query time (the tf / fieldnorm payloads) and
    # scale the build-time bounds, where the fresh snapshot above reads the
    # build's scores -- the A/B of the two scoring modes on identical work
    if rank == 0 and world == 1 and not args.no_extra:
        t0 = time.time()
        more = synth.corpus(1000, synth.VOCAB, 1.0, doc_begin=args.docs, threads=threads)
        g_after = (native.docs_stats(corp.off, corp.tok, synth.VOCAB, threads=threads)
                   + native.docs_stats(more.off, more.tok, synth.VOCAB, threads=threads))
        re_ix = ix.rescore(g_after)
        rescore_ms = (time.time() - t0) * 1e3
        qt_lines = {}
        for name, a_min, a_max, kk, mode in [("AND3_top100", args.terms, args.terms, 100, native.MODE_AND),
                                             ("OR_top20", 2, 5, 20, native.MODE_OR),
                                             ("OR_top1000", 2, 5, 1000, native.MODE_OR)]:
            qo_all, qt_all = synth.queries(4096, a_min, a_max)
            qo = qo_all[: nq + 1].copy()
            qt = qt_all[: qo[-1]].copy()
            res = {}
            for tag, x in (("fresh", ix), ("after_commit", re_ix)):
                pl3 = x.plan(qo, qt, kk, mode=mode)
                o3 = [torch.empty(nq * kk, dtype=torch.float32, device=dev),
                      torch.empty(nq * kk, dtype=torch.int32, device=dev), torch.empty(nq, dtype=torch.int32, device=dev)]
                for _ in range(2):
                    pl3.execute(stream.cuda_stream, *[y.data_ptr() for y in o3])
                torch.cuda.synchronize()
                pl3.profile(True)
                for _ in range(args.extra_steps):
                    pl3.execute(stream.cuda_stream, *[y.data_ptr() for y in o3])
                torch.cuda.synchronize()
                pl3.profile(False)
                kms, kn = pl3.kernel_ms()
                res[tag] = round(kms[0] / max(kn, 1), 4)
                del pl3
            qt_lines[name] = {"kernel": "k_conj" if mode == native.MODE_AND else "k_disj",
                              "kernel_ms_build_time_scores": res["fresh"], "kernel_ms_query_time_scores":
                              res["after_commit"], "ratio": round(res["after_commit"] / res["fresh"], 3)}
        extra["scoring_modes_after_commit"] = {
            "rescore_ms": round(rescore_ms, 1), "lines": qt_lines,
            "note": "one batch of 1024 queries per line on the 10M snapshot as built (its postings' build-time "
                    "scores) and on the same snapshot rescored after a 1000-doc commit (fg_index_rescore: host "
                    "work, no device pass; scores formed at query time from the 2-B tf/fieldnorm payloads, bounds "
                    "scaled per clause); rescore_ms includes the stats of the 10M docs"}
        re_ix.close()
        log(f"[bench] scoring modes: {qt_lines}")

    # ---- end-to-end batches, then the fan-out configs C4 and C5 on this one GPU
    if rank == 0 and world == 1 and not args.no_extra:
        # 96 batches: the steady state (24 measured mostly the 4 workers' ramp-up and drain: 770K vs ~1.0M
        # q/s on the same box, profiles/r05/ab/e2e_workers_r05ad.json)
        extra["e2e_pipelined"] = e2e_pipeline(ix, native, synth, torch, dev, nq, K, 96, args.e2e_workers)
        log(f"[bench] e2e pipelined: {extra['e2e_pipelined']['value']} q/s")
    if rank == 0 and world == 1 and not args.no_extra:
        extra["db_api_default_search_10M_8seg"], extra["commit_10M"] = bench_db_api(ctx, corp, native, synth, ref,
                                                                                     threads)
        log(f"[bench] GET /search (OR, limit 20) through fg_db_search on 8 segments: "
            f"p50 {extra['db_api_default_search_10M_8seg']['p50_ms']} ms")
        log(f"[bench] 16 commits of 1000 docs on the 10M namespace: p50 {extra['commit_10M']['p50_ms']} ms, p99 "
            f"{extra['commit_10M']['p99_ms']} ms, merges {extra['commit_10M']['merges']}")
    del plan
    ix.close()
    if rank == 0 and world == 1 and not args.no_extra:
        extra["C4_8ns_fanout"] = bench_c4(ctx, corp, native, synth, torch, dev, nq, K, args.extra_steps, 2, threads)
        log(f"[bench] C4: {extra['C4_8ns_fanout']['value']} q/s")
        if not args.no_c5:
            ref = None
            del corp
            extra["C5_or_top1000_100M"] = bench_c5(ctx, native, synth, torch, dev, nq, args.extra_steps, 2, threads,
                                                   args.cpu_seconds / 2, not args.no_cpu)
            log(f"[bench] C5: {extra['C5_or_top1000_100M']['value']} q/s")

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(qps, 1),
            "unit": "queries/s",
            **({"namespace_queries_per_s": tput["namespace_queries_per_s"], "queries_per_step": nq,
                "value_counts": "fan-out queries answered (one merged top-k list each over the N namespaces)"}
               if world > 1 else {}),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32+f32",
            "data": "synthetic",
            "config": {
                "workload": (f"{'C3 mixed 1-5' if args.mixed else '2-5-term OR' if args.disj else str(args.terms) + '-term'}"
                             f"{'' if args.disj else ' AND'}, BM25 top-{K}, "
                             f"{args.docs // 1_000_000}M-doc Zipf s=1.0 corpus per namespace, batch {nq}"),
                "n_docs": args.docs, "vocab": synth.VOCAB, "batch": nq, "k": K,
                "terms": wl_terms, "namespaces": world,
                "parallelism": f"namespace-shard x{world}" + (
                    (" + RCCL all-gather top-k" if backend == "nccl" else f" + {backend} all-gather top-k (rehearsal)")
                    + (", overlapped with the next batch" if args.overlap else "") if world > 1 else ""),
            },
            "p50_ms": round(p50_ms, 4) if p50_ms is not None else None,
            "latency_ms": tail_ms,  # batch-of-one p90 / p99 beside p50 (same sample)
            **({"result_sha1": result_sha1} if result_sha1 else {}),
            "roofline": roof,
            **({"per_rank": per_rank} if per_rank else {}),
            "kernels_ms_per_step": {kname: round(ms_k[0] / max(n_prof, 1), 4),
                                    "k_final": round(ms_k[1] / max(n_prof, 1), 4)},
            "cpu_baseline": cpu,
            "parity": parity,
            "speedup_vs_cpu": round(qps / cpu["value"], 1) if cpu else None,
            "secondary": extra,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
