"""bench.py's counting rules (CPU).

At N > 1 the headline step is ONE fan-out batch: each of the nq queries runs on
every rank's namespace and comes back as one merged top-k list (all-gather +
k_merge_rank).  `value` therefore counts nq queries per step at every N; the
(query, namespace) pairs the ranks searched are a separate field.
"""
import ast
import os

from conftest import ROOT


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_fanout_value_counts_merged_queries():
    b = _bench()
    for world in (1, 2, 4, 8):
        f = b.throughput_fields(1024, world, 20, 0.025)
        assert f["value"] == round(1024 * 20 / 0.025, 1)  # 1024 merged answers per step, whatever N
        assert f["namespace_queries_per_s"] == round(1024 * world * 20 / 0.025, 1)
        assert f["queries_per_step"] == 1024


def test_headline_value_comes_from_throughput_fields():
    """The headline line's `value` is throughput_fields(...)['value'] (no other
    query count is multiplied by the world size)."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    tree = ast.parse(src)
    main = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "main")
    body = ast.unparse(main)
    assert "tput = throughput_fields(nq, world, args.steps, elapsed)" in body
    assert "qps = tput['value']" in body
    assert "nq * world * args.steps" not in body


def test_roofline_carries_three_fractions():
    """Every kernel line's roofline quotes the model's fraction, the fraction at
    each query's final threshold (frac_pruned) and the measured DRAM fraction; a
    model more than 1.5x the measured DRAM bytes is not the line's `frac`
    (C3's exhaustive cascade read 0.89 where the kernel moved
    0.38 of HBM)."""
    b = _bench()
    model = {"alg_bytes": 7.5e9, "stream_bytes": 5e9, "probe_bytes": 2.5e9, "output_bytes": 0,
             "line_bytes": 1.7e9, "query_line_bytes": 9e9}
    pruned = {"alg_bytes": 2.0e9, "line_bytes": 1.5e9, "query_line_bytes": 2.6e9}
    orig = b.measured_traffic
    try:
        b.measured_traffic = lambda key: (3.2e9, "profiles/test.json")
        r = b.roofline("k_conj", 1.0, model, "k", "exhaustive cascade", pruned)
        assert r["frac_model"] == round(7.5e9 / 1e-3 / 1e9 / b.HBM_PEAK_GBS, 4)
        assert r["frac_pruned"] == round(2.0e9 / 1e-3 / 1e9 / b.HBM_PEAK_GBS, 4)
        assert r["frac"] == r["hbm_frac_measured"] == round(3.2e9 / 1e-3 / 1e9 / b.HBM_PEAK_GBS, 4)
        assert "measured" in r["frac_rule"]
        b.measured_traffic = lambda key: (6.0e9, "profiles/test.json")
        r = b.roofline("k_conj", 1.0, model, "k", "exhaustive cascade", pruned)
        assert r["frac"] == r["frac_model"] and r["frac_pruned"] < r["frac"]
        b.measured_traffic = lambda key: (None, "no profile")
        r = b.roofline("k_disj", 1.0, model, "k", "k_disj at each query's final k-th score")
        assert r["frac"] == r["frac_model"] == r["frac_pruned"] and r["traffic"] is None
    finally:
        b.measured_traffic = orig
