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
