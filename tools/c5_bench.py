"""bench.py's C5 line alone (bench_c5): 100M docs as 8 global-statistics doc
shards on one GPU; the multi-snapshot step, and every shard ALONE as one GPU of
the 8-GPU split sees it (unseeded, and with the namespace-wide per-term floors).

  python tools/c5_bench.py [--steps K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024)
    args = ap.parse_args()
    import torch

    import bench
    from fugu_amd import native, synth
    threads = bench.host_threads(bench.host_cores())
    dev = torch.device("cuda:0")
    ctx = native.Context((0,))
    ent = bench.bench_c5(ctx, native, synth, torch, dev, args.batch, args.steps, 2, threads, 0.0, False)
    print(json.dumps(ent))


if __name__ == "__main__":
    main()
