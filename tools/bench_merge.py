"""Device time of fg_merge_shards (k_merge_rank, or the serial k_merge past
12288 scores per query) on synthetic per-shard top-k lists of the bench's
shapes: python tools/bench_merge.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    from fugu_amd import native  # noqa: F401  (loads libfugu after torch)
    sys.path.insert(0, ROOT)
    from bench import merge_ms
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(1)
    out = {}
    for S, nq, k in [(2, 1024, 100), (8, 1024, 100), (8, 1024, 1000), (64, 1024, 100), (16, 1024, 1000)]:
        sc = -np.sort(-rng.random((S, nq, k), np.float32) * 10, axis=2)
        dc = rng.integers(0, 1 << 30, (S, nq, k)).astype(np.int32)
        nn = np.full((S, nq), k, np.int32)
        gs = torch.from_numpy(sc.reshape(S, -1)).to(dev)
        gd = torch.from_numpy(dc.reshape(S, -1)).to(dev)
        gn = torch.from_numpy(nn).to(dev)
        out[f"S{S}_k{k}"] = merge_ms(gs, gd, gn, nq, k, torch)
    print(json.dumps({"merge_ms_per_batch_of_1024": out}))


if __name__ == "__main__":
    main()
