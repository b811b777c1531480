#!/usr/bin/env python3
"""Seed kNN timing (pdsc_seed_knn: split copy + knn_dist + knn_select) on random
unit features at a few shapes, for A/B of library variants (PDSC_LIB_VARIANT).
Usage: python tools/knn_bench.py [--iters 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from pointdsc_amd import kernels
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(5)
    res = {}
    shapes = ((128, 1000), (128, 1289), (8, 5000), (8, 5003), (1, 1000), (1, 5000))
    if os.environ.get("AB_SHAPES"):
        shapes = [tuple(int(v) for v in x.split("x")) for x in os.environ["AB_SHAPES"].split(",")]
    for B, N in shapes:
        S = int(0.1 * N)
        f = torch.randn((B, N, 128), generator=g)
        f = (f / f.norm(dim=-1, keepdim=True)).to(dev)
        seeds = torch.stack([torch.randperm(N, generator=g)[:S] for _ in range(B)]).to(torch.int32).to(dev)
        for _ in range(3):
            kernels.seed_knn(f, seeds, 40)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            kernels.seed_knn(f, seeds, 40)
        e1.record()
        torch.cuda.synchronize()
        res[f"{B}x{N}"] = round(e0.elapsed_time(e1) / a.iters * 1e3, 1)
    print(json.dumps({"variant": os.environ.get("PDSC_LIB_VARIANT", ""), "us_per_call": res}))


if __name__ == "__main__":
    main()
