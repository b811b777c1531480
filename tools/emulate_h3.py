"""Numerics check of the 3xf16 product split (attention_h3.hpp) on the CPU.

Runs the oracle's encoder (oracle/pdsc_oracle.py) on the golden cases with
Q K^T and/or P V replaced by an emulation of the kernel's arithmetic --
operands split into fp16 hi + lo, products hi.hi + hi.lo + lo.hi -- and
reports the feature / confidence error against the reference's golden
outputs, next to plain fp32.  Usage: python tools/emulate_h3.py [qk|pv|both|none] [P prescale]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import golden_state_dict, load_golden  # noqa: E402
from oracle import pdsc_oracle as O  # noqa: E402

f32, f16 = np.float32, np.float16


def split(x):
    hi = x.astype(f16)
    return hi, (x - hi.astype(f32)).astype(f16)


def mm3(a, b):
    ah, al = split(a)
    bh, bl = split(b)
    d = lambda x: x.astype(np.float64)  # noqa: E731  (fp16 products are exact in fp64)
    return (d(ah) @ d(bh) + d(ah) @ d(bl) + d(al) @ d(bh)).astype(f32)


def make_block(mode, pscale):
    def nlb(feat, M, sd, p, C):
        Q = O._conv(feat, sd, p + ".projection_q")
        K = O._conv(feat, sd, p + ".projection_k")
        V = O._conv(feat, sd, p + ".projection_v")
        S = (mm3(Q, K.T) if mode in ("qk", "both") else Q @ K.T).astype(f32) / f32(C ** 0.5)
        lg = (M * S).astype(f32)
        e = np.exp(lg - lg.max(-1, keepdims=True)).astype(f32)  # p <= 1, prescaled like the kernel
        msg = (mm3(e * f32(pscale), V) / f32(pscale) if mode in ("pv", "both") else e @ V)
        msg = (msg / e.sum(-1, keepdims=True)).astype(f32)
        h = O._relu(O._bn(O._conv(msg, sd, p + ".fc_message.0"), sd, p + ".fc_message.1"))
        h = O._relu(O._bn(O._conv(h, sd, p + ".fc_message.3"), sd, p + ".fc_message.4"))
        return (feat + O._conv(h, sd, p + ".fc_message.6")).astype(f32)
    return nlb


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "both"
    pscale = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0 ** 15
    O.nonlocal_block = make_block(mode, pscale)
    for name in ["rel_1k", "rel_1k_kitti", "rel_5k_lo"]:
        g = load_golden(name)
        sd = golden_state_dict(g)
        M = O.compat(g["src_keypts"], g["tgt_keypts"], float(f32(g["sigma_d"])))
        f = O.encoder(g["corr_pos"], M, sd, int(g["num_layers"]))
        ref = g["corr_features"]
        print(f"{mode:5s} {name:13s} max|df|/max|f| {abs(f - ref).max() / abs(ref).max():.2e}  "
              f"max|dconf| {abs(O.classify(f, sd) - g['confidence']).max():.2e}")


if __name__ == "__main__":
    main()
