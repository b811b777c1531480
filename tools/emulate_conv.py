"""CPU emulation of the 1x1-convolution arithmetic of the 3xfp16 mode (diagnostic).

The encoder in fp64 (tools/emulate_attn.py's restatement) with every Conv1d
evaluated as the kernels do -- activations split x = xh + xl (fp16), weights
scaled by 2^s and split into fp16 planes -- and the attention as the h3 kernel
does it (emulate_attn.attention_h3, one key split).  Modes:
  w3  three weight planes (hi + mid + lo: every fp32 weight exactly), 4 products
      wh.xh + wh.xl + wm.xh + wl.xh (the shipped kernels)
  w2  two weight planes (hi + mid: 22 bits), 3 products wh.xh + wh.xl + wm.xh
  f32 plain fp32 products
Prints the feature / logit error against exact arithmetic, max and RMS.
Usage: python tools/emulate_conv.py [golden ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
from emulate_attn import attention_h3  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from conftest import golden_state_dict, load_golden  # noqa: E402

F32, F16, F64 = np.float32, np.float16, np.float64


def split2(x):
    hi = x.astype(F16)
    return hi.astype(F64), (x.astype(F32) - hi.astype(F32)).astype(F16).astype(F64)


def weight_planes(w, n):
    """w [out, in] fp32 -> n fp16 planes of w * 2^s (exact sums for n = 3), and 2^-s."""
    w = w.astype(F32)
    m = float(np.abs(w).max())
    s = 0 if m == 0 else 14 - int(np.frexp(np.float32(m))[1])  # largest |w 2^s| just below 2^14
    ws = (w.astype(F64) * 2.0 ** s).astype(F32)
    planes, r = [], ws.astype(F64)
    for _ in range(n):
        p = r.astype(F32).astype(F16)
        planes.append(p.astype(F64))
        r = r - p.astype(F64)
    return planes, 2.0 ** -s


def conv_mode(mode):
    def conv(x, W, b):
        x = x.astype(F32)
        if mode == "f32":
            return (x @ W.astype(F32).T + b.astype(F32)).astype(F32).astype(F64)
        xh, xl = split2(x)
        if mode == "w3":
            (wh, wm, wl), inv = weight_planes(W, 3)
            acc = xh @ wh.T + xl @ wh.T + xh @ wm.T + xh @ wl.T
        else:
            (wh, wm), inv = weight_planes(W, 2)
            acc = xh @ wh.T + xl @ wh.T + xh @ wm.T
        return (acc.astype(F32) * F32(inv) + b.astype(F32)).astype(F32).astype(F64)
    return conv


def encoder(g, sd, conv=None, att=None):
    from oracle import pdsc_oracle as O
    W = {k: np.asarray(v, F64) for k, v in sd.items() if np.asarray(v).dtype != np.int64}
    cv = (lambda x, n: x @ W[n + ".weight"][:, :, 0].T + W[n + ".bias"]) if conv is None else \
        (lambda x, n: conv(x, W[n + ".weight"][:, :, 0], W[n + ".bias"]))

    def bn(x, n):
        a = W[n + ".weight"] / np.sqrt(W[n + ".running_var"] + 1e-5)
        return x * a + (W[n + ".bias"] - W[n + ".running_mean"] * a)

    M = O.compat(g["src_keypts"], g["tgt_keypts"], float(np.float32(g["sigma_d"]))).astype(F64)
    f = np.asarray(g["corr_pos"], F64) @ W["encoder.layer0.weight"][:, :, 0].T + W["encoder.layer0.bias"]
    for i in range(int(g["num_layers"])):
        p = f"encoder.blocks.PointCN_layer_{i}"
        f = np.maximum(bn(cv(f, p + ".0"), p + ".1"), 0)
        p = f"encoder.blocks.NonLocal_layer_{i}"
        q, k, v = (cv(f, f"{p}.projection_{c}") for c in "qkv")
        if att is None:
            x = M * (q @ k.T) / np.sqrt(128)
            A = np.exp(x - x.max(1, keepdims=True))
            msg = (A / A.sum(1, keepdims=True)) @ v
        else:
            msg = att(q, k, v, M).astype(F64)
        h = np.maximum(bn(cv(msg, p + ".fc_message.0"), p + ".fc_message.1"), 0)
        h = np.maximum(bn(cv(h, p + ".fc_message.3"), p + ".fc_message.4"), 0)
        f = f + cv(h, p + ".fc_message.6")
    h = np.maximum(cv(f, "classification.0"), 0)
    h = np.maximum(cv(h, "classification.2"), 0)
    return f, cv(h, "classification.4")[:, 0]


def main():
    names = sys.argv[1:] or ["rel_1k", "degen_1k", "rel_1k_kitti", "wide9_1k"]
    att = lambda q, k, v, M: attention_h3(q, k, v, M, 1, {"vk": 5})  # noqa: E731
    for name in names:
        g = load_golden(name)
        sd = golden_state_dict(g)
        f64, c64 = encoder(g, sd)
        mx = np.abs(f64).max()
        ref_f = np.abs(g["corr_features"] - f64).max() / mx if len(g["corr_features"]) else float("nan")
        print(f"{name}: reference fp32 feature err {ref_f:.3g}, logit err {np.abs(g['confidence'] - c64).max():.3g}")
        for mode in ("f32", "w3", "w2"):
            f, c = encoder(g, sd, conv_mode(mode), att)
            df, dc = f - f64, c - c64
            print(f"  {mode}: feature max {np.abs(df).max() / mx:.3g} rms {np.sqrt(np.mean(df ** 2)) / mx:.3g}  "
                  f"logit max {np.abs(dc).max():.3g} rms {np.sqrt(np.mean(dc ** 2)):.3g}", flush=True)


if __name__ == "__main__":
    main()
