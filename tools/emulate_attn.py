"""CPU emulation of the h3 attention's online softmax (attention_h3.hpp: 32-key
tiles, p = 2^(x - m + PSHIFT - e) split into fp16 hi / lo, lazy re-base by
DEFER, V tiles pre-scaled by 2^e, key splits combined as the combine kernel
does) inside the fp64 encoder of a golden, to see which part of the arithmetic
sets the error against exact math for long key chains (nsplit = 1) against
short ones.  Diagnostic only: python tools/emulate_attn.py wide9_1k [VEXP_TARGET ...]
(no targets: the arithmetic ablations; r04 finding: the V-tile scale target
14 -> 5 takes nsplit-1 feature errors from up to 1.3e-4 to <= 5.6e-6)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from conftest import golden_state_dict, load_golden  # noqa: E402

F32, F16 = np.float32, np.float16
PSHIFT, DEFER, VEXP_MAX = 7, 8.0, 8
QSCALE = F32(np.log2(np.e) / np.sqrt(128))


def split(x):
    hi = x.astype(F16)
    lo = (x - hi.astype(F32)).astype(F16)
    return hi.astype(F32), lo.astype(F32)


def mm3(a, b):  # a [n,k] @ b [k,m] from hi / lo pairs, fp32 accumulation (lo.lo dropped)
    ah, al = split(a.astype(F32))
    bh, bl = split(b.astype(F32))
    return (ah @ bh + ah @ bl + al @ bh).astype(F32)


def vexp(vmax, target=14):
    """attention_h3.hpp h3_vexp: the largest e <= VEXP_MAX with vmax 2^e < 2^target"""
    if not (vmax > 0) or not (vmax < 8192):
        return 0
    _, ex = np.frexp(np.float32(vmax))
    return max(0, min(VEXP_MAX, target - int(ex)))


def attention_h3(q, k, v, M, nsplit, opt):
    N = q.shape[0]
    nt = (N + 31) // 32
    sps = (nt + nsplit - 1) // nsplit
    qs = (q.astype(F32) * QSCALE).astype(F32)
    parts = []
    for s0 in range(0, nt, sps):
        m_run = np.full(N, -np.inf, F32)
        l_run = np.zeros(N, F32)
        O = np.zeros((N, v.shape[1]), F32)
        for t in range(s0, min(nt, s0 + sps)):
            ks = slice(32 * t, min(N, 32 * t + 32))
            vt = v[ks].astype(F32)
            e = 0 if opt.get("novexp") else vexp(np.abs(vt).max(), opt.get("vk", 14))
            S = mm3(qs, k[ks].T) if not opt.get("exactS") else (qs.astype(np.float64) @ k[ks].T.astype(np.float64)).astype(F32)
            x = (M[:, ks].astype(F32) * S).astype(F32)  # logits, log2 units
            mx = x.max(1)
            grp = mx.reshape(-1, 32) if N % 32 == 0 else None
            if t == s0:
                need = mx > m_run + DEFER
            else:
                need = mx > m_run + DEFER
            if opt.get("eager"):
                need = mx > m_run
            # wave-uniform (32 queries): any lane -> every lane of the wave re-bases
            if grp is not None and not opt.get("eager"):
                need = np.repeat(need.reshape(-1, 32).any(1), 32)
            m_new = np.where(need, np.maximum(m_run, mx), m_run)
            alpha = np.exp2(m_run - m_new).astype(F32)
            alpha[np.isnan(alpha)] = 0
            O *= alpha[:, None]
            l_run *= alpha
            m_run = m_new
            p = (x - (m_run - PSHIFT + e)[:, None]).astype(F32)
            P = np.exp2(p).astype(F32)
            if opt.get("exactP"):
                Vs = (vt * F32(2.0 ** e)).astype(F32)
                O += (P @ Vs).astype(F32)
            else:
                Ph, Pl = split(P)
                Vh, Vl = split((vt * F32(2.0 ** e)).astype(F32))
                O += (Ph @ Vh + Ph @ Vl + Pl @ Vh).astype(F32)
            l_run += (P.sum(1) * F32(2.0 ** e)).astype(F32)
        parts.append((O, l_run, ((m_run - PSHIFT) * np.log(2)).astype(F32)))
    m = np.max([p[2] for p in parts], 0)
    num = sum(p[0] * np.exp(p[2] - m)[:, None] for p in parts)
    den = sum(p[1] * np.exp(p[2] - m) for p in parts)
    return (num / den[:, None]).astype(F32)


def encoder(g, sd, att=None):
    from oracle import pdsc_oracle as O
    W = {k: np.asarray(v, np.float64) for k, v in sd.items() if np.asarray(v).dtype != np.int64}
    conv = lambda x, n: x @ W[n + ".weight"][:, :, 0].T + W[n + ".bias"]

    def bn(x, n):
        a = W[n + ".weight"] / np.sqrt(W[n + ".running_var"] + 1e-5)
        return x * a + (W[n + ".bias"] - W[n + ".running_mean"] * a)

    M = O.compat(g["src_keypts"], g["tgt_keypts"], float(np.float32(g["sigma_d"]))).astype(np.float64)
    f = conv(np.asarray(g["corr_pos"], np.float64), "encoder.layer0")
    for i in range(int(g["num_layers"])):
        p = f"encoder.blocks.PointCN_layer_{i}"
        f = np.maximum(bn(conv(f, p + ".0"), p + ".1"), 0)
        p = f"encoder.blocks.NonLocal_layer_{i}"
        q, k, v = (conv(f, f"{p}.projection_{c}") for c in "qkv")
        if att is None:
            x = M * (q @ k.T) / np.sqrt(128)
            A = np.exp(x - x.max(1, keepdims=True))
            msg = (A / A.sum(1, keepdims=True)) @ v
        else:
            msg = att(q, k, v, M).astype(np.float64)
        h = np.maximum(bn(conv(msg, p + ".fc_message.0"), p + ".fc_message.1"), 0)
        h = np.maximum(bn(conv(h, p + ".fc_message.3"), p + ".fc_message.4"), 0)
        f = f + conv(h, p + ".fc_message.6")
    return f


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "wide9_1k"
    g = load_golden(name)
    sd = golden_state_dict(g)
    f64 = encoder(g, sd)
    mx = np.abs(f64).max()
    print(f"{name}: reference fp32 feature err {np.abs(g['corr_features'] - f64).max() / mx:.3g}")
    opts = [{"vk": int(a)} for a in sys.argv[2:]] or [{}, {"exactP": 1}, {"novexp": 1}, {"exactS": 1}, {"eager": 1}]
    for opt in opts:
        for ns in (1, 32):
            f = encoder(g, sd, lambda q, k, v, M: attention_h3(q, k, v, M, ns, opt))
            print(f"  opt {opt} nsplit {ns:2d}: feature err {np.abs(f - f64).max() / mx:.3g}", flush=True)


if __name__ == "__main__":
    main()
