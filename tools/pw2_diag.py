#!/usr/bin/env python3
"""Per-depth encoder error of the HIP path (diagnostics): the network truncated to
l = 1..L layers, HIP features vs exact (fp64) arithmetic.
Usage: PDSC_PW2=<mode> python tools/pw2_diag.py <golden> <out.npz>   (HIP runs)
       python tools/pw2_diag.py <golden> --compare a.npz b.npz ...     (fp64 report)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import encoder_torch, golden_hparams, golden_state_dict, load_golden  # noqa: E402


# (layers, parameters zeroed): isolate the stages of the 2-layer network
VARIANTS = {
    "L2_no_msg1": (2, ["encoder.blocks.NonLocal_layer_1.fc_message.6"]),
    "L2_no_msg0_msg1": (2, ["encoder.blocks.NonLocal_layer_0.fc_message.6",
                            "encoder.blocks.NonLocal_layer_1.fc_message.6"]),
    "L2_no_msg0": (2, ["encoder.blocks.NonLocal_layer_0.fc_message.6"]),
    # PointCN_1 = ReLU(+-identity): the network's output is relu(+-y), y = the residual sum mid computes
    "L2_y_pos": (2, ["encoder.blocks.NonLocal_layer_1.fc_message.6", "pcn1_identity+"]),
    "L2_y_neg": (2, ["encoder.blocks.NonLocal_layer_1.fc_message.6", "pcn1_identity-"]),
}


def variant_sd(sd, zero):
    out = dict(sd)
    for z in zero:
        if z.startswith("pcn1_identity"):
            p = "encoder.blocks.PointCN_layer_1"
            sgn = 1.0 if z.endswith("+") else -1.0
            out[p + ".0.weight"] = (sgn * np.eye(128, dtype=np.float32))[:, :, None]
            out[p + ".0.bias"] = np.zeros(128, np.float32)
            out[p + ".1.weight"] = np.ones(128, np.float32)
            out[p + ".1.bias"] = np.zeros(128, np.float32)
            out[p + ".1.running_mean"] = np.zeros(128, np.float32)
            out[p + ".1.running_var"] = np.full(128, 1.0 - 1e-5, np.float32)
            continue
        for k in (z + ".weight", z + ".bias"):
            out[k] = np.zeros_like(np.asarray(sd[k]))
    return out


def configs(g):
    hp = golden_hparams(g)
    for l in range(1, hp["num_layers"] + 1):
        yield str(l), l, []
    for k, (l, zero) in VARIANTS.items():
        yield k, l, zero


def run(name, out):
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    g = load_golden(name)
    hp = golden_hparams(g)
    dev = torch.device("cuda:0")
    sd0 = golden_state_dict(g)
    corr, src, tgt = (torch.from_numpy(g[k][None]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    res = {}
    for key, l, zero in configs(g):
        sd = {k: torch.from_numpy(np.asarray(v)) for k, v in variant_sd(sd0, zero).items()}
        m = PointDSC(num_layers=l, inlier_threshold=hp["inlier_threshold"], sigma_d=float(g["sigma_d"]),
                     nms_radius=hp["nms_radius"])
        m.load_state_dict(sd, strict=False)
        m = m.to(dev).eval()
        M = kernels.compat(src, tgt, m.sigma_spat)
        feat, _, conf = kernels.encoder(m.pdsc_config(), m.packed_weights(), corr, M)
        res[f"f{key}"], res[f"c{key}"] = feat[0].cpu().numpy(), conf[0].cpu().numpy()
    np.savez(out, **res)


def compare(name, files):
    g = load_golden(name)
    sd0 = golden_state_dict(g)
    runs = [np.load(f) for f in files]
    dev = torch.device("cuda:0") if torch.cuda.is_available() else torch.device("cpu")
    for key, l, zero in configs(g):
        gl = dict(g)
        gl["num_layers"] = l
        sd = variant_sd(sd0, zero)
        f64, c64 = encoder_torch(gl, sd, dev)
        f32, c32 = encoder_torch(gl, sd, dev, torch.float32, seed=0)
        mx = np.abs(f64).max()
        row = {"case": key, "fp32_f": float(np.abs(f32 - f64).max() / mx), "fp32_c": float(np.abs(c32 - c64).max())}
        for f, r in zip(files, runs):
            d = np.abs(r[f"f{key}"] - f64).max(-1) / mx
            row[os.path.basename(f) + "_f"] = float(d.max())
            row[os.path.basename(f) + "_argmax"] = int(d.argmax())
            row[os.path.basename(f) + "_c"] = float(np.abs(r[f"c{key}"] - c64).max())
            if key.startswith("L2_y"):
                i = int(d.argmax())
                ch = np.argsort(-np.abs(r[f"f{key}"][i] - f64[i]))[:6]
                row[os.path.basename(f) + "_worst"] = [[int(c), float(f64[i, c]), float(r[f"f{key}"][i, c] - f64[i, c])]
                                                      for c in ch]
        print(json.dumps(row))


if __name__ == "__main__":
    if sys.argv[2] == "--compare":
        compare(sys.argv[1], sys.argv[3:])
    else:
        run(sys.argv[1], sys.argv[2])
