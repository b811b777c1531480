#!/usr/bin/env python3
"""Measured HIP-path error against every golden case (run on the GPU box).

Prints one JSON object per golden with the quantities the parity tests bound:
feature error relative to max|f|, logit / normed absolute error, seed-list
positions that differ (and the reference score gap of each swap), kNN rows
that differ, NSM weight error, pose error and label mismatches, for each
precision mode the library offers.  Test infrastructure, not product.

Usage:  python tools/parity_report.py [--precision h3|f32|both] [names...]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import golden_hparams, golden_names, golden_state_dict, load_golden  # noqa: E402


def _t(x, dev, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev, dtype)


def encoder64(g, sd, dev):
    """Exact-arithmetic (torch fp64) restatement of models/PointDSC.py:65-77, :156, :171
    on the bit-exact fp32 M: the yardstick both fp32 implementations are measured against."""
    from pointdsc_amd import kernels
    W = {k: torch.as_tensor(np.asarray(v)).to(dev).double() for k, v in sd.items() if np.asarray(v).dtype != np.int64}

    def conv(x, n):
        return x @ W[n + ".weight"][:, :, 0].T + W[n + ".bias"]

    def bn(x, n):
        a = W[n + ".weight"] / torch.sqrt(W[n + ".running_var"] + 1e-5)
        return x * a + (W[n + ".bias"] - W[n + ".running_mean"] * a)

    src, tgt = (_t(g[k][None], dev) for k in ("src_keypts", "tgt_keypts"))
    M = kernels.compat(src, tgt, torch.tensor([float(np.float32(g["sigma_d"]))], device=dev))[0].double()
    f = conv(_t(g["corr_pos"], dev).double(), "encoder.layer0")
    for i in range(int(g["num_layers"])):
        p = f"encoder.blocks.PointCN_layer_{i}"
        f = torch.relu(bn(conv(f, p + ".0"), p + ".1"))
        p = f"encoder.blocks.NonLocal_layer_{i}"
        q, k, v = (conv(f, f"{p}.projection_{c}") for c in "qkv")
        A = torch.softmax(M * (q @ k.T) / 128 ** 0.5, -1)
        h = torch.relu(bn(conv(A @ v, p + ".fc_message.0"), p + ".fc_message.1"))
        h = torch.relu(bn(conv(h, p + ".fc_message.3"), p + ".fc_message.4"))
        f = f + conv(h, p + ".fc_message.6")
    h = torch.relu(conv(f, "classification.0"))
    h = torch.relu(conv(h, "classification.2"))
    return f.cpu().numpy(), conv(h, "classification.4")[:, 0].cpu().numpy()


def report(name, precision, dev):
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    g = load_golden(name)
    hp = golden_hparams(g)
    m = PointDSC(in_dim=6, num_layers=hp["num_layers"], num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=hp["inlier_threshold"], sigma_d=float(g["sigma_d"]), k=40,
                 nms_radius=hp["nms_radius"], **({} if precision == "h3" else {"precision": precision}))
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in golden_state_dict(g).items()})
    m = m.to(dev).eval()
    corr, src, tgt = (_t(g[k][None], dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    cfg, packed = m.pdsc_config(), m.packed_weights()
    M = kernels.compat(src, tgt, m.sigma_spat)
    feat, normed, conf = kernels.encoder(cfg, packed, corr, M)
    f_ref = g["corr_features"].astype(np.float64)
    f = feat[0].double().cpu().numpy()
    n_ref = f_ref / np.maximum(np.linalg.norm(f_ref, axis=1, keepdims=True), 1e-12)
    out = {"name": name, "precision": precision, "N": int(len(f_ref)),
           "feat_rel": float(np.abs(f - f_ref).max() / np.abs(f_ref).max()),
           "logit_abs": float(np.abs(conf[0].double().cpu().numpy() - g["confidence"]).max()),
           "logit_range": [float(g["confidence"].min()), float(g["confidence"].max())],
           "normed_abs": float(np.abs(normed[0].double().cpu().numpy() - n_ref).max())}
    f64, c64 = encoder64(g, golden_state_dict(g), dev)
    mx = np.abs(f64).max()
    out["ref_vs_fp64_feat"] = float(np.abs(f_ref - f64).max() / mx)
    out["ours_vs_fp64_feat"] = float(np.abs(f - f64).max() / mx)
    out["ref_vs_fp64_logit"] = float(np.abs(g["confidence"] - c64).max())
    out["ours_vs_fp64_logit"] = float(np.abs(conf[0].double().cpu().numpy() - c64).max())
    from oracle import pdsc_oracle as O
    lm_o = O.local_max(g["src_keypts"], conf[0].cpu().numpy(), float(g["nms_radius"]))
    out["lm_mismatch"] = int((lm_o != g["is_local_max"]).sum())
    trans, labels, conf2, seeds = kernels.forward_testing(cfg, packed, corr, src, tgt, debug=True)
    score = g["confidence"] * g["is_local_max"]
    s_ours, s_ref = seeds[0].cpu().numpy().astype(np.int64), g["seeds"]
    diff = np.nonzero(s_ours != s_ref)[0]
    out["seed_pos_diff"] = int(len(diff))
    out["seed_swap_gaps"] = [float(abs(score[s_ours[i]] - score[s_ref[i]])) for i in diff[:10]]
    out["seed_set_diff"] = int(len(set(s_ours.tolist()) ^ set(s_ref.tolist())))
    out["seed_min_gap_ref"] = float(g["seed_score_min_gap"])
    out["trans_abs"] = float(np.abs(trans[0].cpu().numpy() - g["final_trans"]).max())
    out["label_mismatch"] = int((labels[0].cpu().numpy() != g["final_labels"]).sum())
    # stage-isolated NSM chain on the reference's own normed / seeds
    normed_ref = _t(n_ref.astype(np.float32), dev)[None]
    sd = golden_state_dict(g)
    k = g["knn_idx"].shape[1]
    knn = kernels.seed_knn(normed_ref, _t(g["seeds"][None], dev, torch.int32), k)[0].cpu().numpy()
    out["knn_rows_diff"] = int(sum(set(a.tolist()) != set(b.tolist()) for a, b in zip(knn, g["knn_idx"])))
    out["knn_order_diff"] = int((knn != g["knn_idx"]).any(1).sum())
    w, _ = kernels.nsm_weights(normed_ref, src, tgt, _t(g["knn_idx"][None], dev, torch.int32), 10,
                               _t(sd["sigma"], dev), _t(sd["sigma_spat"], dev))
    v = g["leading_eig"]
    out["nsm_w_abs"] = float(np.abs(w[0].cpu().numpy() - v / (v.sum(-1, keepdims=True) + 1e-6)).max())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="both", choices=["h3", "f32", "both"])
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    precs = ["h3", "f32"] if a.precision == "both" else [a.precision]
    for name in a.names or golden_names():
        for p in precs:
            print(json.dumps(report(name, p, dev)), flush=True)


if __name__ == "__main__":
    main()
