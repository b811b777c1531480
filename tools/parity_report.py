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

from conftest import fp32_envelope, golden_hparams, golden_names, golden_state_dict, load_golden  # noqa: E402


def _t(x, dev, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev, dtype)


def report(name, precision, dev):
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    g = load_golden(name)
    hp = golden_hparams(g)
    m = PointDSC(in_dim=hp["in_dim"], num_layers=hp["num_layers"], num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=hp["inlier_threshold"], sigma_d=float(g["sigma_d"]), k=40,
                 nms_radius=hp["nms_radius"], precision=precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in golden_state_dict(g).items()})
    m = m.to(dev).eval()
    corr, src, tgt = (_t(g[k][None], dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    cfg, packed = m.pdsc_config(), m.packed_weights()
    M = kernels.compat(src, tgt, m.sigma_spat)
    feat, normed, conf = kernels.encoder(cfg, packed, corr, M)
    e_f, e_c, f64, c64, _, r_f, r_c = fp32_envelope(g, golden_state_dict(g), dev, bulk=True)
    has_f = len(g["corr_features"]) > 0
    f_ref = g["corr_features"].astype(np.float64) if has_f else f64
    f = feat[0].double().cpu().numpy()
    n_ref = f_ref / np.maximum(np.linalg.norm(f_ref, axis=1, keepdims=True), 1e-12)
    out = {"name": name, "precision": precision, "N": int(len(f)),
           "feat_rel": float(np.abs(f - f_ref).max() / np.abs(f_ref).max()) if has_f else None,
           "logit_abs": float(np.abs(conf[0].double().cpu().numpy() - g["confidence"]).max()),
           "logit_range": [float(g["confidence"].min()), float(g["confidence"].max())],
           "normed_abs": float(np.abs(normed[0].double().cpu().numpy() - n_ref).max()) if has_f else None}
    mx = np.abs(f64).max()
    out["ref_vs_fp64_feat"] = float(np.abs(f_ref - f64).max() / mx) if has_f else None
    out["ours_vs_fp64_feat"] = float(np.abs(f - f64).max() / mx)
    out["ref_vs_fp64_logit"] = float(np.abs(g["confidence"] - c64).max())
    out["ours_vs_fp64_logit"] = float(np.abs(conf[0].double().cpu().numpy() - c64).max())
    out["fp32_noise_feat"], out["fp32_noise_logit"] = float(e_f), float(e_c)
    # bulk (RMS) error against the largest RMS of the fp32 realisations
    from conftest import rms
    out["rms_ratio_feat"] = float(rms(f - f64) / mx / r_f) if r_f > 0 else None
    out["rms_ratio_logit"] = float(rms(conf[0].double().cpu().numpy() - c64) / r_c) if r_c > 0 else None
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
    if precision == "h3":  # the same inputs through the exact-fp32 contractions
        cfg32, packed32 = m.pdsc_config("f32"), m.packed_weights("f32")
        T32, L32, c32, _ = kernels.forward_testing(cfg32, packed32, corr, src, tgt, debug=True)
        out["h3_vs_f32_logit"] = float((conf2[0].double() - c32[0].double()).abs().max())
        out["h3_vs_f32_pose"] = float((trans[0] - T32[0]).abs().max())
        out["h3_vs_f32_labels"] = int((labels[0] != L32[0]).sum())
        out["f32_trans_abs"] = float(np.abs(T32[0].cpu().numpy() - g["final_trans"]).max())
    if not has_f:
        return out
    # stage-isolated NSM chain on the reference's own normed / seeds
    normed_ref = _t(n_ref.astype(np.float32), dev)[None]
    sd = golden_state_dict(g)
    k = g["knn_idx"].shape[1]
    knn = kernels.seed_knn(normed_ref, _t(g["seeds"][None], dev, torch.int32), k, precision=precision)[0].cpu().numpy()
    out["knn_rows_diff"] = int(sum(set(a.tolist()) != set(b.tolist()) for a, b in zip(knn, g["knn_idx"])))
    out["knn_order_diff"] = int((knn != g["knn_idx"]).any(1).sum())
    w, _ = kernels.nsm_weights(normed_ref, src, tgt, _t(g["knn_idx"][None], dev, torch.int32), 10,
                               _t(sd["sigma"], dev), _t(sd["sigma_spat"], dev), precision=precision)
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
