"""Spectral-matching baseline on the GPU.

``SM(corr, src_keypts, tgt_keypts, ...)`` mirrors
baseline_scripts/baseline_3DMatch.py:19-53 -- same inputs (``corr`` is the
loader's ``corr_pos`` [1,N,6]), same outputs ``(pred_trans [1,4,4],
pred_labels [1,N])`` -- with ``args.inlier_threshold`` passed as a keyword.
Runs on pointdsc_amd/csrc/sm.hip through the C ABI (pdsc_spectral_matching):
dense M built once, 10 matrix-vector power iterates (HBM/MALL-bound), top-10 %
selection and the weighted Kabsch of a9.  No CPU fallback.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import check
from .kernels import _dev, _p, _stream, _workspace


def SM(corr, src_keypts, tgt_keypts, inlier_threshold: float = 0.10, top_ratio: float = 0.1,
       num_iterations: int = 10, return_eig: bool = False):
    corr, src, tgt = _dev(corr, "corr"), _dev(src_keypts, "src_keypts"), _dev(tgt_keypts, "tgt_keypts")
    assert corr.shape[0] == 1, "SM: bs = 1 (baseline_3DMatch.py:48)"
    N = corr.shape[1]
    if corr.shape != (1, N, 6) or src.shape != (1, N, 3) or tgt.shape != (1, N, 3):
        raise ValueError(f"shapes {tuple(corr.shape)} {tuple(src.shape)} {tuple(tgt.shape)}")
    dev = corr.device
    L = _lib.load()
    nb = L.pdsc_spectral_matching_workspace_bytes(N)
    ws = _workspace(nb, dev)
    trans = torch.empty((1, 4, 4), dtype=torch.float32, device=dev)
    labels = torch.empty((1, N), dtype=torch.float32, device=dev)
    eig = torch.empty((1, N), dtype=torch.float32, device=dev)
    check(L.pdsc_spectral_matching(_p(corr), _p(src), _p(tgt), N, float(inlier_threshold), float(top_ratio),
                                   int(num_iterations), _p(trans), _p(labels), _p(eig), _p(ws), nb, _stream(dev)),
          "pdsc_spectral_matching")
    return (trans, labels, eig) if return_eig else (trans, labels)


def sm_matvec(M, v):
    """y = M v (one SM power-iteration product; M [N,N], v [N])."""
    M, v = _dev(M, "M"), _dev(v, "v")
    N = v.shape[0]
    y = torch.empty(N, dtype=torch.float32, device=v.device)
    check(_lib.load().pdsc_sm_matvec(_p(M), _p(v), N, _p(y), _stream(v.device)), "pdsc_sm_matvec")
    return y
