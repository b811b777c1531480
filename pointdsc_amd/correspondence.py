"""Correspondence construction on the GPU: the step that
turns per-point descriptors into the forward's inputs.

Restates the tail of ``ThreeDMatchTestset.__getitem__``
(datasets/ThreeDMatch.py:277-308; the KITTI loader repeats it at
datasets/KITTI.py:85-99) and the matching block of demo_registration.py:101-108:

    distance = np.sqrt(2 - 2 * (src_desc @ tgt_desc.T) + 1e-6)
    source_idx = np.argmin(distance, axis=1)
    mutual: target_idx = np.argmin(distance, axis=0); keep i with target_idx[source_idx[i]] == i
    labels = |transform(src, gt_trans) - tgt| < inlier_threshold
    corr_pos = concat(src, tgt) - mean            (in_dim = 6)

on hand-written HIP kernels (``pointdsc_amd/csrc/corr.hip``): the Ns x Nt
distance matrix is reduced tile by tile and never written.  Keypoint
subsampling (``num_node``, host RNG) and descriptor extraction / FPFH
normalisation happen upstream and are not part of this call.  No CPU fallback.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import check
from .kernels import _dev, _p, _stream, _workspace


def mutual_nn(src_desc: torch.Tensor, tgt_desc: torch.Tensor):
    """(source_idx [Ns], target_idx [Nt]) int32: row / column argmin of the
    descriptor distance, first index on ties (numpy.argmin)."""
    a, b = _dev(src_desc, "src_desc"), _dev(tgt_desc, "tgt_desc")
    (Ns, D), Nt = a.shape, b.shape[0]
    if b.shape[1] != D:
        raise ValueError(f"descriptor widths differ: {D} vs {b.shape[1]}")
    L = _lib.load()
    nb = L.pdsc_mutual_nn_workspace_bytes(Ns, Nt)
    ws = _workspace(nb, a.device)
    si = torch.empty(Ns, dtype=torch.int32, device=a.device)
    ti = torch.empty(Nt, dtype=torch.int32, device=a.device)
    check(L.pdsc_mutual_nn(_p(a), _p(b), Ns, Nt, D, _p(si), _p(ti), _p(ws), nb, _stream(a.device)),
          "pdsc_mutual_nn")
    return si, ti


def build_correspondences(src_keypts: torch.Tensor, tgt_keypts: torch.Tensor, src_desc: torch.Tensor,
                          tgt_desc: torch.Tensor, use_mutual: bool = True, gt_trans=None,
                          inlier_threshold: float = 0.10):
    """The forward's inputs for one scan pair, as the reference's test loaders build them.

    src_keypts [Ns,3], tgt_keypts [Nt,3], src_desc [Ns,D], tgt_desc [Nt,D]: fp32
    device tensors (the already-selected keypoints and their descriptors).
    gt_trans: optional [4,4] (any float dtype; used in float64, as the loader's
    float64 ground truth).  Returns a dict with ``corr`` [n,2] int64,
    ``corr_pos`` [n,6], ``src_keypts`` / ``tgt_keypts`` [n,3] fp32 and, with
    gt_trans, ``labels`` [n] fp32 -- the loader's outputs
    (datasets/ThreeDMatch.py:328-332) before batching."""
    sk, tk = _dev(src_keypts, "src_keypts"), _dev(tgt_keypts, "tgt_keypts")
    a, b = _dev(src_desc, "src_desc"), _dev(tgt_desc, "tgt_desc")
    (Ns, D), Nt = a.shape, b.shape[0]
    if sk.shape != (Ns, 3) or tk.shape != (Nt, 3) or b.shape[1] != D:
        raise ValueError(f"shapes: keypts {tuple(sk.shape)}/{tuple(tk.shape)}, desc {tuple(a.shape)}/{tuple(b.shape)}")
    dev = a.device
    gt = None
    if gt_trans is not None:
        gt = torch.as_tensor(gt_trans).to(device=dev, dtype=torch.float64).reshape(4, 4).contiguous()
    L = _lib.load()
    nb = L.pdsc_mutual_nn_workspace_bytes(Ns, Nt)
    ws = _workspace(nb, dev)
    corr = torch.empty((Ns, 2), dtype=torch.int32, device=dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    corr_pos = torch.empty((Ns, 6), dtype=torch.float32, device=dev)
    so = torch.empty((Ns, 3), dtype=torch.float32, device=dev)
    to = torch.empty((Ns, 3), dtype=torch.float32, device=dev)
    labels = torch.empty(Ns, dtype=torch.float32, device=dev) if gt is not None else None
    check(L.pdsc_build_correspondences(_p(a), _p(b), _p(sk), _p(tk), Ns, Nt, D, int(bool(use_mutual)), _p(gt),
                                       float(inlier_threshold), _p(corr), _p(count), _p(corr_pos), _p(so), _p(to),
                                       _p(labels), _p(ws), nb, _stream(dev)), "pdsc_build_correspondences")
    n = int(count.item())
    out = {"corr": corr[:n].long(), "corr_pos": corr_pos[:n], "src_keypts": so[:n], "tgt_keypts": to[:n]}
    if labels is not None:
        out["labels"] = labels[:n]
    return out
