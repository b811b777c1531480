"""Drop-in ``models.PointDSC`` for MI355X: same classes, constructor, state_dict
keys and ``forward(data)`` contract as the reference (models/PointDSC.py:9-438
of AmnonDrory/PointDSC), with the testing-mode forward executed by the
hand-written gfx950 kernels of ``libpdsc.so``.

Usage from the reference's drivers (evaluation/test_3DMatch.py:215-225,
demo_registration.py:78-88, evaluation/test_KITTI.py:280-293)::

    from pointdsc_amd.PointDSC import PointDSC          # instead of models.PointDSC
    model = PointDSC(in_dim=6, num_layers=12, ...)
    model.load_state_dict(torch.load(ckpt), strict=False)
    model = model.cuda().eval()
    res = model({'corr_pos': ..., 'src_keypts': ..., 'tgt_keypts': ..., 'testing': True})

Scope: the testing path (``'testing' in data``) and the training branch's
evaluation-mode forward (no 'testing' key under ``model.eval()``: the
validation loop of libs/trainer.py:202-239 -- final_trans, the logits as
final_labels, and the N x N feature-similarity M its SpectralMatchingLoss
consumes).  Training proper (BatchNorm batch statistics in ``model.train()``,
autograd through the encoder and the SVD) is out of scope and raises
``NotImplementedError``; the sub-modules exist only to hold the reference's
parameters (their own ``forward`` raises as well) -- the encoder runs fused
inside the kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib, kernels


class NonLocalBlock(nn.Module):
    """Parameter holder with the reference's layout (models/PointDSC.py:9-25)."""

    def __init__(self, num_channels=128, num_heads=1):
        super().__init__()
        half = num_channels // 2
        self.fc_message = nn.Sequential(
            nn.Conv1d(num_channels, half, kernel_size=1), nn.BatchNorm1d(half), nn.ReLU(inplace=True),
            nn.Conv1d(half, half, kernel_size=1), nn.BatchNorm1d(half), nn.ReLU(inplace=True),
            nn.Conv1d(half, num_channels, kernel_size=1),
        )
        self.projection_q = nn.Conv1d(num_channels, num_channels, kernel_size=1)
        self.projection_k = nn.Conv1d(num_channels, num_channels, kernel_size=1)
        self.projection_v = nn.Conv1d(num_channels, num_channels, kernel_size=1)
        self.num_channels = num_channels
        self.head = num_heads

    def forward(self, feat, attention):
        raise NotImplementedError("NonLocalBlock runs fused inside PointDSC.forward on the HIP path "
                                  "(or pointdsc_amd.kernels.attention for the attention core)")


class NonLocalNet(nn.Module):
    """Parameter holder with the reference's layout (models/PointDSC.py:48-63)."""

    def __init__(self, in_dim=6, num_layers=6, num_channels=128):
        super().__init__()
        self.num_layers = num_layers
        self.blocks = nn.ModuleDict()
        self.layer0 = nn.Conv1d(in_dim, num_channels, kernel_size=1, bias=True)
        for i in range(num_layers):
            self.blocks[f"PointCN_layer_{i}"] = nn.Sequential(
                nn.Conv1d(num_channels, num_channels, kernel_size=1, bias=True),
                nn.BatchNorm1d(num_channels), nn.ReLU(inplace=True))
            self.blocks[f"NonLocal_layer_{i}"] = NonLocalBlock(num_channels)

    def forward(self, corr_feat, corr_compatibility):
        raise NotImplementedError("NonLocalNet runs fused inside PointDSC.forward on the HIP path "
                                  "(or pointdsc_amd.kernels.encoder)")


class PointDSC(nn.Module):
    """models/PointDSC.py:80-438 with the testing forward on libpdsc."""

    def __init__(self, in_dim=6, num_layers=6, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=0.10, sigma_d=0.10, k=40, nms_radius=0.10, precision="h3"):
        """The reference's constructor (models/PointDSC.py:81-121) plus ``precision``
        (not in the reference): 'h3' (default) runs the fp32 contractions as three
        fp16 MFMA products, 'f32' on exact fp32 MFMA (include/pdsc.h)."""
        super().__init__()
        _lib.precision_code(precision)
        self.precision = precision
        self.in_dim = in_dim
        self.num_layers = num_layers
        self.num_iterations = num_iterations
        self.ratio = ratio
        self.num_channels = num_channels
        self.inlier_threshold = inlier_threshold
        self.sigma = nn.Parameter(torch.Tensor([1.0]).float(), requires_grad=True)
        self.sigma_spat = nn.Parameter(torch.Tensor([sigma_d]).float(), requires_grad=False)
        self.k = k
        self.nms_radius = nms_radius
        self.encoder = NonLocalNet(in_dim=in_dim, num_layers=num_layers, num_channels=num_channels)
        self.classification = nn.Sequential(
            nn.Conv1d(num_channels, 32, kernel_size=1, bias=True), nn.ReLU(inplace=True),
            nn.Conv1d(32, 32, kernel_size=1, bias=True), nn.ReLU(inplace=True),
            nn.Conv1d(32, 1, kernel_size=1, bias=True),
        )
        for m in self.modules():  # the reference's initialisation (:115-121)
            if isinstance(m, (nn.Conv1d, nn.Linear)):
                nn.init.xavier_normal_(m.weight, gain=1)
            elif isinstance(m, nn.BatchNorm1d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        self._packed = None
        self._packed_key = None

    # ------------------------------------------------------------- internals
    def pdsc_config(self) -> _lib.PdscConfig:
        """Hyper-parameters as the C ABI's ``pdsc_config`` (read at call time,
        so attribute edits after construction are honoured like the reference)."""
        return _lib.make_config(self.in_dim, self.num_layers, self.num_channels, self.num_iterations,
                                self.k, self.ratio, self.inlier_threshold, self.nms_radius, self.precision)

    def packed_weights(self) -> torch.Tensor:
        """Kernel-layout weights, re-packed whenever a parameter/buffer changes."""
        named = dict(self.named_parameters())
        named.update(dict(self.named_buffers()))
        key = (self.precision,) + tuple((n, t.data_ptr(), t._version) for n, t in sorted(named.items()))
        if self._packed is None or self._packed_key != key:
            self._packed = kernels.pack_weights(self.pdsc_config(), named)
            self._packed_key = key
        return self._packed

    # --------------------------------------------------------------- forward
    def forward(self, data):
        """models/PointDSC.py:128-197.  Testing mode: bs must be 1 as in :210/:414.
        Without 'testing' (eval mode only, any bs): {final_trans, final_labels =
        the logits, M = the feature-similarity matrix} (:158-163, :176-191)."""
        corr_pos, src, tgt = data["corr_pos"], data["src_keypts"], data["tgt_keypts"]
        if "testing" not in data.keys():
            if self.training:
                raise NotImplementedError(
                    "training-mode forward in model.train() (BatchNorm batch statistics, autograd) is out of "
                    "scope for the MI355X build; call model.eval() for the validation forward (DESIGN.md)")
            trans, conf, M, _ = kernels.forward_training(self.pdsc_config(), self.packed_weights(), corr_pos, src,
                                                         tgt)
            return {"final_trans": trans, "final_labels": conf, "M": M}
        assert corr_pos.shape[0] == 1  # pick_seeds / post_refinement support bs = 1 only
        trans, labels = kernels.forward_testing(self.pdsc_config(), self.packed_weights(), corr_pos, src, tgt)
        return {"final_trans": trans, "final_labels": labels, "M": None}

    def forward_list(self, datas):
        """A list of testing inputs of DIFFERENT sizes -- the evaluation loop's
        pairs (datasets/ThreeDMatch.py:268-290 keeps every keypoint, so N varies;
        evaluation/test_3DMatch.py:33-53 runs them at bs = 1) -- in ONE batched
        call (pdsc_forward_testing_ragged).  Each element is a ``forward`` input
        dict (tensors [1,n,.] or [n,.]; the 'testing' key is implied); returns one
        ``forward`` result dict per element: final_trans [1,4,4], final_labels
        [1,n], M None -- equal to calling ``forward`` on each."""
        if not datas:
            return []
        corr, counts = kernels.pad_pairs([d["corr_pos"] for d in datas])
        src, _ = kernels.pad_pairs([d["src_keypts"] for d in datas])
        tgt, _ = kernels.pad_pairs([d["tgt_keypts"] for d in datas])
        trans, labels = kernels.forward_ragged(self.pdsc_config(), self.packed_weights(), corr, src, tgt, counts)
        return [{"final_trans": trans[b:b + 1], "final_labels": labels[b:b + 1, :n], "M": None}
                for b, n in enumerate(counts)]

    def forward_batched(self, corr_pos, src_keypts, tgt_keypts):
        """B independent pairs in one call (same N): (final_trans [B,4,4], final_labels [B,N]).
        Equivalent to B calls of ``forward`` with bs = 1."""
        return kernels.forward_testing(self.pdsc_config(), self.packed_weights(), corr_pos, src_keypts,
                                       tgt_keypts)
