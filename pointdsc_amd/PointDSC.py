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

import ctypes
import warnings

import torch
import torch.nn as nn
from torch.nn.modules import module as _nn_module

from . import _lib, kernels

# Bumped whenever ANY module registers (or replaces) a parameter, buffer or
# sub-module -- e.g. ``model.encoder.layer0.weight = nn.Parameter(...)``: every
# PointDSC then compares its own packed tensors' identities on its next forward
# and re-packs only if one of ITS tensors was replaced (PointDSC.packed_weights).
_REGISTRATION_EPOCH = [0]


def _bump_epoch(*_):
    _REGISTRATION_EPOCH[0] += 1


_nn_module.register_module_parameter_registration_hook(_bump_epoch)
_nn_module.register_module_buffer_registration_hook(_bump_epoch)
_nn_module.register_module_module_registration_hook(_bump_epoch)

# workspaces up to this size stay cached per stream between forwards
_WS_CACHE_LIMIT = 256 << 20

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


def _rows(tensors, idx):
    """The batch rows idx of each tensor (idx None: the tensors themselves)."""
    return tensors if idx is None else tuple(t[idx] for t in tensors)


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

    # ------------------------------------------------------------- internals
    def pdsc_config(self, precision=None) -> _lib.PdscConfig:
        """Hyper-parameters as the C ABI's ``pdsc_config`` (read at call time,
        so attribute edits after construction are honoured like the reference)."""
        key = (self.in_dim, self.num_layers, self.num_channels, self.num_iterations, self.k, self.ratio,
               self.inlier_threshold, self.nms_radius, precision or self.precision)
        cache = self.__dict__.setdefault("_cfg_cache", {})
        cfg = cache.get(key)
        if cfg is None:
            cfg = cache[key] = _lib.make_config(*key[:4], key[4], *key[5:])
        return cfg

    def invalidate_packing(self):
        """Forget the packed weights (rebuilt on the next forward).  Needed only
        after edits the change check cannot see: writes through ``.data`` (a
        tensor with its own version counter) or to storage shared with another
        tensor; in-place edits of the parameters/buffers themselves,
        ``load_state_dict``, ``.to()/.cuda()`` and parameter replacement are
        detected."""
        self.__dict__["_pack"] = None

    def _apply(self, fn, *args, **kwargs):  # .to() / .cuda() / .float() ...
        self.invalidate_packing()
        return super()._apply(fn, *args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        self.invalidate_packing()
        return super().load_state_dict(*args, **kwargs)

    def _packable(self, cfg):
        """{state_dict key: tensor} the kernels' blob is packed from (pdsc_param_name order)."""
        cache = self.__dict__.setdefault("_names_cache", {})
        lkey = (cfg.in_dim, cfg.num_layers, cfg.num_channels)
        names = cache.get(lkey)
        if names is None:
            L = _lib.load()
            names = cache[lkey] = [L.pdsc_param_name(ctypes.byref(cfg), i).decode()
                                   for i in range(L.pdsc_param_count(ctypes.byref(cfg)))]
        named = dict(self.named_parameters())
        named.update(self.named_buffers())
        missing = [n for n in names if n not in named]
        if missing:
            raise KeyError(f"missing parameters {missing[:4]}")
        return {n: named[n] for n in names}

    def _flatten(self, tensors, device_only=True):
        """Re-home the packed parameters/buffers as views of ONE flat device buffer:
        views share their base's version counter, so any in-place edit of any of
        them (optimizer steps under no_grad, ``copy_`` in ``load_state_dict``,
        ``mul_``...) bumps ``flat._version`` -- the per-forward change check is one
        integer compare instead of walking 358 tensors (60-130 us of Python per
        call).  Every Parameter / buffer keeps its Python object (its contents are
        swapped in place by ``torch.utils.swap_tensors``), so optimizers, hooks and
        references taken before the first forward stay live; values, names,
        shapes, requires_grad and .grad are unchanged.  The flat buffer is built
        outside inference mode, so a first forward under ``torch.inference_mode()``
        leaves ordinary tensors behind.  Returns None (no flattening: the caller
        falls back to the per-tensor check) when a tensor is not a float32 device
        tensor or cannot be swapped (e.g. it has weak references)."""
        ts = list(tensors.values())
        dev = ts[0].device
        if not all((t.is_cuda or not device_only) and t.device == dev and t.dtype == torch.float32 for t in ts):
            return None  # pack_weights raises the precise error (CPU tensor, dtype)
        with torch.inference_mode(False), torch.no_grad():
            flat = torch.cat([t.detach().reshape(-1) for t in ts])
            news, off = [], 0
            for t in ts:
                view = flat[off:off + t.numel()].view(t.shape)
                off += t.numel()
                if isinstance(t, nn.Parameter):
                    new = nn.Parameter(view, requires_grad=t.requires_grad)
                    if t.grad is not None:
                        new.grad = t.grad
                else:
                    new = view.detach()  # shares flat's version counter, not a view object
                news.append(new)
            done = []
            try:
                for t, new in zip(ts, news):
                    torch.utils.swap_tensors(t, new)
                    done.append((t, new))
            except RuntimeError:
                for t, new in reversed(done):  # undo: every tensor back on its own storage
                    torch.utils.swap_tensors(t, new)
                return None
        return flat

    def _same_tensors(self, st, cfg):
        """True if this model's packed parameters/buffers are still the objects
        ``st`` flattened, all still on its flat buffer: a registration elsewhere in
        the process (another module built) then needs no re-flatten."""
        if st["flat"] is None:
            return False
        lo = st["flat"].data_ptr()
        hi = lo + st["flat"].numel() * 4
        cur = self._packable(cfg)
        return all(cur[n] is t and lo <= t.data_ptr() < hi for n, t in st["tensors"].items())

    def packed_weights(self, precision=None) -> torch.Tensor:
        """Kernel-layout weights (one cached packing per precision), re-packed
        when a parameter/buffer changed since: checked per call by the flat
        buffer's version counter (or, without one, every tensor's) and, after
        any module registration in the process, by this model's own tensor
        identities (see ``_flatten``, ``invalidate_packing``)."""
        precision = precision or self.precision
        st = self.__dict__.get("_pack")
        layout = (self.in_dim, self.num_layers, self.num_channels)
        epoch = _REGISTRATION_EPOCH[0]
        if st is not None and st["epoch"] != epoch and st["layout"] == layout \
                and self._same_tensors(st, self.pdsc_config(precision)):
            st["epoch"] = epoch  # the registration was not ours
        if st is None or st["epoch"] != epoch or st["layout"] != layout:
            cfg = self.pdsc_config(precision)
            tensors = self._packable(cfg)
            flat = self._flatten(tensors)
            st = self.__dict__["_pack"] = {"epoch": epoch, "layout": layout, "flat": flat,
                                           "version": flat._version if flat is not None
                                           else [t._version for t in tensors.values()],
                                           "tensors": tensors, "packed": {}}
        elif st["flat"] is not None:
            if st["flat"]._version != st["version"]:  # values edited in place
                st["version"], st["packed"] = st["flat"]._version, {}
        else:
            v = [t._version for t in st["tensors"].values()]
            if v != st["version"]:
                st["version"], st["packed"] = v, {}
        if precision not in st["packed"]:
            st["packed"][precision] = kernels.pack_weights(self.pdsc_config(precision), st["tensors"])
            self.__dict__["pack_count"] = self.__dict__.get("pack_count", 0) + 1
        return st["packed"][precision]

    def _workspace(self, cfg, B, N, device):
        """The forward's workspace for (cfg, B, N) on the current stream, cached
        per stream (stream order keeps consecutive forwards apart)."""
        nb = _lib.load().pdsc_forward_workspace_bytes(ctypes.byref(cfg), B, N)
        if nb == 0 or nb > _WS_CACHE_LIMIT:
            return None  # forward_testing allocates (or reports the unsupported configuration)
        key = (device, torch.cuda.current_stream(device).cuda_stream)
        cache = self.__dict__.setdefault("_ws_cache", {})
        ws = cache.get(key)
        if ws is None or ws.numel() < nb:
            ws = cache[key] = torch.empty(nb, dtype=torch.uint8, device=device)
        return ws

    def _range_guarded(self, run):
        """run(cfg, packed, idx) -> the outputs' tuple for the pairs idx (None: all).
        Pairs the fp16 range guard marks (kernels.RangeError; include/pdsc.h) are
        run again with exact fp32 contractions and spliced into the result, so a
        forward never returns the 3xfp16 path's NaN pose for them.  A pair still
        marked in exact fp32 (non-finite logits, e.g. from non-finite inputs;
        also the 'f32' model's only marks) keeps the marked result -- NaN pose,
        zero labels, as the reference's own arithmetic would give NaN -- with a
        warning: the other pairs' results are returned either way."""
        try:
            return run(self.pdsc_config(), self.packed_weights(), None)
        except kernels.RangeError as e:
            out, bad = e.outputs, e.pairs
        if self.precision != "f32":
            warnings.warn(f"pairs {bad}: activations beyond fp16's range in the 3xfp16 path; "
                          f"recomputed with exact fp32 contractions", RuntimeWarning, stacklevel=3)
            try:
                redo, still = run(self.pdsc_config("f32"), self.packed_weights("f32"), bad), []
            except kernels.RangeError as e2:
                redo, still = e2.outputs, [bad[i] for i in e2.pairs]
            idx = torch.tensor(bad, device=out[0].device)
            for t, r in zip(out, redo):
                if t is not None:
                    t[idx] = r
            bad = still
        if bad:
            warnings.warn(f"pairs {bad}: non-finite logits in exact fp32 as well (non-finite inputs?); their "
                          f"final_trans is NaN and final_labels 0", RuntimeWarning, stacklevel=3)
        return out

    def _forward_one(self, corr_pos, src, tgt):
        """The drop-in call's path (bs = 1, the reference drivers' shape): one C
        call on the current stream with the cached workspace, then the fp16 range
        guard's answer through pdsc_range_poll (a one-wavefront kernel stores it
        into a coherent host word the host spins on: no D2H copy, no stream
        synchronisation; tools/dropin_breakdown.py times the alternatives).
        Returns None -- the caller then takes the
        general path, which raises the precise error or re-runs a marked pair in
        exact fp32 -- when the workspace is not cacheable or the pair is marked."""
        dev = src.device
        f32 = torch.float32
        if not (corr_pos.dtype is f32 and src.dtype is f32 and tgt.dtype is f32 and corr_pos.is_cuda and tgt.is_cuda
                and corr_pos.is_contiguous() and src.is_contiguous() and tgt.is_contiguous()):
            corr_pos, src, tgt = (kernels._dev(corr_pos, "corr_pos"), kernels._dev(src, "src_keypts"),
                                  kernels._dev(tgt, "tgt_keypts"))
        cfg, pk = self.pdsc_config(), self.packed_weights()
        kernels._check_inputs(cfg, corr_pos, src, tgt)
        N = src.shape[1]
        sh = torch._C._cuda_getCurrentRawStream(dev.index)  # = torch.cuda.current_stream(dev).cuda_stream
        cache = self.__dict__.setdefault("_one_cache", {})
        ent = cache.get((dev, sh, N, id(cfg)))
        if ent is None:
            ws = self._workspace(cfg, 1, N, dev)
            if ws is None:
                return None
            if len(cache) > 256:
                cache.clear()
            L = _lib.load()
            ent = cache[(dev, sh, N, id(cfg))] = (
                L.pdsc_forward_testing, ctypes.byref(cfg), L.pdsc_forward_workspace_bytes(ctypes.byref(cfg), 1, N),
                self.__dict__["_ws_cache"], (dev, sh), ctypes.c_void_p(sh), L.pdsc_range_poll)
        fwd, cfgp, nb, wsc, wkey, sp, poll = ent
        ws = wsc.get(wkey)
        if ws is None or ws.numel() < nb:  # another model size / N grew the stream's workspace meanwhile
            ws = self._workspace(cfg, 1, N, dev)
        out = torch.empty(16 + N, dtype=torch.float32, device=dev)  # one allocation, two views
        trans, labels = out.as_strided((1, 4, 4), (16, 4, 1)), out.as_strided((1, N), (N, 1), 16)
        wp = ws.data_ptr()
        _lib.check(fwd(cfgp, pk.data_ptr(), corr_pos.data_ptr(), src.data_ptr(), tgt.data_ptr(), 1, N,
                       trans.data_ptr(), labels.data_ptr(), None, None, wp, nb, sp), "pdsc_forward_testing")
        # the range guard's answer through pdsc_range_poll's host word (include/pdsc.h):
        # PDSC_ERR_RANGE (marked) -> the general path re-runs the pair in exact fp32;
        # any other error -> the general path reports it precisely
        if poll(ctypes.c_void_p(wp), 1, sp) != 0:
            return None
        return {"final_trans": trans, "final_labels": labels, "M": None}

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
            trans, conf, M, _ = self._range_guarded(lambda cfg, pk, i: kernels.forward_training(
                cfg, pk, *_rows((corr_pos, src, tgt), i)))
            return {"final_trans": trans, "final_labels": conf, "M": M}
        assert corr_pos.shape[0] == 1  # pick_seeds / post_refinement support bs = 1 only
        if isinstance(src, torch.Tensor) and src.is_cuda:
            res = self._forward_one(corr_pos, src, tgt)
            if res is not None:
                return res
        trans, labels = self._range_guarded(lambda cfg, pk, i: kernels.forward_testing(
            cfg, pk, *_rows((corr_pos, src, tgt), i),
            ws=self._workspace(cfg, 1, src.shape[1], src.device) if src.is_cuda and i is None else None))
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
        trans, labels = self.forward_padded(corr, src, tgt, counts)
        return [{"final_trans": trans[b:b + 1], "final_labels": labels[b:b + 1, :n], "M": None}
                for b, n in enumerate(counts)]

    def forward_padded(self, corr_pos, src_keypts, tgt_keypts, counts):
        """A zero-padded ragged batch (kernels.pad_pairs): pair b in the first
        counts[b] rows.  Returns (final_trans [B,4,4], final_labels [B,N], rows past
        counts[b] 0), each pair as its own bs = 1 ``forward``.  The ragged kernels
        run every pair with the batch's neighbourhood k (include/pdsc.h); a pair
        with count <= k, whose forward clips k to count - 1 (:250), runs alone."""
        counts = [int(c) for c in counts]
        B, N = corr_pos.shape[:2]
        big = [b for b, n in enumerate(counts) if n >= self.k + 1]
        if len(big) == B:
            return self._range_guarded(lambda cfg, pk, i: kernels.forward_ragged(
                cfg, pk, *_rows((corr_pos, src_keypts, tgt_keypts), i),
                counts if i is None else [counts[b] for b in i]))
        trans = torch.empty((B, 4, 4), dtype=torch.float32, device=corr_pos.device)
        labels = torch.zeros((B, N), dtype=torch.float32, device=corr_pos.device)
        if big:
            T, L = self.forward_padded(*_rows((corr_pos, src_keypts, tgt_keypts), big), [counts[b] for b in big])
            trans[big], labels[big] = T, L
        for b in (b for b in range(B) if counts[b] < self.k + 1):
            n = counts[b]
            r = self({"corr_pos": corr_pos[b:b + 1, :n], "src_keypts": src_keypts[b:b + 1, :n],
                      "tgt_keypts": tgt_keypts[b:b + 1, :n], "testing": True})
            trans[b], labels[b, :n] = r["final_trans"][0], r["final_labels"][0]
        return trans, labels

    def forward_batched(self, corr_pos, src_keypts, tgt_keypts):
        """B independent pairs in one call (same N): (final_trans [B,4,4], final_labels [B,N]).
        Equivalent to B calls of ``forward`` with bs = 1."""
        return self._range_guarded(lambda cfg, pk, i: kernels.forward_testing(
            cfg, pk, *_rows((corr_pos, src_keypts, tgt_keypts), i)))
