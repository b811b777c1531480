"""libpdsc.so loads and exports the C ABI of include/pdsc.h; host-side logic
(argument checks, parameter order, workspace queries) -- no GPU needed."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from pointdsc_amd import _lib
from pointdsc_amd.synthetic import state_dict_keys


def header_functions():
    src = open(os.path.join(ROOT, "include", "pdsc.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(pdsc_[a-z_0-9]+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 20, names
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/pdsc.h but not exported"
    assert set(names) == set(_lib.EXPORTS)


def test_version():
    assert b"gfx950" in _lib.load().pdsc_version()


@pytest.mark.parametrize("L", [1, 2, 12])
def test_param_order_matches_reference_state_dict(L):
    lib = _lib.load()
    cfg = _lib.make_config(num_layers=L)
    names = [lib.pdsc_param_name(ctypes.byref(cfg), i).decode() for i in range(lib.pdsc_param_count(ctypes.byref(cfg)))]
    ref = [k for k in state_dict_keys(L) if not k.endswith("num_batches_tracked")]
    assert names == ref


def test_refine_threshold_rule():
    # models/PointDSC.py:415-418
    assert abs(_lib.make_config(inlier_threshold=0.10).refine_threshold - 0.10) < 1e-7
    assert abs(_lib.make_config(inlier_threshold=0.6).refine_threshold - 1.2) < 1e-7


def test_workspace_queries():
    lib = _lib.load()
    cfg = _lib.make_config()
    for B, N in [(1, 1000), (4, 5000), (1, 30)]:
        assert lib.pdsc_forward_workspace_bytes(ctypes.byref(cfg), B, N) > 4 * B * N * N
        assert lib.pdsc_encoder_workspace_bytes(ctypes.byref(cfg), B, N) > 0
    assert lib.pdsc_forward_workspace_bytes(ctypes.byref(cfg), 1, 5) == 0  # int(5*0.1) = 0 seeds
    bad = _lib.make_config(num_channels=64)
    assert lib.pdsc_forward_workspace_bytes(ctypes.byref(bad), 1, 1000) == 0
    assert b"num_channels" in lib.pdsc_last_error()


def test_argument_errors_without_device():
    lib = _lib.load()
    assert lib.pdsc_compat_f32(None, None, 1, 10, None, None, None) == 1
    assert b"null" in lib.pdsc_last_error()
    cfg = _lib.make_config()
    rc = lib.pdsc_forward_testing(ctypes.byref(cfg), None, None, None, None, 1, 1000, None, None, None,
                                  None, None, 0, None)
    assert rc == 1


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.load()


def test_module_state_dict_keys_match_reference():
    import torch
    from pointdsc_amd.PointDSC import PointDSC
    m = PointDSC(num_layers=12)
    assert list(m.state_dict().keys()) == state_dict_keys(12)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in
          __import__("pointdsc_amd.synthetic", fromlist=["x"]).trained_state_dict("3dmatch", 12).items()}
    m.load_state_dict(sd, strict=True)


def test_module_refuses_cpu_and_training():
    import torch
    from pointdsc_amd.PointDSC import PointDSC
    m = PointDSC(num_layers=2)
    data = {"corr_pos": torch.zeros(1, 50, 6), "src_keypts": torch.zeros(1, 50, 3),
            "tgt_keypts": torch.zeros(1, 50, 3)}
    with pytest.raises(NotImplementedError):
        m(data)
    data["testing"] = True
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(data)


def test_query_functions_reject_bad_precision():
    lib = _lib.load()
    a, b = ctypes.c_int32(), ctypes.c_int32()
    assert lib.pdsc_attention_layout(4, 1000, 0, ctypes.byref(a), ctypes.byref(b)) == 0
    assert lib.pdsc_encoder_plan(4, 1000, 1, ctypes.byref(a)) == 0
    assert lib.pdsc_attention_layout(4, 1000, 7, ctypes.byref(a), ctypes.byref(b)) == 1
    assert b"precision" in lib.pdsc_last_error()
    assert lib.pdsc_encoder_plan(4, 1000, -1, ctypes.byref(a)) == 1


def test_ragged_counts_validated_on_host():
    """pdsc_forward_testing_ragged rejects counts that would change a pair's k
    (min(k, count - 1) must equal the batch's) or leave it without seeds, before
    touching any buffer (dummy non-null pointers: nothing is dereferenced)."""
    lib = _lib.load()
    cfg = _lib.make_config()
    dummy = ctypes.c_void_p(16)
    for counts in ([1000, 40], [1000, 1001], [1000, 0]):
        arr = (ctypes.c_int32 * 2)(*counts)
        rc = lib.pdsc_forward_testing_ragged(ctypes.byref(cfg), dummy, dummy, dummy, dummy, 2, 1000, arr, dummy,
                                             dummy, None, dummy, 1, None)
        assert rc == 1 and b"counts[1]" in lib.pdsc_last_error(), counts
    rc = lib.pdsc_forward_testing_ragged(ctypes.byref(cfg), dummy, dummy, dummy, dummy, 2, 1000, None, dummy,
                                         dummy, None, dummy, 1, None)
    assert rc == 1


def test_flat_weight_views_track_edits():
    """PointDSC re-homes the packed parameters/buffers as views of one flat
    buffer (PointDSC._flatten; on the device in a forward, on the CPU here):
    state_dict keys, values and requires_grad are unchanged, and every kind of
    in-place edit -- an optimizer-style update under no_grad, load_state_dict's
    copy_, a running statistic -- bumps the ONE version counter the per-forward
    change check reads; replacing a Parameter bumps the registration epoch."""
    import torch
    import torch.nn as nn
    from pointdsc_amd import PointDSC as mod
    m = mod.PointDSC(num_layers=3)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    grads = {k: p.requires_grad for k, p in m.named_parameters()}
    tensors = m._packable(m.pdsc_config())
    flat = m._flatten(tensors, device_only=False)
    assert flat is not None and flat.numel() == sum(t.numel() for t in tensors.values())
    after = m.state_dict()
    assert list(after) == list(before)
    assert all(torch.equal(after[k], before[k]) for k in before)
    assert {k: p.requires_grad for k, p in m.named_parameters()} == grads
    views = m._packable(m.pdsc_config())
    assert all(t.data_ptr() >= flat.data_ptr() for t in views.values())
    v = flat._version
    with torch.no_grad():
        m.encoder.layer0.weight.mul_(2)
    assert flat._version != v
    v = flat._version
    m.encoder.blocks["PointCN_layer_1"][1].running_var.add_(1)
    assert flat._version != v
    v = flat._version
    m.load_state_dict(before)
    assert flat._version != v and torch.equal(m.state_dict()["encoder.layer0.weight"], before["encoder.layer0.weight"])
    e = mod._REGISTRATION_EPOCH[0]
    m.classification[4].bias = nn.Parameter(torch.zeros(1))
    assert mod._REGISTRATION_EPOCH[0] != e


def test_flatten_keeps_parameter_objects_and_inference_mode():
    """the flat buffer keeps every Parameter / buffer OBJECT (an
    optimizer built before the first forward still updates the model, and its
    steps bump the flat version), it is built outside inference mode (a first
    forward under torch.inference_mode() leaves ordinary tensors: later in-place
    edits and load_state_dict outside it work), and a registration in another
    module does not count as a change of this model's tensors."""
    import torch
    import torch.nn as nn
    from pointdsc_amd import PointDSC as mod
    m = mod.PointDSC(num_layers=2)
    ids = {k: id(v) for k, v in m.named_parameters()}
    bufs = {k: id(v) for k, v in m.named_buffers()}
    opt = torch.optim.SGD(m.parameters(), lr=0.5)
    w0 = m.encoder.layer0.weight
    w0.grad = torch.ones_like(w0)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    cfg = m.pdsc_config()
    with torch.inference_mode():
        flat = m._flatten(m._packable(cfg), device_only=False)
        _ = flat._version  # readable: not an inference tensor
    assert flat is not None and not flat.is_inference()
    assert {k: id(v) for k, v in m.named_parameters()} == ids
    assert {k: id(v) for k, v in m.named_buffers()} == bufs
    assert m.encoder.layer0.weight is w0 and torch.equal(w0.grad, torch.ones_like(w0))
    assert all(not v.is_inference() for v in m.state_dict().values())
    assert all(torch.equal(m.state_dict()[k], before[k]) for k in before)
    assert flat.data_ptr() <= w0.data_ptr() < flat.data_ptr() + flat.numel() * 4
    v = flat._version
    opt.step()  # the optimizer's own Parameter references
    assert flat._version != v
    assert torch.allclose(m.encoder.layer0.weight, before["encoder.layer0.weight"] - 0.5)
    v = flat._version
    m.load_state_dict(before)  # outside inference mode, after the flatten
    assert flat._version != v and torch.equal(m.encoder.layer0.weight, before["encoder.layer0.weight"])
    # identity check after an unrelated registration (what packed_weights does on an epoch bump)
    st = {"flat": flat, "tensors": m._packable(cfg)}
    nn.Linear(2, 2)
    assert m._same_tensors(st, cfg)
    m.encoder.layer0.bias = nn.Parameter(torch.zeros_like(m.encoder.layer0.bias))
    assert not m._same_tensors(st, cfg)
