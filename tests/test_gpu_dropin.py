"""The drop-in call as the reference's drivers make it (run with -m gpu):
``model(data)`` once per pair at bs = 1 (evaluation/test_3DMatch.py:52-53,
demo_registration.py:117).  The packed weights are cached and re-packed only
when a parameter or buffer changed: an in-place edit after a forward must show
in the next forward's results (equal to a fresh model holding the edited
weights), and a forward without an edit must reuse the packing."""
import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _model(dev):
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, trained_state_dict
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    return m.to(dev).eval()


def _data(dev, N=1000, seed=77):
    from pointdsc_amd.synthetic import synthetic_pair
    q = synthetic_pair(N, seed)
    d = {k: torch.from_numpy(q[k][None]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts")}
    d["testing"] = True
    return d


def _fresh(dev, m, data):
    """The same weights in a model that never ran: packed from scratch."""
    f = _model(dev)
    f.load_state_dict(m.state_dict())
    return f(data)


def _same(a, b):
    return torch.equal(a["final_trans"], b["final_trans"]) and torch.equal(a["final_labels"], b["final_labels"])


def test_packing_reused_without_edits(gpu_device):
    m, data = _model(gpu_device), _data(gpu_device)
    r1 = m(data)
    pc, pk = m.pack_count, m.packed_weights()
    for _ in range(3):
        r = m(data)
        assert _same(r, r1)
    assert m.pack_count == pc and m.packed_weights() is pk
    # a different pair size or the evaluation-mode batch forward: still the same packing
    m(_data(gpu_device, N=777))
    assert m.pack_count == pc


def test_inplace_edit_after_forward_repacks(gpu_device):
    m, data = _model(gpu_device), _data(gpu_device)
    r0 = m(data)
    pc = m.pack_count
    with torch.no_grad():  # an optimizer-style in-place update of one tensor
        m.sigma_spat.mul_(1.5)  # sigma_d: M, hence every stage, changes
    r1 = m(data)
    assert m.pack_count == pc + 1
    assert not _same(r0, r1)
    assert _same(r1, _fresh(gpu_device, m, data))
    with torch.no_grad():
        m.encoder.blocks["PointCN_layer_3"][0].weight.mul_(0.5)
    r2 = m(data)
    assert m.pack_count == pc + 2 and _same(r2, _fresh(gpu_device, m, data))
    # a running statistic (buffer) edited in place
    m.encoder.blocks["PointCN_layer_5"][1].running_var.mul_(4.0)
    r3 = m(data)
    assert m.pack_count == pc + 3 and _same(r3, _fresh(gpu_device, m, data))


def test_replace_load_and_move_repack(gpu_device):
    m, data = _model(gpu_device), _data(gpu_device)
    m(data)
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    # a replaced Parameter object (registration epoch)
    w = m.encoder.layer0.weight.detach().clone() * -1.0
    m.encoder.layer0.weight = nn.Parameter(w)
    r = m(data)
    assert _same(r, _fresh(gpu_device, m, data))
    # load_state_dict back to the original weights
    m.load_state_dict(sd0)
    r = m(data)
    assert _same(r, _fresh(gpu_device, m, data))
    # a round trip through the host and back (.cpu() / .to()): same results as before it
    m = m.cpu().to(gpu_device)
    assert _same(m(data), r)
    # a write through .data bypasses every version counter: invalidate_packing() picks it up
    m.encoder.layer0.weight.data.mul_(-1.0)
    m.invalidate_packing()
    assert _same(m(data), _fresh(gpu_device, m, data))


def test_state_dict_after_forward_matches_reference_layout(gpu_device):
    """After the first forward the parameters are views of one flat buffer: the
    state dict keeps the reference's 358 keys, shapes and values."""
    m, data = _model(gpu_device), _data(gpu_device)
    before = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    m(data)
    after = m.state_dict()
    assert list(after) == list(before)
    for k, v in before.items():
        assert after[k].shape == v.shape and torch.equal(after[k].cpu(), v), k
    assert all(p.is_leaf for p in m.parameters())


def test_forward_under_inference_mode_then_edit(gpu_device):
    """the first forward inside torch.inference_mode() must
    work, and leave ordinary tensors: an in-place edit, an optimizer step and
    load_state_dict outside it afterwards work and show in the next forward."""
    m, data = _model(gpu_device), _data(gpu_device)
    opt = torch.optim.SGD([m.sigma_spat], lr=0.0)
    s0 = m.sigma_spat.detach().clone()
    with torch.inference_mode():
        r0 = m(data)
    assert not m.sigma_spat.is_inference()
    with torch.no_grad():
        m.sigma_spat.mul_(1.5)
    r1 = m(data)
    assert not _same(r0, r1) and _same(r1, _fresh(gpu_device, m, data))
    # the optimizer's reference (taken before the first forward) is the model's tensor
    assert opt.param_groups[0]["params"][0] is m.sigma_spat
    with torch.no_grad():
        opt.param_groups[0]["params"][0].copy_(s0)
    with torch.inference_mode():
        r2 = m(data)
    assert _same(r2, r0)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    assert _same(m(data), r0)


def test_unrelated_registration_keeps_packing(gpu_device):
    """building another module (a process-wide
    registration) does not re-pack this model; replacing one of its own
    parameters does."""
    m, data = _model(gpu_device), _data(gpu_device)
    r0 = m(data)
    pc = m.pack_count
    nn.Linear(4, 4)
    assert _same(m(data), r0) and m.pack_count == pc
    m.encoder.layer0.bias = nn.Parameter(m.encoder.layer0.bias.detach().clone() + 0.25)
    r1 = m(data)
    assert m.pack_count == pc + 1 and _same(r1, _fresh(gpu_device, m, data))
