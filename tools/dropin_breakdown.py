"""Where the drop-in call's host wall goes (run on the GPU box):
PointDSC.forward at bs = 1 against its pieces -- the raw C call, the Python
wrapper, the range-guard read, and the per-call bookkeeping -- each as the mean
host wall over REPS back-to-back calls.  Measurement only (bench.py reports the
product numbers)."""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REPS = 200


def wall(fn, reps=REPS):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    from pointdsc_amd import _lib, kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_batch, trained_state_dict
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    m = m.to(dev).eval()
    d = synthetic_batch(1, N, seed=7000)
    c, s, t = (torch.from_numpy(d[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    data = {"corr_pos": c, "src_keypts": s, "tgt_keypts": t, "testing": True}
    L = _lib.load()
    cfg, pk = m.pdsc_config(), m.packed_weights()
    nb = L.pdsc_forward_workspace_bytes(ctypes.byref(cfg), 1, N)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    tr = torch.empty((1, 4, 4), device=dev)
    lab = torch.empty((1, N), device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    hip = ctypes.CDLL("libamdhip64.so")
    args = (ctypes.byref(cfg), ctypes.c_void_p(pk.data_ptr()), ctypes.c_void_p(c.data_ptr()),
            ctypes.c_void_p(s.data_ptr()), ctypes.c_void_p(t.data_ptr()), 1, N, ctypes.c_void_p(tr.data_ptr()),
            ctypes.c_void_p(lab.data_ptr()), None, None, ctypes.c_void_p(ws.data_ptr()), nb, sp)
    pinned = torch.empty(1, dtype=torch.int32, pin_memory=True)
    flags = ws[:4].view(torch.int32)

    def raw():
        L.pdsc_forward_testing(*args)

    def raw_sync():
        L.pdsc_forward_testing(*args)
        hip.hipStreamSynchronize(sp)

    def raw_rs():
        L.pdsc_forward_testing(*args)
        kernels.range_flags(ws, 1, dev)

    def raw_pinned():
        L.pdsc_forward_testing(*args)
        pinned.copy_(flags, non_blocking=True)
        stream.synchronize()
        return int(pinned[0])

    def raw_poll():
        L.pdsc_forward_testing(*args)
        return L.pdsc_range_poll(ctypes.c_void_p(ws.data_ptr()), 1, sp)

    def wrap():
        kernels.forward_testing(cfg, pk, c, s, t, ws=ws, check_range=False)

    out = {"N": N, "reps": REPS}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    raw()
    ev0.record()
    for _ in range(50):
        raw()
    ev1.record()
    ev1.synchronize()
    out["device_us"] = ev0.elapsed_time(ev1) / 50 * 1e3
    out["raw_async_us"] = wall(raw)
    out["raw_sync_each_us"] = wall(raw_sync)
    out["raw_range_status_us"] = wall(raw_rs)
    out["raw_pinned_copy_us"] = wall(raw_pinned)
    out["raw_poll_us"] = wall(raw_poll)
    out["wrapper_async_us"] = wall(wrap)
    out["dropin_us"] = wall(lambda: m(data))
    # host-only pieces (GPU idle)
    torch.cuda.synchronize()
    out["range_status_idle_us"] = wall(lambda: kernels.range_flags(ws, 1, dev))
    out["pinned_copy_idle_us"] = wall(lambda: (pinned.copy_(flags, non_blocking=True), stream.synchronize()))
    out["poll_idle_us"] = wall(lambda: L.pdsc_range_poll(ctypes.c_void_p(ws.data_ptr()), 1, sp))
    out["stream_sync_idle_us"] = wall(lambda: hip.hipStreamSynchronize(sp))
    out["current_stream_us"] = wall(lambda: torch.cuda.current_stream(dev), 2000)
    out["empty_4x4_us"] = wall(lambda: torch.empty((1, 4, 4), dtype=torch.float32, device=dev), 2000)
    out["ws_bytes_us"] = wall(lambda: L.pdsc_forward_workspace_bytes(ctypes.byref(cfg), 1, N), 2000)
    out["pdsc_config_us"] = wall(m.pdsc_config, 2000)
    out["packed_weights_us"] = wall(m.packed_weights, 2000)
    out["contiguous3_us"] = wall(lambda: (c.contiguous(), s.contiguous(), t.contiguous()), 2000)
    print(json.dumps({k: round(v, 2) if isinstance(v, float) else v for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
