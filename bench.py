#!/usr/bin/env python3
"""Throughput of PointDSC's testing-mode hot path on MI355X (BASELINE.json metric).

A step = one batched forward (compat -> SCNonlocal encoder -> classifier ->
NMS seeds -> seed kNN -> NSM power iteration -> Kabsch hypotheses ->
verification -> post-refinement) over --pairs synthetic scan pairs of
--num-corr correspondences each, inputs resident in HBM.  One process per GPU
(torchrun); pairs are independent, so ranks shard them with no data-path
collective (weak scaling); the only collectives are the barrier around the
timed region and a max-reduce of the elapsed time.

Prints ONE JSON line (rank 0).  Also measured live with HIP events on the
stream the kernels run on:
  roofline      -- the dominant kernel (SCNonlocal attention), MFMA bound; its fp32
                   products run as 3 fp16 MFMAs, so the peak is 2500/3 TFLOP/s
  roofline_hbm  -- the forward's a1 compatibility kernel (symmetric-packed M), HBM-write bound;
                   roofline_hbm_dense: the dense-M form
  roofline_path -- SURVEY 8(d)'s target: the compat + seed-kNN + NSM power-iteration
                   stages at N=5000 (stage events inside the forward), HBM bound,
                   priced with the algorithmic bytes B(N) = 24N + 4N^2 + S*k*(C+6)*4 + 4*S*k
  stages        -- per-stage ms of the headline forward (pdsc_forward_timing events)
  roofline_sm   -- SURVEY 8(f) row 3: the SM baseline's matrix-vector product at N=9000 (M past the
                   Infinity Cache), HBM bound
  single_pair   -- configs[1] literally: one N=1000 pair per forward, eager and as a HIP graph,
                   per-stage split, and the drop-in PointDSC.forward's host wall
  single_pair_5k -- the same at N=5000: the reference drivers' own call (bs = 1, N ~ 5000)
  ragged        -- one call over P pairs of mixed N (0.7-1.3 N), the evaluation loop's shape
Each roofline's `traffic` is the HBM bytes per launch of the same kernel at the
same launch shape from the committed rocprofv3 profile (profiles/traffic_current.json).
  cpu_baseline  -- the CPU oracle (oracle/, numpy + C) on a bounded sample
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md, v_mfma_f32_32x32x2_f32
PEAK_F16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md, dense v_mfma_f32_32x32x16_f16
MEASURED_F16_MFMA_TFLOPS = 1287.8  # profiles/r05_mfma_shape.log: 32x32x16 f16, all CUs, random operands
# the attention computes each fp32 product as 3 fp16 MFMA products (hi.hi + hi.lo + lo.hi,
# attention_h3.hpp): its ceiling in ALGORITHMIC (fp32) flop/s is the fp16 peak / 3
PEAK_H3_TFLOPS = PEAK_F16_MFMA_TFLOPS / 3
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md, HBM3E spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--num-corr", type=int, default=1000)
    ap.add_argument("--pairs", type=int, default=128, help="scan pairs per GPU per step")
    ap.add_argument("--preset", default="3dmatch", choices=["3dmatch", "kitti"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=20, help="launches per standalone-kernel timing (>= 1)")
    ap.add_argument("--f32-steps", type=int, default=3, help="steps of the exact-fp32 leg (0 = skip)")
    ap.add_argument("--path-n", type=int, default=5000, help="N of the compat+NSM path roofline (0 = skip)")
    ap.add_argument("--path-pairs", type=int, default=8)
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="exercise the multi-rank launch/gather plumbing on CPU (gloo), no forward")
    a = ap.parse_args()
    if a.kernel_iters < 1 or a.steps < 1:
        ap.error("--kernel-iters and --steps must be >= 1")
    return a


STAGES = ["compat", "encoder", "seeds", "seed_knn", "nsm", "hypotheses", "post_refine"]


class EventPool:
    """A flat array of hipEvent_t for libpdsc's pdsc_forward_timing hook."""

    def __init__(self, n):
        import ctypes
        self.ct = ctypes
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.n = n
        self.ev = (ctypes.c_void_p * n)()
        for i in range(n):
            e = ctypes.c_void_p()
            assert self.hip.hipEventCreate(ctypes.byref(e)) == 0
            self.ev[i] = e.value
        self.count = ctypes.c_int32(0)

    def ms(self, a, b):
        out = self.ct.c_float()
        assert self.hip.hipEventElapsedTime(self.ct.byref(out), self.ct.c_void_p(self.ev[a]),
                                            self.ct.c_void_p(self.ev[b])) == 0
        return out.value

    def stage_means(self):
        """{stage: mean ms} over the forwards recorded so far."""
        per = len(STAGES) + 1
        calls = self.count.value // per
        out = {}
        for j, name in enumerate(STAGES):
            out[name] = sum(self.ms(c * per + j, c * per + j + 1) for c in range(calls)) / max(calls, 1)
        return out, calls

    def __del__(self):
        for i in range(self.n):
            self.hip.hipEventDestroy(self.ct.c_void_p(self.ev[i]))


def profiled(kernel, grid_threads):
    """The committed rocprofv3 numbers (profiles/traffic_current.json, written by
    tools/summarize_profile.py from separate --pmc FETCH_SIZE / WRITE_SIZE passes of
    this bench) for one kernel at one launch shape: HBM bytes per dispatch
    (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 read correction) and the profiled
    average duration.  None when no profile of that shape is committed."""
    path = os.path.join(ROOT, "profiles", "traffic_current.json")
    try:
        with open(path) as f:
            prof = json.load(f)
        ks = prof["kernels"]
        # a templated kernel's rows are named with their arguments (nsm_seed_kernel<false, 48>):
        # a bare name matches the one instantiation launched at this grid
        names = [kernel] if kernel in ks else [k for k in ks if k.split("<")[0] == kernel and str(grid_threads) in ks[k]]
        if len(names) != 1:
            return None
        ent = ks[names[0]][str(grid_threads)]
    except (OSError, KeyError, ValueError):
        return None
    return {"tag": prof["tag"], "hbm_bytes": ent.get("hbm_bytes"), "avg_ms": ent["avg_us"] / 1e3}


def path_bytes(N, S, k, C=128):
    """algorithmic HBM bytes of compat + power-iteration path for one pair."""
    return 24.0 * N + 4.0 * N * N + S * k * (C + 6) * 4.0 + 4.0 * S * k


class HipEvents:
    """hipEvent_t pairs created through libamdhip64 (handed to libpdsc's timing hook)."""

    def __init__(self, n):
        import ctypes
        self.ct = ctypes
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.n = n
        self.start = (ctypes.c_void_p * n)()
        self.stop = (ctypes.c_void_p * n)()
        for arr in (self.start, self.stop):
            for i in range(n):
                ev = ctypes.c_void_p()
                assert self.hip.hipEventCreate(ctypes.byref(ev)) == 0
                arr[i] = ev.value
        self.count = ctypes.c_int32(0)

    def elapsed_ms(self, i):
        ms = self.ct.c_float()
        assert self.hip.hipEventElapsedTime(self.ct.byref(ms), self.ct.c_void_p(self.start[i]),
                                            self.ct.c_void_p(self.stop[i])) == 0
        return ms.value

    def __del__(self):
        for arr in (self.start, self.stop):
            for i in range(self.n):
                self.hip.hipEventDestroy(self.ct.c_void_p(arr[i]))


def event_time(fn, iters, stream):
    """Average ms per call of fn() measured with HIP events on `stream`."""
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        fn()
        start.record(stream)
        for _ in range(iters):
            fn()
        end.record(stream)
    end.synchronize()
    return start.elapsed_time(end) / iters


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args):
    """`bench.py --gpus N` without a launcher around it: start N rank processes
    of this script (one per GPU, like the reference's mp.spawn in
    evaluation/test_KITTI.py:220-228), wait for all of them and fail if any
    fails.  The parent never touches the GPU (no HIP call before the children
    start, no exec); rank 0's child prints the JSON line."""
    import signal
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, WORLD_SIZE=str(args.gpus), RANK=str(r), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    log(f"[launcher] rank {procs.index(p)} exited with {code}; stopping the others")
                    for q in pending:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


def selftest(args, world, rank):
    """--launcher-selftest: the multi-rank plumbing of the bench without a GPU
    (gloo on CPU, used by tests/test_bench_launcher.py): strided global pair
    ids, the all-gather of per-pair result rows, the max-reduce of the timed
    region and rank 0's single JSON line.  No forward is run, so `value` is null."""
    import torch.distributed as tdist
    from pointdsc_amd import dist as pdist
    from pointdsc_amd.evaluate import pair_stats
    from pointdsc_amd.synthetic import synthetic_pair
    if world > 1:
        tdist.init_process_group("gloo", init_method="env://")
    n_glob = args.pairs * world
    mine = pdist.shard_indices(n_glob, rank, world)
    ps = [synthetic_pair(32, 1000 + g, args.preset) for g in mine]
    gtT = torch.from_numpy(np.stack([p["gt_trans"] for p in ps]))
    gtL = torch.from_numpy(np.stack([p["gt_labels"] for p in ps]))
    rows = torch.cat([pair_stats(gtT, gtT, gtL, gtL), torch.tensor(mine, dtype=torch.float64)[:, None]], 1)
    t0 = time.perf_counter()
    if world > 1:
        tdist.barrier()
    allrows = pdist.gather_rows(rows, n_glob)
    _, elapsed = pdist.job_throughput(len(mine), time.perf_counter() - t0)
    if rank == 0:
        print(json.dumps({"selftest": True, "value": None, "n_gpus": world, "pairs_total": n_glob,
                          "pair_ids": allrows[:, -1].long().tolist(),
                          "synthetic_recall": float(allrows[:, 0].mean()), "elapsed_max_s": elapsed}), flush=True)
    if world > 1:
        tdist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and not (args.gpus == 1 and "WORLD_SIZE" not in os.environ):
        log(f"[rank {rank}] --gpus {args.gpus} but WORLD_SIZE={world}: the process group decides (n_gpus={world})")
    if args.launcher_selftest:
        return selftest(args, world, rank)
    # a process group whenever a launcher started this rank (torchrun or our own
    # spawn set RANK), so even a 1-rank job runs its gather / max-reduce on RCCL
    grp = world > 1 or "RANK" in os.environ
    if grp:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from pointdsc_amd import kernels
    from pointdsc_amd import _lib
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_batch, trained_state_dict

    p = PRESETS[args.preset]
    P, N = args.pairs, args.num_corr
    model = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                     inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40,
                     nms_radius=p["nms_radius"])
    # the trained stand-in weights with the classifier rescaled so that every bench
    # pair's seed ranking is tie-free (synthetic.BENCH_CLS): the headline workload is
    # then pinned to the reference itself (tests/golden/bench_3dmatch_1k_tf.npz)
    sd_bench = trained_state_dict(args.preset, 12, *BENCH_CLS)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd_bench.items()})
    model = model.to(dev).eval()
    cfg, packed = model.pdsc_config(), model.packed_weights()

    # the job is P pairs per rank; rank r owns the global pairs r, r + W, ... (strided like
    # DistributedSampler(shuffle=False), evaluation/test_KITTI.py:246-251), pair g seeded by g
    from pointdsc_amd import dist as pdist
    from pointdsc_amd.synthetic import synthetic_pair
    mine = pdist.shard_indices(P * world, rank, world)
    ps = [synthetic_pair(N, 1000 * 100003 + g, args.preset) for g in mine]
    data = {k: np.stack([q[k] for q in ps]) for k in ps[0]}
    corr, src, tgt = (torch.from_numpy(data[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    plan = kernels.ForwardPlan(cfg, packed, P, N, dev)
    stream = torch.cuda.current_stream(dev)

    log(f"[rank {rank}] warmup {args.warmup} steps of {P} pairs x N={N}")
    for _ in range(args.warmup):
        plan.run(corr, src, tgt)
    torch.cuda.synchronize(dev)

    def barrier():
        if grp:
            torch.distributed.barrier()

    # HIP events around every attention launch inside the timed region (the
    # dominant kernel), recorded on the stream the kernels run on
    import ctypes
    L = _lib.load()
    # (on the LAST timed step only: a timed event pair around every launch of every
    # step costs the step ~1 %, and 70 us per single-pair forward -- measured r04)
    evs = HipEvents(12)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == args.steps - 1:
            _lib.check(L.pdsc_attention_timing(evs.start, evs.stop, evs.n, ctypes.byref(evs.count)),
                       "pdsc_attention_timing")
        plan.run(corr, src, tgt)
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    L.pdsc_attention_timing(None, None, 0, None)
    att_times = [evs.elapsed_ms(i) for i in range(evs.count.value)]
    # per-stage ms from 3 more forwards with the stage events (outside the clock: a
    # stage-timed forward runs a1 on the caller's stream, not beside the encoder)
    sev = EventPool(3 * (len(STAGES) + 1))
    _lib.check(L.pdsc_forward_timing(sev.ev, sev.n, ctypes.byref(sev.count)), "pdsc_forward_timing")
    for _ in range(3):
        plan.run(corr, src, tgt)
    torch.cuda.synchronize(dev)
    L.pdsc_forward_timing(None, 0, None)
    own_elapsed = elapsed
    elapsed_min = elapsed
    if grp:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        tmin = torch.tensor([own_elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(tmin, op=torch.distributed.ReduceOp.MIN)
        elapsed, elapsed_min = float(t.item()), float(tmin.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = world * P * N * args.steps / elapsed
    # the fp16 range guard's marks of the last timed step (include/pdsc.h; after the clock)
    range_marked = len(plan.range_flags())
    if range_marked:
        log(f"[rank {rank}] WARNING: {range_marked} pairs marked by the fp16 range guard")
    log(f"[rank {rank}] {ms_per_step:.3f} ms/step -> {value:.4g} correspondences/s")

    # the last step's per-pair result rows (libs/loss.py metrics, evaluate.pair_stats), gathered
    # over all ranks with one all_gather (RCCL over xGMI for W > 1): registration recall of the job
    from pointdsc_amd.evaluate import THRESHOLDS, pair_stats
    gtT, gtL = torch.from_numpy(data["gt_trans"]).to(dev), torch.from_numpy(data["gt_labels"]).to(dev)
    rows = pair_stats(plan.trans, gtT, plan.labels, gtL, *THRESHOLDS[args.preset])
    rows = torch.cat([rows, torch.tensor(mine, dtype=rows.dtype, device=rows.device)[:, None]], 1)
    allrows = pdist.gather_rows(rows, P * world, device=dev)
    recall = float(allrows[:, 0].mean())
    pair_ids_ok = sorted(allrows[:, -1].long().tolist()) == list(range(P * world))

    result = None
    if rank == 0:
        # ---- dominant kernel: the attention (fused with the following pointwise chain
        # where the encoder plan says so), HIP events around each launch in the timed region
        att_ms = sum(att_times) / len(att_times)
        npad, nsplit, fused = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _lib.check(L.pdsc_attention_layout(P, N, 0, ctypes.byref(npad), ctypes.byref(nsplit)), "attention_layout")
        _lib.check(L.pdsc_encoder_plan(P, N, 0, ctypes.byref(fused)), "encoder_plan")
        grid = P * (npad.value // 128) * nsplit.value * 256
        if fused.value == 2:  # the split path's 64-query-wave attention (one 256-query workgroup per CU)
            grid = P * ((N + 255) // 256) * nsplit.value * 256
        if fused.value == 1:
            # attention 4 N^2 C + chain 2 x (fc0 128x64 + fc3 64x64 + fc6 64x128 + PointCN/Q/K/V 4 x 128x128) per point
            flops = P * (4.0 * N * N * 128 + 2.0 * 86016 * N)
            kname, kdesc, n_launch = "attn_pw2_kernel<1>", "attn_pw2_kernel (attention_l + pointwise chain_l, packed M)", 11
        elif fused.value == 2:
            # the split grid (attention_w64_kernel) or, where one round of one workgroup per CU
            # beats it, the stream-K form (attention_w64_sk_kernel, always 256 workgroups): the
            # committed profile does not record which batch shape a stream-K row is, so no lookup
            flops = P * 4.0 * N * N * 128
            kname, kdesc, n_launch = None, "attention_w64 (64-query waves, symmetric-packed M; split grid or stream-K)", 12
        else:
            flops = P * 4.0 * N * N * 128
            kname, kdesc, n_launch = "attention_h3_kernel<4>", "attention_h3_kernel<4,xcd>", 12
        achieved = flops / (att_ms * 1e-3) / 1e12
        att_prof = profiled(kname, grid) if kname else None
        roofline = {"kernel": kdesc, "bound": "mfma",
                    "achieved": round(achieved, 3), "peak": round(PEAK_H3_TFLOPS, 1), "unit": "TFLOP/s",
                    "frac": round(achieved / PEAK_H3_TFLOPS, 4),
                    "traffic": att_prof and att_prof["hbm_bytes"],
                    "traffic_unit": "HBM bytes per launch (rocprofv3 2*FETCH_SIZE+WRITE_SIZE)",
                    "profile": att_prof,
                    "peak_note": "fp16 MFMA 2500 TFLOP/s / 3 products per fp32 product (the attention's and, "
                                 "from r04, the fused chain's convolutions'); exact-fp32 MFMA peak is 157.3",
                    "fp16_mfma_util": round(3 * achieved / PEAK_F16_MFMA_TFLOPS, 4),
                    # context, not the roofline: the fp16 MFMA rate the chip sustains on random
                    # operands with every CU busy (the clock falls under load), measured by
                    # tools/mfma_shape_probe.hip (profiles/r05_mfma_shape.log), per 3 products
                    "measured_ceiling": {"value": round(MEASURED_F16_MFMA_TFLOPS / 3, 1), "unit": "TFLOP/s",
                                         "frac": round(achieved / (MEASURED_F16_MFMA_TFLOPS / 3), 4),
                                         "source": "tools/mfma_shape_probe.hip, two waves per SIMD, 1.71 GHz"},
                    "launch_ms": round(att_ms, 4), "launches_timed": len(att_times),
                    "flop_per_launch": flops, "share_of_step": round(n_launch * att_ms / ms_per_step, 3)}
        sp = ctypes.c_void_p(stream.cuda_stream)
        sd = model.sigma_spat.detach()
        ntile = (N + 63) // 64
        # the forward's a1 kernel: M written once as the symmetric-packed 32 x 32 tiles
        # (pdsc_compat_packed_f32), priced on the bytes it moves (packed M out + 24 N in)
        nfp = L.pdsc_compat_packed_floats(N)
        Mp = torch.empty((P, nfp), dtype=torch.float32, device=dev)

        def comp_p():
            L.pdsc_compat_packed_f32(src.data_ptr(), tgt.data_ptr(), P, N, sd.data_ptr(), Mp.data_ptr(), sp)

        cp_ms = event_time(comp_p, args.kernel_iters, stream)
        cpbytes = P * (4.0 * nfp + 24.0 * N)
        cpach = cpbytes / (cp_ms * 1e-3) / 1e9
        cp_prof = profiled("compat_packed_kernel", ntile * (ntile + 1) // 2 * P * 256)
        roofline_hbm = {"kernel": "compat_packed_kernel (the forward's a1)", "bound": "hbm",
                        "achieved": round(cpach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(cpach / PEAK_HBM_GBS, 4),
                        "traffic": cp_prof and cp_prof["hbm_bytes"], "profile": cp_prof,
                        "launch_ms": round(cp_ms, 4), "bytes_per_launch": cpbytes,
                        "dense_equivalent_GBs": round(P * (4.0 * N * N + 24.0 * N) / (cp_ms * 1e-3) / 1e9, 1),
                        "note": "bytes = the packed upper-triangle tiles written (about 2 N^2 per pair) + 24 N read; "
                                "dense_equivalent prices the same launch at the reference's dense 4 N^2"}
        del Mp
        # the dense form (pdsc_compat_f32: the exact-fp32 forward and the standalone API)
        Mo = torch.empty((P, N, N), dtype=torch.float32, device=dev)

        def comp():
            L.pdsc_compat_f32(src.data_ptr(), tgt.data_ptr(), P, N, sd.data_ptr(), Mo.data_ptr(), sp)

        c_ms = event_time(comp, args.kernel_iters, stream)
        cbytes = P * (4.0 * N * N + 24.0 * N)
        cach = cbytes / (c_ms * 1e-3) / 1e9
        c_prof = profiled("compat_kernel", ntile * (ntile + 1) // 2 * P * 256)
        roofline_hbm_dense = {"kernel": "compat_kernel (dense M)", "bound": "hbm", "achieved": round(cach, 1),
                              "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(cach / PEAK_HBM_GBS, 4),
                              "traffic": c_prof and c_prof["hbm_bytes"], "profile": c_prof,
                              "launch_ms": round(c_ms, 4), "bytes_per_launch": cbytes}
        del Mo

        stage_ms, _ = sev.stage_means()
        stages = {k: round(v, 4) for k, v in stage_ms.items()}

        # ---- SURVEY 8(d) target: compat + seed kNN + NSM stages at N = path_n
        roofline_path = None
        if args.path_n > 0:
            P5, N5 = args.path_pairs, args.path_n
            d5 = synthetic_batch(P5, N5, seed=5000 + rank, preset=args.preset)
            c5, s5, t5 = (torch.from_numpy(d5[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
            plan5 = kernels.ForwardPlan(cfg, packed, P5, N5, dev)
            for _ in range(2):
                plan5.run(c5, s5, t5)
            reps = 5
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(reps):
                plan5.run(c5, s5, t5)
            torch.cuda.synchronize(dev)
            fwd5 = (time.perf_counter() - t0) / reps
            ev5 = EventPool(reps * (len(STAGES) + 1))  # the stages: separate, stage-timed forwards
            L.pdsc_forward_timing(ev5.ev, ev5.n, ctypes.byref(ev5.count))
            for _ in range(reps):
                plan5.run(c5, s5, t5)
            torch.cuda.synchronize(dev)
            L.pdsc_forward_timing(None, 0, None)
            st5, _ = ev5.stage_means()
            S5, k5 = int(N5 * 0.1), min(40, N5 - 1)
            pb = P5 * path_bytes(N5, S5, k5)
            # measured HBM bytes of the same stages from the committed profile (launch
            # shapes as api.hip launches them at this N, P)
            nt5 = (N5 + 63) // 64
            shapes = [("compat_packed_kernel", nt5 * (nt5 + 1) // 2 * P5 * 256),
                      ("knn_dist_kernel", ((N5 + 31) // 32 + 4) // 5 * ((S5 + 127) // 128) * P5 * 256),
                      ("knn_select_kernel", (S5 + 3) // 4 * P5 * 256),
                      ("nsm_seed_kernel", (S5 + 3) // 4 * P5 * 256), ("nsm_finish_kernel", S5 * P5 * 64)]
            profs = [profiled(kname, g) for kname, g in shapes]
            path_traffic = (sum(pr["hbm_bytes"] for pr in profs)
                            if profs and all(pr and pr["hbm_bytes"] is not None for pr in profs) else None)
            t_path = st5["compat"] + st5["seed_knn"] + st5["nsm"]
            ach = pb / (t_path * 1e-3) / 1e9
            roofline_path = {"stages": "compat + seed_knn + nsm", "bound": "hbm", "achieved": round(ach, 1),
                             "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4),
                             "traffic": path_traffic, "traffic_note": "HBM bytes of the stages' kernels per forward "
                             "(rocprofv3 2*FETCH_SIZE+WRITE_SIZE, profiles/traffic_current.json)",
                             "traffic_achieved": path_traffic and round(path_traffic / (t_path * 1e-3) / 1e9, 1),
                             "traffic_frac": path_traffic and round(path_traffic / (t_path * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                             "num_corr": N5, "pairs": P5, "path_ms": round(t_path, 4),
                             "bytes_per_pair": path_bytes(N5, S5, k5),
                             "stage_ms": {k: round(v, 4) for k, v in st5.items()},
                             "forward_ms": round(fwd5 * 1e3, 3),
                             "correspondences_per_s": round(P5 * N5 / fwd5, 1)}
            del plan5, c5, s5, t5

        # ---- the SM baseline's power-iteration product (HBM bound)
        # and the whole SM call, at N = path_n
        roofline_sm = None
        if args.path_n > 0:
            from pointdsc_amd.baselines import SM, sm_matvec
            # the matrix-vector product at N = 9000: M = 324 MB, past the 256 MB Infinity
            # Cache, so each product streams M from HBM; the whole SM call at N = path_n
            Ns = args.path_n
            Nmv = max(Ns, 9000)
            Mm = torch.rand((Nmv, Nmv), dtype=torch.float32, device=dev)
            vv = torch.rand(Nmv, dtype=torch.float32, device=dev)
            mv_ms = event_time(lambda: sm_matvec(Mm, vv), 50, stream)
            mvb = 4.0 * Nmv * Nmv + 8.0 * Nmv
            d1s = synthetic_batch(1, Ns, seed=9000 + rank, preset=args.preset)
            cs, ss, ts = (torch.from_numpy(d1s[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
            sm_ms = event_time(lambda: SM(cs, ss, ts, inlier_threshold=p["inlier_threshold"]), 5, stream)
            mv_prof = profiled("sm_matvec_kernel", (Nmv + 3) // 4 * 256)
            roofline_sm = {"kernel": "sm_matvec_kernel", "bound": "hbm", "num_corr": Nmv, "sm_num_corr": Ns,
                           "traffic": mv_prof and mv_prof["hbm_bytes"], "profile": mv_prof,
                           "achieved": round(mvb / (mv_ms * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                           "frac": round(mvb / (mv_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4), "launch_ms": round(mv_ms, 4),
                           "bytes_per_launch": mvb,
                           "note": f"M ({4 * Nmv * Nmv / 1e6:.0f} MB) exceeds the 256 MB Infinity Cache: "
                                   "every product streams it from HBM",
                           "sm_pair_ms": round(sm_ms, 3)}
            del Mm, vv

        # ---- configs[1] literally: a single N pair per forward (latency), eager and graph-replayed;
        # and the reference drivers' own call at N = 5000 (configs[2] / [4]: evaluation/test_3DMatch.py:53,
        # test_KITTI.py:75 run model(data) once per pair at bs = 1 with N ~ 5000)
        def single_leg(Ns, seed, n_drop):
            d1 = synthetic_batch(1, Ns, seed=seed, preset=args.preset)
            c1, s1, t1 = (torch.from_numpy(d1[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
            plan1 = kernels.ForwardPlan(cfg, packed, 1, Ns, dev)
            e_ms = event_time(lambda: plan1.run(c1, s1, t1), 20, stream)
            sev1 = EventPool(5 * (len(STAGES) + 1))  # per-stage device time of 5 more eager forwards
            L.pdsc_forward_timing(sev1.ev, sev1.n, ctypes.byref(sev1.count))
            for _ in range(5):
                plan1.run(c1, s1, t1)
            torch.cuda.synchronize(dev)
            L.pdsc_forward_timing(None, 0, None)
            st1, _ = sev1.stage_means()
            plan1.capture(c1, s1, t1)
            g_ms = event_time(lambda: plan1.run(c1, s1, t1), 50, stream)
            del plan1
            # the drop-in call as the reference's drivers make it (evaluation/test_3DMatch.py:52-53,
            # demo_registration.py:117): model(data) per pair at bs = 1, host wall time of the whole
            # call -- argument checks, packed-weight change check, workspace, ~48 launches and the
            # synchronising fp16 range-guard read -- one call after the other
            data1 = {"corr_pos": c1, "src_keypts": s1, "tgt_keypts": t1, "testing": True}
            for _ in range(5):
                model(data1)
            torch.cuda.synchronize(dev)
            packs0, walls = model.pack_count, []
            for _ in range(n_drop):
                t0 = time.perf_counter()
                model(data1)
                walls.append((time.perf_counter() - t0) * 1e3)
            return {"num_corr": Ns, "eager_ms": round(e_ms, 4), "graph_ms": round(g_ms, 4),
                    "graph_correspondences_per_s": round(Ns / (g_ms * 1e-3), 1),
                    "stage_ms": {k: round(v, 4) for k, v in st1.items()},
                    "drop_in_ms": round(float(np.mean(walls)), 4), "drop_in_median_ms": round(float(np.median(walls)), 4),
                    "drop_in_over_eager": round(float(np.mean(walls)) / e_ms, 3),
                    "drop_in_correspondences_per_s": round(Ns / (float(np.mean(walls)) * 1e-3), 1),
                    "drop_in_repacks": model.pack_count - packs0,
                    "drop_in_note": f"PointDSC.forward({{'testing': True, ...}}) at bs = 1, host wall per call over "
                                    f"{n_drop} calls (range-guard read included); eager_ms / graph_ms / stage_ms: "
                                    f"device time of ForwardPlan.run by HIP events"}

        single = single_leg(N, 7000 + rank, 50)
        single_5k = single_leg(5000, 7500 + rank, 20) if args.path_n > 0 else None

        # ---- a ragged batch (pdsc_forward_testing_ragged): P pairs of N_b ~ U[0.7 N, 1.3 N],
        # the evaluation loop's mixed sizes in one call (datasets/ThreeDMatch.py:268-290)
        rng = np.random.RandomState(11 + rank)
        rsizes = rng.randint(int(0.7 * N), int(1.3 * N) + 1, size=P).tolist()
        rps = [synthetic_pair(n, 2000 * 100003 + i, args.preset) for i, n in enumerate(rsizes)]
        rN = max(rsizes)
        rcorr, rsrc, rtgt = (torch.zeros((P, rN, w), dtype=torch.float32, device=dev) for w in (6, 3, 3))
        for i, q in enumerate(rps):
            n = rsizes[i]
            rcorr[i, :n], rsrc[i, :n], rtgt[i, :n] = (torch.from_numpy(q[k]).to(dev)
                                                      for k in ("corr_pos", "src_keypts", "tgt_keypts"))
        # (the range marks are read once after the timed calls: a per-call read synchronises)
        r_ms = event_time(lambda: kernels.forward_ragged(cfg, packed, rcorr, rsrc, rtgt, rsizes, check_range=False),
                          5, stream)
        kernels.forward_ragged(cfg, packed, rcorr, rsrc, rtgt, rsizes)  # raises RangeError on a marked pair
        ragged = {"pairs": P, "num_corr_range": [int(0.7 * N), int(1.3 * N)], "padded_N": rN,
                  "correspondences": int(sum(rsizes)), "ms_per_call": round(r_ms, 4),
                  "correspondences_per_s": round(sum(rsizes) / (r_ms * 1e-3), 1)}
        del rcorr, rsrc, rtgt

        # ---- the exact-fp32 mode (pdsc_config.precision = f32: fp32 MFMA 32x32x2 contractions)
        # on the same resident batch: its rate, and its agreement with the headline (3xf16) path
        exact = None
        if args.f32_steps > 0:
            model.precision = "f32"
            cfg32, packed32 = model.pdsc_config(), model.packed_weights()
            plan32 = kernels.ForwardPlan(cfg32, packed32, P, N, dev)
            plan32.run(corr, src, tgt)
            plan.run(corr, src, tgt)
            torch.cuda.synchronize(dev)
            t_lab, t_tr = plan.labels.clone(), plan.trans.clone()
            f32_out = (plan32.trans.cpu().numpy(), plan32.labels.cpu().numpy())
            t0 = time.perf_counter()
            for _ in range(args.f32_steps):
                plan32.run(corr, src, tgt)
            torch.cuda.synchronize(dev)
            e32 = (time.perf_counter() - t0) / args.f32_steps
            exact = {"precision": "f32 (exact-fp32 MFMA contractions)", "ms_per_step": round(e32 * 1e3, 3),
                     "value": round(P * N / e32, 1), "steps": args.f32_steps,
                     "labels_equal_frac": float((plan32.labels == t_lab).float().mean()),
                     "max_pose_diff_vs_h3": float((plan32.trans - t_tr).abs().max())}
            model.precision = "h3"
            del plan32, packed32

        cpu = parity = None
        if not args.no_cpu_baseline and world == 1:
            from oracle import pdsc_oracle as O
            sd_np = sd_bench
            hip_out = {"h3": (plan.trans.cpu().numpy(), plan.labels.cpu().numpy())}
            if exact is not None:
                hip_out["f32"] = f32_out
            ref_out = []
            try:
                from threadpoolctl import threadpool_info
                cores = max([i.get("num_threads", 1) for i in threadpool_info()] + [1])
            except Exception:
                cores = int(os.environ.get("OMP_NUM_THREADS", "1"))
            n_done, t_c = 0, time.perf_counter()
            while n_done < P and (n_done < 2 or time.perf_counter() - t_c < args.cpu_seconds):
                r = O.forward_testing(data["corr_pos"][n_done], data["src_keypts"][n_done],
                                      data["tgt_keypts"][n_done], sd_np, num_layers=12,
                                      inlier_threshold=p["inlier_threshold"], nms_radius=p["nms_radius"])
                ref_out.append((r["final_trans"], r["final_labels"]))
                n_done += 1
            t_c = time.perf_counter() - t_c
            # the headline pairs' outputs against the oracle (the cpu leg's own results):
            # labels bit-exact, poses within north_star's 1e-4
            parity = {"vs": "oracle.pdsc_oracle.forward_testing on the same pairs and weights (the oracle is "
                            "pinned to the reference's outputs on all 128 bench pairs: "
                            "tests/golden/bench_3dmatch_1k_tf.npz)", "pairs": n_done,
                      "note": "poses beyond 1e-4 come from seed / kNN near-ties decided by fp32 rounding; "
                              "tests/test_gpu_bench_parity.py pins the stages after them on the HIP path's own "
                              "seeds and kNN rows at 1e-4"}
            for mode, (tr, lab) in hip_out.items():
                dT = [float(np.abs(tr[i] - ref_out[i][0]).max()) for i in range(n_done)]
                eq = [bool(np.array_equal(lab[i], ref_out[i][1])) for i in range(n_done)]
                parity[mode] = {"labels_equal_frac": sum(eq) / n_done, "max_pose_diff": max(dT),
                                "pairs_pose_gt_1e-4": [i for i in range(n_done) if dT[i] > 1e-4]}
            cpu = {"value": round(n_done * N / t_c, 1), "unit": "correspondences/s", "cores": cores,
                   "kind": "port",
                   "sample": f"{n_done} of the {P} bench pairs (N={N}) through oracle.pdsc_oracle."
                             f"forward_testing (numpy/BLAS + C), {t_c:.1f} s",
                   "note": "the oracle port, not the reference: it is slower than the reference's own torch "
                           "CPU forward, which SURVEY.md section 6 measured at about 19k correspondences/s "
                           "(N = 1000, 8 threads) in the build container; the reference itself does not "
                           "travel to the GPU box"}

        result = {
            "metric": "correspondence-pairs/sec through NSM (N=1k/5k) at 1/2/4/8 GPUs; 3DMatch recall parity",
            "value": round(value, 1), "unit": "correspondences/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32 (3xf16-split contractions)",
            "dtype_note": "fp32 inputs, outputs and accumulation; the attention, 1x1-conv and kNN/NSM "
                          "contractions run as 3 fp16 MFMA products (hi*hi + hi*lo + lo*hi) per fp32 product",
            "data": "synthetic",
            "config": {"workload": f"synthetic random correspondences N={N} ({args.preset}-like, 30% inliers), "
                                   f"{P} scan pairs per GPU per step, full PointDSC testing forward "
                                   f"(12 layers x 128 ch, trained synthetic weights, classifier rescaled "
                                   f"by synthetic.BENCH_CLS for tie-free seed ranking)",
                       "num_corr": N, "pairs_per_gpu_per_step": P, "global_batch": P * world,
                       "parallelism": f"dp{world} (independent pairs)"},
            "scan_pairs_per_s": round(world * P * args.steps / elapsed, 2),
            "synthetic_recall": recall, "pairs_gathered": int(allrows.shape[0]),
            # self-check of the multi-rank run (the driver's SCALE runs): the process group's size,
            # the spread of the ranks' own timed regions, and every global pair gathered once
            "distributed": {"world_size": torch.distributed.get_world_size() if grp else 1,
                            "backend": torch.distributed.get_backend() if grp else None,
                            "rank_ms_per_step": {"min": round(elapsed_min / args.steps * 1e3, 4),
                                                 "max": round(ms_per_step, 4)},
                            "pairs_expected": P * world, "pairs_gathered": int(allrows.shape[0]),
                            "pair_ids_ok": pair_ids_ok},
            "range_marked_pairs": range_marked,
            "roofline": roofline, "roofline_hbm": roofline_hbm, "roofline_hbm_dense": roofline_hbm_dense,
            "roofline_path": roofline_path,
            "roofline_sm": roofline_sm,
            "stages_ms": stages, "single_pair": single, "single_pair_5k": single_5k, "ragged": ragged, "exact_f32": exact, "cpu_baseline": cpu, "parity": parity,
        }
        print(json.dumps(result), flush=True)
    if grp:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
