#!/usr/bin/env python3
"""bench.py — scans/sec of the FAST-LIO scan-matching hot path on MI355X.

Metric (BASELINE.json): "scans/sec (100k-pt scan vs N-pt map) + ms/IESKF-iteration, 1 GPU".
One step = one complete iterated-ESKF update (lio_ieskf_update: up to
max_iteration+1 = 4 h_share_model evaluations, kNN on the iterations where
ekfom_data.converge is true, host 23-dim algebra) of one synthetic scan whose
points are already resident in HBM (a ring of pre-uploaded scans).

Default workload = BASELINE.json configs[2] ("C3", the north_star target):
131,072-pt Livox-style scan vs a 5M-pt map grown through map_incremental by 20
scans, max_iteration = 3.  `value` has the scans resident in HBM; the rate with
each scan uploaded from pinned host memory through lio_scan_set (the C-ABI a
C++ caller uses) inside the step is reported beside it ("upload_inclusive").  Multi-GPU: the front end does not shard
(replicas only) — each rank runs its own replica on its own scans
(weak scaling); the loop-closure ICP (C4: 500k vs 500k) is sharded across the
ranks with the record all-gather (lio_gpu.dist) and reported in "loop_icp".

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import ctypes
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fast-lio-sam_gps_amd"))

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_PT_KNN = 112       # h-evaluation with kNN
BYTES_PER_PT_REUSE = 32      # h-evaluation reusing kNN
BYTES_PER_PT_ICP = 24        # per ICP iteration and source point


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def usable_cpus():
    """Threads the CPU baseline may use: the affinity set, capped by the cgroup CPU quota when one is
    set (the GPU box shows the whole host's CPUs but grants this job a share of them)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    if quota is not None and quota < aff:
        return quota, f"cgroup CPU quota ({quota} of {aff} CPUs in the affinity set, {os.cpu_count()} on the host)"
    return aff, f"all CPUs in the affinity set ({aff} of {os.cpu_count()} on the host)"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--prewarm-s", type=float, default=0.5,
                    help="untimed steps for this many seconds before the --warmup steps (GPU clock ramp)")
    ap.add_argument("--config", default="C3", choices=["C1", "C2", "C3", "C5"])
    ap.add_argument("--scans", type=int, default=8, help="distinct resident scans cycled through")
    ap.add_argument("--cell", type=float, default=1.0)
    ap.add_argument("--no-icp", action="store_true")
    ap.add_argument("--icp-reps", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--streams", default="2,8",
                    help="secondary figure: S independent scan streams (own map + ctx + HIP stream each) "
                         "driven by S host threads in this process; '' to skip (reported under 'multi_stream')")
    ap.add_argument("--cpu-scans", type=int, default=50, help="CPU baseline: median per-scan latency of this "
                    "many full IESKF updates after --cpu-warmup ones, at 1, 3 and all usable threads (SURVEY §8d)")
    ap.add_argument("--cpu-warmup", type=int, default=5)
    ap.add_argument("--pipeline", type=int, default=8, metavar="N",
                    help="secondary figure (rank 0): the C5 stream (BASELINE.json configs[4]) — N raw 120k-point "
                         "sweeps on the 10M map, half out and half back past the same places 40 s later, each "
                         "through Preprocess + UndistortPcl + downSizeFilterSurf -> IESKF update -> map_incremental "
                         "-> keyframe, then the loop leg (fetchClosestKeyframeIdx -> setSrcAndDstCloud -> "
                         "icpAlignment) on the newest keyframe; reported under 'pipeline' (0: skip)")
    ap.add_argument("--loop-seq", type=int, default=12, metavar="N",
                    help="secondary figure (rank 0): the loop leg as the node runs it — N loopTimerFunc calls "
                         "(fast_lio_sam.cpp:682-728) from C++ on one LoopClosure handle while the keyframe database "
                         "grows, submaps of a different size on every call; reported under 'loop_sequence' (0: skip)")
    ap.add_argument("--grow-scans", type=int, default=20,
                    help="C3/C5: scans appended through map_incremental before timing (SURVEY §8d)")
    ap.add_argument("--watchdog-s", type=float, default=240.0,
                    help="N > 1: seconds after the headline measurement before rank 0 prints what it has and every "
                         "rank exits (a collective of the secondary sections that never returns)")
    ap.add_argument("--pmc-sq", default=os.path.join(ROOT, "profiles", "r06_pmc_sq_c3.json"),
                    help="SQ issue / wait breakdown per kernel (scripts/pmc_sq_summary.py of a rocprofv3 --pmc pass)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_summary.json"),
                    help="per-launch HBM traffic measured with rocprofv3 --pmc (profiles/)")
    return ap.parse_args()


def _spawn_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) outside a launcher: start N rank processes through
    torch.distributed.run (one per GPU, 127.0.0.1 rendezvous) BEFORE this process touches the GPU, and
    return their exit status; rank 0 prints the JSON line."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def _time_double(args, LC, src, dst, local):
    """Side figure (one rank): the loop ICP in the OPT-IN double statistics (lio_icp_params.umeyama_float =
    LIO_ICP_UMEYAMA_DOUBLE) — faster, but 1.2-1.9e-4 from PCL's float arithmetic at C4 (outside the 1e-5
    bar), so never the headline."""
    lc = LC.LoopClosure(LC.LoopClosureConfig(), device=local, umeyama_float=LC.DOUBLE_STATS)
    lc.setInputSource(src)
    lc.setInputTarget(dst)
    r = lc.align(keep_aligned=False)
    ti = time.perf_counter()
    iters = 0
    for _ in range(args.icp_reps):
        r = lc.align(keep_aligned=False)
        iters += r.iterations
    s = time.perf_counter() - ti
    lc.close()
    return {"mode": "double statistics about a fixed centre (opt-in; outside the 1e-5 parity bar)",
            "ms_per_alignment": round(s / args.icp_reps * 1e3, 3), "iterations": r.iterations,
            "ms_per_iteration": round(s / max(iters, 1) * 1e3, 3), "score": r.score}


def _loop_icp(args, LC, synth, local, world, rank, dist, rehearse, coll_dev, barrier, torch):
    """The C4 loop ICP (secondary key loop_icp), sharded over the ranks; returns (loop_icp, src, dst)."""
    # C4 with a 2.5 m / 4 deg initial offset: PCL's criteria with the reference's epsilons take 9
    # iterations (the 0.3 m / 1.5 deg pair of round 1 converged after 1, so ms/iteration meant nothing)
    src, dst, Tgt = synth.make_icp_pair(n_points=500_000, seed=4321, disp=(2.5, 4.0))
    double = _time_double(args, LC, src, dst, local) if rank == 0 else None
    # the headline: the DEFAULT mode = PCL's float Umeyama in the Eigen 3.3 order (the reference's arithmetic,
    # loop_closure.h:42), sharded over the ranks (each rank its window of the float chains: block sums, event
    # lists and depth blocks all-gathered)
    lc = LC.LoopClosure(LC.LoopClosureConfig(), device=local)
    cb = None
    exchange = "none (1 rank)"
    if world > 1:
        from lio_gpu import dist as ldist

        port = os.environ.get("MASTER_PORT", "0")
        if rehearse:  # ranks sharing one GPU (RCCL refuses that): the C++ shared-memory exchange
            lc.set_shard_shm(rank, world, f"/lio_icp_{port}_{os.getppid()}", len(src))
            exchange = "host (C++ shared-memory all-gather, one GPU rehearsal; no Python per pass)"
        else:
            try:  # one RCCL communicator per rank created in C++; ncclAllGather enqueued by the library
                lc.set_shard_rccl(rank, world)
                exchange = "device (RCCL ncclAllGather enqueued from C++ on the handle's stream; no Python per pass)"
            except Exception as e:  # the torch.distributed form of the same device exchange
                cb = ldist.DeviceExchange()
                lc.set_shard_device(rank, world, cb)
                exchange = (f"device (RCCL all_gather_into_tensor on the handle's stream via torch; C++ "
                            f"communicator failed: {type(e).__name__}: {e})")
    lc.setInputSource(src)
    lc.setInputTarget(dst)
    lc.align(keep_aligned=False)
    barrier()
    # ms per alignment without the diagnostic timing events (each adds a marker packet between the
    # kernels of a pass: +0.05 ms per alignment); the kernel breakdown comes from a separate timed loop
    ti = time.perf_counter()
    iters = 0
    for _ in range(args.icp_reps):
        r = lc.align(keep_aligned=False)
        iters += r.iterations
    barrier()
    icp_s = time.perf_counter() - ti
    if dist is not None:
        t = torch.tensor([icp_s], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        icp_s = float(t.item())
    lc.set_timing(True)
    for _ in range(args.icp_reps):
        lc.align(keep_aligned=False)
    itm = lc.timing()
    lc.set_timing(False)
    full = []  # the whole icpAlignment (warm handle): source binning + target grid + align; median of 3
    for _ in range(3):
        barrier()
        tf = time.perf_counter()
        lc.setInputSource(src)
        lc.setInputTarget(dst)
        lc.align(keep_aligned=False)
        barrier()
        full.append((time.perf_counter() - tf) * 1e3)
    full_ms = float(sorted(full)[1])
    passes = itm["icp_launches"]
    shard_n = len(src) // world
    icp_kernel_ms = itm["icp_ms"] / max(passes, 1)
    nn_ms = itm["icp_nn_ms"] / max(itm["icp_nn_launches"], 1)
    loop_icp = {"config": "C4: 500k vs 500k, voxel 0.3 m, 2.5 m / 4 deg initial offset, PCL ICP semantics",
                "mode": f"umeyama_float={LC.FIDELITY_ORDER} (default: PCL's float Umeyama, sequential float means, "
                        "Eigen 3.3 GEMM sigma kc(32 KiB L1); seqsum: parallel, verified bit-exact; sharded: each rank "
                        "its source window; per pass records + block sums, event lists, depth blocks all-gathered)",
                "seqsum": lc.fidelity_stats(),
                # side figure: the opt-in double statistics (outside the 1e-5 bar), one rank
                "double_stats": double,
                "n_gpus": world, "passes_per_alignment": passes / max(args.icp_reps, 1),
                "ms_per_alignment": round(icp_s / args.icp_reps * 1e3, 3),
                "iterations": r.iterations, "ms_per_iteration": round(icp_s / max(iters, 1) * 1e3, 3),
                "exchange": exchange, "ms_full_icpAlignment": round(full_ms, 3),
                "score": r.score, "converged": bool(r.is_converged), "scaling": "strong",
                # the pass (correspondence + statistics kernels) and the correspondence kernel alone
                "kernel_ms_per_pass": round(icp_kernel_ms, 4),
                "nn_kernel_ms_per_pass": round(nn_ms, 4),
                "kernel_gbs": round(BYTES_PER_PT_ICP * shard_n / (icp_kernel_ms * 1e-3) / 1e9, 2)
                if passes else None,
                # NOT measured in this run: counter passes committed under profiles/ 
                "from_profile": {"sq_breakdown": _icp_sq(args), "traffic": _icp_traffic()}}
    return loop_icp, src, dst


def _profile_meta(path):
    """where a figure read from a committed counter pass comes from: the file and the measurement it records"""
    try:
        pm = json.load(open(path))
    except Exception:
        pm = {}
    return {"source": os.path.relpath(path, ROOT), "measured": pm.get("measured") if isinstance(pm, dict) else None}


def _icp_traffic():
    """the ICP tile kernel's HBM traffic per pass from the committed FETCH_SIZE / WRITE_SIZE passes
    (scripts/icp_pmc_traffic.py over scripts/icp_ab.py 1.0 1)"""
    path = os.path.join(ROOT, "profiles", "r06_pmc_icp_traffic.json")
    try:
        pm = json.load(open(path))
    except Exception:
        return None
    return {"mean_bytes_per_pass": pm["mean_hbm_traffic_bytes"], "x_algorithmic_mean": pm["mean_x_algorithmic"],
            "x_algorithmic_max": pm["max_x_algorithmic"], "algorithmic_bytes": pm["algorithmic_bytes_per_pass"],
            "source": os.path.relpath(path, ROOT)}


def _icp_sq(args):
    """the ICP correspondence kernels' issue / wait breakdown from the committed SQ counter pass (C4 pairs A
    and B, scripts/icp_ab.py under rocprofv3 --pmc; scripts/pmc_sq_summary.py)"""
    path = os.path.join(ROOT, "profiles", "r06_pmc_sq_icp.json")
    try:
        pm = json.load(open(path))
    except Exception:
        return None
    out = {k: {f: v[f] for f in ("avg_us", "valu_busy_frac", "wait_frac", "issue_stall_frac")}
           for k, v in pm.items() if k.startswith(("icp_tile_kernel", "icp_heavy_kernel"))}
    return dict(out, source=os.path.relpath(path, ROOT)) if out else None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(args))
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # LIO_BENCH_REHEARSE=1: every rank on device 0 with gloo collectives (CPU tensors), to rehearse
    # the multi-rank path on a one-GPU box; the driver's N-GPU runs use one device per rank over RCCL
    rehearse = os.environ.get("LIO_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    coll_dev = torch.device("cpu") if rehearse else dev  # tensors handed to collectives

    from lio_gpu import frontend as F
    from lio_gpu import loop_closure as LC
    from lio_gpu import synth

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # ---------------------------------------------------------------- inputs
    t0 = time.time()
    mp, L, sp, kind = synth.CONFIGS[args.config]
    scene = synth.make_scene(L, 1234)
    mappts = synth.sample_surface(scene, mp, 1234)
    scans = []
    for k in range(args.scans):
        x = -0.15 * L + (k + rank * args.scans) * 3.7
        scans.append(synth.make_scan(scene, sp, kind, pos_gt=[x, 0.6 * np.sin(0.7 * k), 0.0],
                                     yaw_gt=0.05 * np.sin(0.3 * k), seed=99 + k + 1000 * rank))
    if os.environ.get("LIO_BENCH_PERMUTE") == "tiles":  # diagnostics: spatially tiled query order
        for sc in scans:
            b = sc.body.astype(np.float64)
            t = np.floor(b[:, :2] / float(os.environ.get("LIO_BENCH_TILE", "8"))).astype(np.int64)
            t -= t.min(axis=0)
            sc.body = np.ascontiguousarray(sc.body[np.lexsort((b[:, 2], t[:, 0], t[:, 1]))])
    gen_s = time.time() - t0
    d_map = torch.from_numpy(mappts).to(dev)
    d_scans = [torch.from_numpy(s.body).to(dev) for s in scans]
    torch.cuda.synchronize()
    tree = F.IkdTreeGPU(cell_size=args.cell, device=local)
    tb = time.time()
    tree.Build_device(d_map.data_ptr(), len(mappts))
    build_ms = (time.time() - tb) * 1e3
    hm = F.HShareModelGPU(tree)
    kf = F.EsekfGPU(hm, laser_point_cov=0.001, max_iteration=3, epsi=0.001)
    P0 = synth.initial_cov()
    states = [synth.initial_state(s.pos_init, s.rot_init) for s in scans]

    # per-scan inputs prepared once (a C++ caller of lio_ieskf_update owns its state / P the
    # same way); the timed step copies them and calls through the C-ABI without conversions
    init_c = [F.state_to_c(st) for st in states]
    s_c = type(init_c[0])()
    P_c = np.empty((23, 23))
    st_c = type(F._capi.IeskfStats())()
    ptrs = [(d.data_ptr(), len(s.body)) for d, s in zip(d_scans, scans)]

    # the C-ABI calls with their arguments prepared once (what a C++ caller's loop passes): bind the
    # resident scan, reset state and covariance, one full lio_ieskf_update
    lib_ = F._capi.lib()
    s_addr, s_size = ctypes.addressof(s_c), ctypes.sizeof(s_c)
    init_addr = [ctypes.addressof(c) for c in init_c]
    P0_c = np.ascontiguousarray(P0, dtype=np.float64)
    P_addr, P0_addr, P_bytes = P_c.ctypes.data, P0_c.ctypes.data, P_c.nbytes
    bind_args = [(hm._h, ctypes.c_void_p(p), n) for p, n in ptrs]
    upd_args = (kf.model._h, ctypes.byref(s_c), P_c.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                ctypes.byref(kf.params), ctypes.byref(st_c))
    bind_fn, upd_fn, memmove = lib_.lio_scan_bind_device, lib_.lio_ieskf_update, ctypes.memmove

    def step(k):
        j = k % len(scans)
        rc = bind_fn(*bind_args[j])  # scans stay resident in HBM (torch tensors)
        if rc:
            F.check(rc)
        memmove(s_addr, init_addr[j], s_size)
        memmove(P_addr, P0_addr, P_bytes)
        rc = upd_fn(*upd_args)
        if rc:
            F.check(rc)
        return st_c

    # C3/C5: the map is grown through the insert path (FAST-LIO map_incremental
    # after each update, filter_size_map = 0.5, kitti.launch:10) before timing
    incr = None
    if args.config in ("C3", "C5") and args.grow_scans > 0:
        grow = []
        for k in range(args.grow_scans):
            x = -0.15 * L + 1.85 + (k + rank * args.grow_scans) * 3.7
            grow.append(synth.make_scan(scene, sp, kind, pos_gt=[x, 0.6 * np.sin(0.7 * k + 0.3), 0.0],
                                        yaw_gt=0.05 * np.sin(0.3 * k + 0.2), seed=5099 + k + 1000 * rank))
        d_grow = [torch.from_numpy(s.body).to(dev) for s in grow]
        torch.cuda.synchronize()
        t_list = []
        added = 0
        for k, s in enumerate(grow):
            hm.set_scan_device(d_grow[k].data_ptr(), len(s.body))
            xg, _, _ = kf.update_iterated_dyn_share_modified(synth.initial_state(s.pos_init, s.rot_init), P0)
            ti = time.perf_counter()
            st_i = hm.map_incremental(synth.pose24(xg), 0.5)
            t_list.append(time.perf_counter() - ti)
            added += st_i["n_to_add"] + st_i["n_no_downsample"]
        incr = {"scans": len(grow), "ms_per_scan": round(sum(t_list) / len(grow) * 1e3, 3),
                "ms_per_scan_median": round(float(np.median(t_list)) * 1e3, 3),
                "points_offered_per_scan": round(added / len(grow), 1), "map_size_after": tree.size(),
                "map_ids_after": tree.num_ids()}

    # collector pauses stay out of the timed region (a C++ caller of the C-ABI has none), and the collection
    # runs BEFORE the warm-up so that the GPU has not idled (clocks down) when the first timed step starts
    gc.collect()
    gc.disable()
    # clock ramp: a fresh box's GPU can sit in a low power state for the first ~0.1-1 s of work (a 20-step run
    # measured 0.22 ms on every step there vs 0.17-0.18 after), so the W warm-ups are preceded by untimed steps
    # for --prewarm-s seconds of wall time
    t_pre = time.perf_counter() + args.prewarm_s
    k_pre = 0
    while time.perf_counter() < t_pre:
        step(k_pre)
        k_pre += 1
    for k in range(args.warmup):
        step(k)
    barrier()
    # the timed region: exactly args.steps C-ABI updates and a clock read per step, nothing else (the
    # per-step statistics come from an untimed pass over the same steps below)
    t_steps = [0.0] * (args.steps + 1)
    clock = time.perf_counter
    t_start = clock()
    t_steps[0] = t_start
    for k in range(args.steps):
        step(k)
        t_steps[k + 1] = clock()
    barrier()
    elapsed = time.perf_counter() - t_start
    gc.enable()
    t_steps = [b - a for a, b in zip(t_steps[:-1], t_steps[1:])]
    # untimed statistics pass over the same steps (the updates are deterministic per scan): host split,
    # evaluations per scan, pose error against the ground truth
    h_evals = knn_calls = 0
    capi_ms = launch_ms = wait_ms = solve_ms = 0.0
    pos_err = []
    for k in range(args.steps):
        st = step(k)
        capi_ms += st.wall_ms
        launch_ms += st.launch_ms
        wait_ms += st.wait_ms
        solve_ms += st.solve_ms
        h_evals += st.h_evals
        knn_calls += st.knn_calls
        if k < len(scans):
            pos_err.append(float(np.linalg.norm(np.array(list(s_c.pos)) - scans[k % len(scans)].pos_gt)))
    # the integration path a C++ caller takes: the scan is handed over in host memory
    # and uploaded by lio_scan_set (pinned buffer -> hipMemcpyAsync on the ctx stream) inside the step.
    # Reported beside `value`, never as it (value = inputs already resident in HBM).
    h_scans = [torch.from_numpy(s.body).pin_memory() for s in scans]
    lib = F._capi.lib()
    h_ptrs = [ctypes.cast(t.data_ptr(), ctypes.POINTER(ctypes.c_float)) for t in h_scans]

    def step_upload(k):
        j = k % len(scans)
        F.check(lib.lio_scan_set(hm._h, h_ptrs[j], len(scans[j].body)))
        ctypes.pointer(s_c)[0] = init_c[j]
        np.copyto(P_c, P0)
        kf.update_raw(s_c, P_c, st_c)

    for k in range(min(args.warmup, 5)):
        step_upload(k)
    barrier()
    t_up = time.perf_counter()
    for k in range(args.steps):
        step_upload(k)
    barrier()
    up_s = time.perf_counter() - t_up
    # kernel durations for the roofline: a separate pass with HIP events on the
    # ctx stream (events cost host time, so they stay out of the timed region)
    hm.reset_timing()
    hm.set_timing(True)
    for k in range(min(args.steps, 50)):
        step(k)
    hm.set_timing(False)
    tm = hm.timing()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_scans = args.steps * world
    value = total_scans / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    ms_per_iter = elapsed / max(h_evals, 1) * 1e3

    n_pts = sp
    knn_avg_ms = tm["knn_ms"] / max(tm["knn_launches"], 1)
    near_avg_ms = tm["near_ms"] / max(tm["near_launches"], 1)
    far_avg_ms = tm["far_ms"] / max(tm["far_launches"], 1)
    reuse_avg_ms = tm["reuse_ms"] / max(tm["reuse_launches"], 1)
    achieved = BYTES_PER_PT_KNN * n_pts / (knn_avg_ms * 1e-3) / 1e9 if tm["knn_launches"] else None
    traffic = None
    if os.path.exists(args.pmc):
        try:
            pmc = json.load(open(args.pmc))
            if pmc.get("config") == args.config:
                traffic = pmc.get("knn_hbm_bytes_per_launch")
        except Exception:
            traffic = None
    # unit of work = one kNN h-evaluation (112 B/pt), which runs as
    # knn_near_kernel + knn_far_kernel + plane_kernel back to back on the ctx
    # stream; achieved = algorithmic bytes / the sum of the three kernels' own
    # execution spans (hipExtLaunchKernel start/stop events on that stream, a
    # separate pass after the timed loop: the spans rocprofv3 reports, no gaps)
    # issue / wait breakdown of the evaluation's kernels from a separate SQ + GRBM counter pass on this config
    # (profiles/, scripts/pmc_sq_summary.py: VALU busy at 2 cycles per wave64 instruction, wait = SQ_WAIT_ANY /
    # SQ_WAVE_CYCLES, issue stall = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES)
    sq = None
    if args.config == "C3" and os.path.exists(args.pmc_sq):
        try:
            pm = json.load(open(args.pmc_sq))
            pick = {"near_first": "knn_near_kernel<false, false", "near_seeded": "knn_near_kernel<false, true",
                    "far": "knn_far_kernel", "plane": "plane_kernel", "reuse": "h_model_reuse_kernel"}
            sq = {}
            for name, pre in pick.items():
                k = next((k for k in pm if k.startswith(pre)), None)
                if k:
                    sq[name] = {f: pm[k][f] for f in ("valu_busy_frac", "wait_frac", "issue_stall_frac")}
            sq = sq or None
        except Exception:
            sq = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
                # traffic: HBM bytes per launch from a separate rocprofv3 --pmc pass (not this run)
                "traffic": traffic,
                "kernel": "kNN h-evaluation = knn_near_kernel + knn_far_kernel + plane_kernel",
                "bytes_per_launch": BYTES_PER_PT_KNN * n_pts, "avg_launch_ms": round(knn_avg_ms, 5),
                "near_kernel_avg_ms": round(near_avg_ms, 5), "far_kernel_avg_ms": round(far_avg_ms, 5),
                "plane_kernel_avg_ms": round(tm["plane_ms"] / max(tm["plane_launches"], 1), 5),
                "reuse_kernel_avg_ms": round(reuse_avg_ms, 5),
                "reuse_achieved_gbs": round(BYTES_PER_PT_REUSE * n_pts / (reuse_avg_ms * 1e-3) / 1e9, 2)
                if tm["reuse_launches"] else None,
                # NOT measured in this run: counter passes committed under profiles/ 
                "from_profile": {"traffic": _profile_meta(args.pmc) if traffic is not None else None,
                                 "sq_breakdown": sq, "sq": _profile_meta(args.pmc_sq) if sq else None}}

    line = {
        "metric": "scans/sec (100k-pt scan vs N-pt map) + ms/IESKF-iteration, 1 GPU",
        "value": round(value, 3), "unit": "scans/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "prewarm_s": args.prewarm_s, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32/f64",
        "data": "synthetic (seeded urban-canyon scene, ray-cast scans; no datasets offline)",
        "config": {"workload": f"{args.config}: {sp}-pt {kind} scan vs {mp}-pt "
                               + (f"map grown by {incr['scans']} scans (map_incremental)" if incr else "static map")
                               + ", "
                               "max_iteration=3 (<=4 h-evals/scan)",
                   "scan_points": sp, "map_points": mp, "resident_scans": len(scans),
                   "parallelism": f"replicas x{world} (front end does not shard)"},
        "ms_per_ieskf_iteration": round(ms_per_iter, 4),
        "ms_per_step_pct": {q: round(float(np.percentile(t_steps, int(q[1:]))) * 1e3, 4)
                            for q in ("p10", "p50", "p90", "p99")},  # this rank's per-step spread
        "ms_per_step_mean": round(float(np.mean(t_steps)) * 1e3, 4),
        # runs of <= 50 steps: every step's time with the resident scan it used
        "step_ms": [[k % len(scans), round(t * 1e3, 4)] for k, t in enumerate(t_steps)] if args.steps <= 50 else None,
        "capi_ms_per_scan": round(capi_ms / args.steps, 4),
        "host_ms_per_scan": {"launch": round(launch_ms / args.steps, 4), "wait": round(wait_ms / args.steps, 4),
                             "ieskf_algebra": round(solve_ms / args.steps, 4)},
        "h_evals_per_scan": round(h_evals / args.steps, 3), "knn_evals_per_scan": round(knn_calls / args.steps, 3),
        "pos_err_m": round(float(np.mean(pos_err)), 5) if pos_err else None,
        "map_build_ms": round(build_ms, 2), "input_gen_s": round(gen_s, 1),
        "upload_inclusive": {"scans_per_s": round(args.steps / up_s, 3),
                             "ms_per_step": round(up_s / args.steps * 1e3, 4),
                             "bytes_per_scan": 12 * sp,
                             "note": "scan uploaded from pinned host memory by lio_scan_set inside each step "
                                     "(rank-local; PCIe included)"},
        "roofline": roofline, "cpu_baseline": None, "loop_icp": None, "multi_stream": None, "map_incremental": incr,
        "pipeline": None, "loop_sequence": None,
    }

    # the headline is measured; the secondary keys follow.  N > 1: a watchdog prints what rank 0 has if a
    # collective of the secondary sections (the loop ICP's RCCL exchange) never returns, so a hang there
    # cannot cost the scaling run its line
    watchdog = None
    if dist is not None:
        import threading

        def _abandon():
            if rank == 0:
                line["watchdog"] = f"secondary sections abandoned after {args.watchdog_s:.0f} s"
                print(json.dumps(line), flush=True)
            os._exit(3)  # a hang is a failure: the launcher and the harness see a non-zero status

        watchdog = threading.Timer(args.watchdog_s, _abandon)
        watchdog.daemon = True
        watchdog.start()

    # ------------------------------------------------- C5 stream with its loop leg (secondary)
    pipeline = None
    if args.pipeline > 0 and rank == 0:
        from lio_gpu import pipeline as PL

        pmp, pL, psp, pkind = synth.CONFIGS["C5"]
        tg = time.time()
        pscene = synth.make_scene(pL, 1234)
        pmap = synth.sample_surface(pscene, pmp, 1234)
        stream = synth.make_loop_stream(pscene, n_out=max(args.pipeline // 2, 1), n_points=psp, kind=pkind)
        pgen = time.time() - tg
        d_pmap = torch.from_numpy(pmap).to(dev)
        ptree = F.IkdTreeGPU(cell_size=args.cell, downsample_size=0.5, device=local)
        ptree.Build_device(d_pmap.data_ptr(), len(pmap))
        fs = PL.FastLioSamStream(ptree, LC.LoopClosureConfig(), device=local)
        sweeps = [fs.process(raw, poses, end24, st0, P0, t) for raw, poses, end24, st0, t in stream]
        idx, out, _ = fs.loop(submap_range=2)
        # the loop leg's two stages timed separately (median of 5): submap assembly on the GPU
        # (transformPcd of the keyframes + voxelizePcd, host keyframes uploaded) and icpAlignment
        q = fs.keyframes[-1]
        t_sub, t_icp = [], []
        for _ in range(5):
            ta = time.perf_counter()
            src_c, dst_c = fs.lc.setSrcAndDstCloud(fs.keyframes, q.idx_, idx, 2, fs.config.voxel_res_)
            tb = time.perf_counter()
            reg = fs.lc.icpAlignment(src_c, dst_c)
            t_icp.append(time.perf_counter() - tb)
            t_sub.append(tb - ta)
        steady = sweeps[1:] if len(sweeps) > 1 else sweeps  # the first sweep allocates the stream's buffers
        med = {k: float(np.median([w["ms"][k] for w in steady])) for k in steady[0]["ms"]}
        per_sweep = float(np.median([sum(w["ms"].values()) for w in steady]))
        pipeline = {
            "config": f"C5: {len(stream)} raw {psp}-pt {pkind} sweeps ({len(stream) // 2} out, {len(stream) - len(stream) // 2} "
                      f"back 40 s later) on the {pmp}-pt map, keyframe every sweep, loop leg on the newest",
            "sweeps": len(sweeps), "raw_points": psp,
            "down_points_mean": round(float(np.mean([w["n_down"] for w in sweeps])), 1),
            "undistorted_points_mean": round(float(np.mean([w["n_undistorted"] for w in sweeps])), 1),
            "ms_per_sweep_median": round(per_sweep, 3), "sweeps_per_s": round(1e3 / per_sweep, 1),
            "stage_ms_median": {k: round(v, 3) for k, v in med.items()},
            "h_evals_per_sweep": round(float(np.mean([w["stats"]["h_evals"] for w in sweeps])), 2),
            "pos_err_m": round(float(np.mean([np.linalg.norm(w["state"]["pos"] - e[2][9:12])
                                               for w, e in zip(sweeps, stream)])), 4),
            "map_size_after": ptree.size(),
            "loop": {"query_idx": q.idx_, "closest_idx": int(idx), "is_valid": bool(reg.is_valid_),
                     "score": round(float(reg.score_), 5), "iterations": int(reg.iterations),
                     "src_points": int(len(src_c)), "dst_points": int(len(dst_c)),
                     "submaps_ms": round(float(np.median(t_sub)) * 1e3, 3),
                     "icp_ms": round(float(np.median(t_icp)) * 1e3, 3),
                     "ms": round(float(np.median(t_sub) + np.median(t_icp)) * 1e3, 3)},
            "input_gen_s": round(pgen, 1),
            "note": "host wall times; raw sweeps uploaded from host memory per sweep (PCIe included); the keyframe "
                    "stage copies feats_undistort back and builds the PosePcd on the host (fast_lio_sam glue)"}
        fs.close()
        ptree.close()
        del d_pmap
        # the same stream driven from C++ (tests/cpp/c5_stream.cpp through include/lio_gpu.hpp): no Python
        # between the stages; its own process, map and handles
        try:
            import tempfile

            with tempfile.TemporaryDirectory() as td:
                fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
                PL.write_stream_input(fin, pmap, stream, P0, submap_range=2)
                pipeline["cpp"] = PL.run_cpp_stream(fin, fout, timeout=300)
        except Exception as e:  # secondary section: report, never fail the bench line
            pipeline["cpp"] = {"error": str(e)[-300:]}
    line["pipeline"] = pipeline

    # ------------------------------------------------- the loop leg as the node runs it (secondary)
    # tests/cpp/loop_sequence.cpp: one lio_gpu::LoopClosure, keyframes_ growing by one per call, each call timed
    # like loopTimerFunc's "loop: %.1f" (fetchClosestKeyframeIdx + performLoopClosure); the LoopClosure is
    # prewarmed when the node starts (prewarm_ms: buffers at their floors, code objects loaded), so no call is
    # cold, and no call after the first may allocate (lio_alloc_count)
    loop_seq = None
    if args.loop_seq > 0 and rank == 0:
        try:
            import tempfile

            from lio_gpu import pipeline as PL

            n_back = args.loop_seq
            tg = time.time()
            kfs = PL.make_loop_keyframes(n_out=n_back, n_back=n_back)
            lgen = time.time() - tg
            with tempfile.TemporaryDirectory() as td:
                fin = os.path.join(td, "ls.bin")
                PL.write_loop_sequence(fin, kfs, range(n_back, 2 * n_back))
                lo = PL.run_loop_sequence(fin, timeout=300)
            pc = lo.pop("per_call")
            loop_seq = {
                "config": f"{2 * n_back} keyframes ({n_back} out, {n_back} back 40 s later with a growing odometry "
                          f"drift), synthetic KITTI-64 scans of {len(kfs[0].pcd_)}..{len(kfs[-1].pcd_)} points; one "
                          f"loopTimerFunc call per return keyframe (keyframes_ = keyframes[0..k]), C++ driver, PCL "
                          f"float order 2",
                **{k: (round(v, 4) if isinstance(v, float) else v) for k, v in lo.items()},
                "warm_p99_over_p50": round(lo["warm_p99_ms"] / lo["warm_p50_ms"], 3) if lo["warm_p50_ms"] > 0 else None,
                "per_call": [{"k": c["k"], "ms": round(c["ms"], 3), "closest": c["closest"], "n_src": c["n_src"],
                              "n_dst": c["n_dst"], "iterations": c["iterations"], "valid": c["valid"],
                              "submaps_ms": round(c["submaps_ms"], 3), "icp_ms": round(c["icp_ms"], 3),
                              "allocs": c["allocs"]} for c in pc],
                "input_gen_s": round(lgen, 1),
            }
        except Exception as e:  # secondary section: report, never fail the bench line
            loop_seq = {"error": str(e)[-300:]}
    line["loop_sequence"] = loop_seq

    # ------------------------------------------------- several scan streams on one GPU (secondary)
    # One stream is latency-bound (host round trip per h-evaluation); independent sensors / robots
    # can share the card. Each stream: its own map replica, ctx and HIP stream, one host thread.
    multi = None
    if args.streams and rank == 0:
        import threading

        multi = []
        for S in [int(v) for v in args.streams.split(",") if v.strip()]:
            sess = []
            for _ in range(S):
                t_s = F.IkdTreeGPU(cell_size=args.cell, device=local)
                t_s.Build_device(d_map.data_ptr(), len(mappts))
                h_s = F.HShareModelGPU(t_s)
                k_s = F.EsekfGPU(h_s, laser_point_cov=0.001, max_iteration=3, epsi=0.001)
                sess.append((t_s, h_s, k_s, type(init_c[0])(), np.empty((23, 23)), type(F._capi.IeskfStats())()))

            def run(si, n):
                _, h_s, k_s, x_s, p_s, st_s = sess[si]
                for k in range(n):
                    j = (k + si) % len(scans)
                    h_s.bind_scan_device(*ptrs[j])
                    ctypes.pointer(x_s)[0] = init_c[j]
                    np.copyto(p_s, P0)
                    k_s.update_raw(x_s, p_s, st_s)

            n_per = max(args.steps, 50)
            for si in range(S):
                run(si, 5)  # warm-up
            torch.cuda.synchronize()
            th = [threading.Thread(target=run, args=(si, n_per)) for si in range(S)]
            tm0 = time.perf_counter()
            for t in th:
                t.start()
            for t in th:
                t.join()
            torch.cuda.synchronize()
            dt = time.perf_counter() - tm0
            multi.append({"streams": S, "scans_per_s": round(S * n_per / dt, 1), "scans_per_stream": n_per})
            for t_s, h_s, k_s, *_ in sess:
                h_s.close()
            del sess

    line["multi_stream"] = multi

    # ------------------------------------------------------------- loop ICP (sharded)
    loop_icp = src = dst = None
    if not args.no_icp:
        try:
            loop_icp, src, dst = _loop_icp(args, LC, synth, local, world, rank, dist, rehearse, coll_dev, barrier, torch)
        except Exception as e:  # N > 1: an exchange failure must not cost the headline line
            if world == 1:
                raise
            import traceback

            traceback.print_exc()
            loop_icp = {"error": f"{type(e).__name__}: {e}"}

    # ------------------------------------------------------------- CPU baseline
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_py as O

        threads, how = usable_cpus()
        om = O.OracleMap(tree.points() if incr else mappts)  # the same map content as the GPU's

        def cpu_lat(nthr):
            # median per-scan latency of args.cpu_scans full IESKF updates after
            # args.cpu_warmup untimed ones, on the same scans / map the GPU step uses
            lat, its = [], 0
            for k in range(args.cpu_warmup + args.cpu_scans):
                j = k % len(scans)
                tc = time.perf_counter()
                _, _, so, _ = O.ieskf_update(om, scans[j].body, states[j], P0, threads=nthr)
                dt = time.perf_counter() - tc
                if k >= args.cpu_warmup:
                    lat.append(dt)
                    its += int(so[0])
            return float(np.median(lat)), sum(lat), its

        by_thr = {}
        for nthr in sorted({1, 3, threads}):  # 1 thread, FAST-LIO's MP_PROC_NUM = 3, all usable
            med, tot, its = cpu_lat(nthr)
            by_thr[nthr] = {"median_ms_per_scan": round(med * 1e3, 3), "scans_per_s": round(1.0 / med, 3),
                            "ms_per_iteration": round(tot / max(its, 1) * 1e3, 3)}
        top = by_thr[threads]
        if loop_icp is not None:
            # the loop ICP on the host cores: the restatement's kd-tree + float-order
            # Umeyama ICP, the whole icpAlignment (target tree built inside align, as PCL does lazily)
            # on the same C4 pair B, median of `reps` alignments per thread count
            icp_by = {}
            for nthr, reps in sorted({(1, 1), (3, 1), (threads, 3)}):
                lat = []
                pfid = O.default_icp_params()
                pfid.umeyama_float = LC.FIDELITY_ORDER  # the same float arithmetic as the GPU default
                for _ in range(reps):
                    tc = time.perf_counter()
                    ro = O.icp_align(src, dst, params=pfid, threads=nthr)
                    lat.append(time.perf_counter() - tc)
                icp_by[str(nthr)] = {"ms_per_alignment": round(float(np.median(lat)) * 1e3, 1),
                                     "iterations": int(ro["iterations"])}
            loop_icp["cpu_baseline"] = {
                "ms_per_alignment": icp_by[str(threads)]["ms_per_alignment"], "cores": threads, "kind": "port",
                "sample": f"median of 3 full icpAlignment calls on C4 pair B ({len(src)} vs {len(dst)} pts), "
                          "oracle/lio_oracle.cpp kd-tree 1-NN + float Umeyama (order "
                          f"{LC.FIDELITY_ORDER}, the GPU default) ICP with PCL's criteria, OpenMP over the "
                          f"correspondence search; {how}",
                "by_threads": icp_by, "gpu_full_ms": loop_icp.get("ms_full_icpAlignment")}
        # UndistortPcl's sin / cos: the reference calls libm, the restatement and the GPU a pinned routine;
        # count the C5 points (8 sweeps, undistorted and downsampled) the choice changes
        lm = {"undistorted_points": 0, "downsampled_points": 0, "differing_points": 0}
        try:
            pmp, pL, psp, pkind = synth.CONFIGS["C5"]
            for raw, poses, end24, _, _ in synth.make_loop_stream(synth.make_scene(pL, 1234)):
                for leaf, key in ((0.0, "undistorted_points"), (0.5, "downsampled_points")):
                    O.set_sincos_libm(False)
                    a = O.preprocess(raw, poses, end24, leaf=leaf)
                    O.set_sincos_libm(True)
                    b = O.preprocess(raw, poses, end24, leaf=leaf)
                    lm[key] += len(a)
                    lm["differing_points"] += (abs(len(a) - len(b)) + int(np.count_nonzero(np.any(
                        a[:min(len(a), len(b))].view(np.uint32) != b[:min(len(a), len(b))].view(np.uint32), axis=1))))
        finally:
            O.set_sincos_libm(False)
        cpu = {"value": top["scans_per_s"], "unit": "scans/s", "cores": threads, "kind": "port",
               "undistort_libm_vs_pinned_sincos": lm,
               "sample": f"1 / median per-scan latency of {args.cpu_scans} full IESKF updates (after "
                         f"{args.cpu_warmup} warm-ups) of {args.config} scans ({sp} pts) vs the same "
                         f"{tree.size() if incr else mp}-pt map, oracle/lio_oracle.cpp kd-tree + OpenMP, "
                         f"{threads} threads = {how}",
               "ms_per_iteration": top["ms_per_iteration"],
               "by_threads": {str(k): v for k, v in by_thr.items()},
               "host_cpus": os.cpu_count(), "cpu_model": _cpu_model()}

    if watchdog is not None:
        watchdog.cancel()
    if rank == 0:
        line.update({"cpu_baseline": cpu, "loop_icp": loop_icp, "multi_stream": multi, "pipeline": pipeline,
                     "loop_sequence": loop_seq})
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
