"""Benchmark of the MI355X pose-lifting MLP (BASELINE.json metric: poses/s at batch 64).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode infer|train|eval|stress|data]

Modes (BASELINE.json configs):
  infer  (default, configs[1]) L=1024, 2 residual blocks, BN, batch 64, fp32 inference.
         One step = one forward pass over one batch of 64 poses (its own synthetic
         batch, resident in HBM).  Headline path: p3d_serve (k_serve), one persistent
         launch per <= --launch-steps steps; each XCD runs whole batch-64 steps (all six
         layers of a step on that XCD's CUs, hand-offs in its L2), steps dealt round-robin
         over the XCDs.  Beside it ("stream_chain"): the per-step kernel chain (six
         launches per step, p3d_forward_ex), S = 4 streams each replaying a HIP graph of
         steps over a private workspace slot; its single-stream rate as "single_stream".
  train  (configs[2]) same model, one step = fwd + MSE + bwd + [RCCL all-reduce] +
         TF1 Adam at batch 64 per GPU, keep_prob 0.5.
  eval   (configs[3]) evaluateActionWise sweep over a synthetic 15-action H3.6M-shaped
         test set, batches sharded across ranks, one all-reduce of per-action sums
         (also reported as "eval_sweep" beside the default infer line).
  stress (configs[4]) L=4096, 4 blocks, bf16/fp32-acc, batch 1024 inference.
  data   H3.6M train-set preprocessing on the GPU: projection into 4
         cameras, camera-frame 3D, root-centring, mean/std, normalisation, float64
         (also reported as "data_pipeline" beside the default infer line).

Multi-GPU: one process per GPU (torch.distributed.run); inference shards by batch
with no data-path collective (scaling "weak"); train is data parallel (RCCL).
Rank 0 prints ONE JSON line.  Alongside `value` it reports `roofline` (dominant
kernel timed live with hipEvent pairs, see p3d_profile_*) and `cpu_baseline`
(the numpy fp32 restatement of the TF1 path, oracle/ref_mlp.py, on the host).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)

FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix = vector peak (spec)
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (AMD's 5 PF figure is 2:1 sparse)

L, NBLK, IN, OUT, BATCH = 1024, 2, 32, 48, 64


def flops_per_pose(L=L, N=NBLK):
    """2*(32L + 2N*L^2 + 48L) GEMM FLOP per pose (forward)."""
    return 2 * (IN * L + 2 * N * L * L + OUT * L)


def _free_port():
    import dist_utils
    return dist_utils.free_port()


def launch_ranks(n, dry=False):
    """`bench.py --gpus N` outside a launcher: run N ranks of this script under
    torch.distributed.run (127.0.0.1 rendezvous, a free port) as a child process and
    return its exit code.  Rank 0 prints the JSON line."""
    import subprocess
    port = _free_port()
    argv = [a for a in sys.argv[1:] if a != "--launch-dry-run"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + argv
    if dry:
        print(json.dumps({"launch": cmd}), flush=True)
        return 0
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # RCCL over dmabuf IPC on this host driver
    return subprocess.run(cmd, env=env).returncode


def setup_dist():
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # P3D_BENCH_BACKEND=gloo (+ P3D_BENCH_DEVICE=0): rehearse the N-rank path with several
    # ranks sharing one GPU (RCCL refuses two ranks on one device); the product path is nccl
    backend = os.environ.get("P3D_BENCH_BACKEND", "nccl")
    dev = int(os.environ.get("P3D_BENCH_DEVICE", local))
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    return rank, world, dev


def init_world1_group():
    """A 1-rank RCCL process group (127.0.0.1 rendezvous) so the data-parallel train step --
    bucketed all-reduce included -- can be timed on one GPU beside the fused single-GPU step."""
    import torch
    import torch.distributed as dist
    if dist.is_initialized():
        return False
    port = _free_port()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=torch.device("cuda", torch.cuda.current_device()))
    return True


def barrier_sync(world):
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world):
    import torch
    import torch.distributed as dist
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_model(seed=1234, max_batch=BATCH, data_parallel=None):
    """Kaiming weights (LinearModel.initialize) + non-trivial BN statistics."""
    import linear_model
    m = linear_model.LinearModel(L, NBLK, True, True, False, BATCH, 1e-3, "/tmp/p3d_bench", seed=seed,
                                 max_batch=max_batch, data_parallel=data_parallel)
    rng = np.random.default_rng(2)
    bn = {}
    for name, numel, kind, _ in m.param_table:
        if name.endswith("/gamma"):
            bn[name] = rng.uniform(0.5, 1.5, numel)
        elif name.endswith("/beta") or name.endswith("/moving_mean"):
            bn[name] = rng.normal(0.0, 0.1, numel)
        elif name.endswith("/moving_variance"):
            bn[name] = rng.uniform(0.5, 2.0, numel)
    m.set_weights(bn)
    return m, None


def profile_kernels(model, fn, n_launch_max=4096):
    """Run fn() with every model kernel bracketed by hipEvent pairs -> {tag: (count, avg_us)}."""
    import ctypes
    import _p3d
    _p3d.check(_p3d.lib().p3d_profile_start(model._h, n_launch_max), "p3d_profile_start")
    fn()
    buf = ctypes.create_string_buffer(1 << 16)
    _p3d.check(_p3d.lib().p3d_profile_stop(model._h, buf, len(buf)), "p3d_profile_stop")
    out = {}
    for line in buf.value.decode().strip().splitlines():
        tag, cnt, tot, mn, mx = line.split("\t")
        out[tag] = (int(cnt), float(tot) / int(cnt), float(mn), float(mx))
    return out


def kernel_name(model, what):
    """rocprof name of the kernel the library launches for `what` (p3d_kernel_name)."""
    import ctypes
    import _p3d
    buf = ctypes.create_string_buffer(256)
    _p3d.check(_p3d.lib().p3d_kernel_name(model._h, what, buf, len(buf)), "p3d_kernel_name")
    return buf.value.decode()


def _pmc_files(config):
    """Committed rocprofv3 PMC summaries (profiles/*pmc_traffic*.json, FETCH_SIZE x2 +
    WRITE_SIZE; tools/pmc_traffic.py) measured on the configuration this run uses: every
    entry of `config` must equal the file's "__config__" (newest file first).  A figure
    measured on another configuration (e.g. 1000 steps per launch instead of 20) is never
    reported as this run's traffic."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        have = d.get("__config__", {})
        if all(have.get(k) == v for k, v in config.items()):
            yield {k: v for k, v in d.items() if k != "__config__"}


def _committed_traffic(symbol, config):
    """HBM bytes per launch of `symbol` on `config` (see _pmc_files), or None."""
    # (k_serve6's single-unit forms are named without the pair flag by p3d_kernel_name; their
    # symbols carry it: "k_serve6<4, 3, 2, 10>" is "k_serve6<4, 3, 2, 10, false>(ServeArgs)")
    alt = symbol[:-1] + ", false>" if symbol.startswith("k_serve6<") and symbol.endswith(">") else None
    for d in _pmc_files(config):
        for k, v in d.items():
            if symbol in k or (alt and alt in k):
                return v["hbm_bytes_per_launch"]
    return None


def _committed_serve_launches(kname, steps_per_launch, flop):
    """The committed rocprofv3 trace of the same command (profiles/*serve_launches.json, newest first;
    tools/serve_launches.py): rocprof's durations of the paired repeats' launches beside this
    bench's event-timed durations of the same launches in that profiled run.  The dispatch-attached
    event pair brackets ~4 us more than rocprof's kernel timestamps (an empty kernel measures ~4 us
    with the events), so the event-timed frac is the conservative one."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*serve_launches.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if not any(kname[:-1] in k for k in d.get("kernel", [])) or d.get("paired_repeats_median_us") is None:
            continue
        rp, ev = d["paired_repeats_median_us"], d.get("bench_paired_event_median_us_same_run")
        out = {"file": os.path.relpath(f, ROOT), "rocprof_median_us": rp, "event_median_us_same_run": ev,
               "frac_rocprof": round(flop / (rp * 1e-6) / 1e12 / FP32_PEAK_TFLOPS, 4)}
        if ev:
            out["frac_event_same_run"] = round(flop / (ev * 1e-6) / 1e12 / FP32_PEAK_TFLOPS, 4)
        return out
    return None


def _committed_traffic_avg(symbol, config):
    """Launch-weighted mean HBM bytes per launch over every committed kernel matching `symbol`."""
    for d in _pmc_files(config):
        hits = [v for k, v in d.items() if symbol in k]
        if hits:
            n = sum(v["launches"] for v in hits)
            return int(sum(v["hbm_bytes_per_launch"] * v["launches"] for v in hits) / max(1, n))
    return None


def cpu_baseline(mode, seconds=12.0, Lc=L, Nc=NBLK):
    """numpy fp32 restatement of the TF1 path (oracle/ref_mlp.py) on this host's cores."""
    from oracle import ref_mlp
    try:
        from threadpoolctl import threadpool_info
        threads = max([d.get("num_threads", 1) for d in threadpool_info() if d.get("user_api") == "blas"] or [1])
    except Exception:
        threads = 1
    cfg = ref_mlp.Cfg(linear_size=Lc, num_layers=Nc, residual=True, batch_norm=True)
    st = ref_mlp.init_state(cfg, seed=1, bn_seed=2)
    rng = np.random.default_rng(0)
    x = rng.standard_normal((BATCH, IN)).astype(np.float32)
    t = rng.standard_normal((BATCH, OUT)).astype(np.float32)
    fn = (lambda: ref_mlp.eval_step(st, x, t, dt=np.float32)) if mode != "train" else \
        (lambda: ref_mlp.train_step(st, x, t, 0.5, 1e-3, seed=1, dt=np.float32))
    for _ in range(3):
        fn()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()
        n += 1
    dt = time.perf_counter() - t0
    out = {"value": round(n * BATCH / dt, 1), "unit": "poses/s", "cores": int(threads), "kind": "port",
           "sample": "%d %s batches of 64 (L=%d, %d blocks, fp32 numpy restatement of src/linear_model.py), %.1f s"
                     % (n, "train-step" if mode == "train" else "inference", Lc, Nc, dt)}
    try:   # the same restatement on one core (SURVEY 8d asks for both)
        from threadpoolctl import threadpool_limits
        with threadpool_limits(limits=1):
            n1, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < seconds / 3:
                fn()
                n1 += 1
            dt1 = time.perf_counter() - t0
        out["one_core"] = {"value": round(n1 * BATCH / dt1, 1), "unit": "poses/s", "cores": 1,
                           "sample": "%d batches, %.1f s" % (n1, dt1)}
    except Exception as exc:
        out["one_core"] = {"error": repr(exc)[:200]}
    return out


def bench_cfg1(seconds=3.0, steps=400):
    """BASELINE.json configs[0]: L=256, 1 residual block, batch 64, fp32 -- the reference's
    CPU-runnable plumbing case: the numpy restatement of the TF1 path on the host (inference and
    train step) beside the HIP path on the same shapes (per-step kernel chain, one stream,
    eager launches; BN-train layers one launch each)."""
    import torch
    import linear_model
    out = {"workload": "cfg1: L=256, 1 residual block, BN, batch 64, fp32 (keep 1.0 inference, keep 0.5 train)",
           "cpu": {"infer": cpu_baseline("infer", seconds, 256, 1), "train": cpu_baseline("train", seconds, 256, 1)}}
    m = linear_model.LinearModel(256, 1, True, True, False, BATCH, 1e-3, "/tmp/p3d_bench", seed=5, max_batch=BATCH,
                                 data_parallel=False)
    rng = np.random.default_rng(7)
    X = torch.from_numpy(rng.standard_normal((steps, BATCH, IN)).astype(np.float32)).cuda()
    T = torch.from_numpy(rng.standard_normal((steps, BATCH, OUT)).astype(np.float32)).cuda()
    Y = torch.empty((BATCH, OUT), dtype=torch.float32, device="cuda")
    gpu = {}
    for mode in ("infer", "train"):
        def run(k):
            for i in range(k):
                if mode == "infer":
                    m.forward_device(X[i], False, 1.0, out=Y)
                else:
                    m.train_step_device(X[i], T[i], 0.5, out=Y)
        run(20)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        gpu[mode] = {"value": round(steps * BATCH / dt, 1), "unit": "poses/s", "ms_per_step": round(1e3 * dt / steps, 5),
                     "note": "%d eager steps, one stream" % steps}
    m.close()
    out["gpu"] = gpu
    return out


def distinct_queue_streams(n, pool=16, cycles=200_000):
    """n streams that run concurrently, i.e. are bound to n different hardware queues.

    HIP binds each stream to one of GPU_MAX_HW_QUEUES queues at first use; which one is not
    a function of creation order we can rely on (tools/dispatch_probe.hip: of streams 0..3
    only two ran concurrently, of 0, 2, 4, 6 all four).  So the binding is observed: a
    candidate joins when a spin kernel on it overlaps one on every stream already chosen."""
    import torch
    cands = [torch.cuda.Stream() for _ in range(pool)]
    for st in cands:
        with torch.cuda.stream(st):
            torch.cuda._sleep(10)
    torch.cuda.synchronize()

    def spin_time(streams):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for st in streams:
            with torch.cuda.stream(st):
                torch.cuda._sleep(cycles)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    t1 = min(spin_time([cands[0]]) for _ in range(3))
    chosen = [cands[0]]
    for c in cands[1:]:
        if len(chosen) == n:
            break
        if all(min(spin_time([c, d]) for _ in range(2)) < 1.5 * t1 for d in chosen):
            chosen.append(c)
    if len(chosen) < n:
        chosen += [c for c in cands if c not in chosen][:n - len(chosen)]
    return chosen


def bench_serve(args, rank, world):
    """K forward steps of one 64-pose batch each through p3d_serve: R persistent launches of
    K/R steps (<= --launch-steps), every step a batch of 64 of its own (x [K, 64, 32] resident
    in HBM before the timed region).  Each XCD of the chip runs whole steps -- the six
    layers of a step on its ~32 CUs, layer hand-offs in its L2 -- and the steps are dealt
    round-robin over the XCDs; rows never mix across steps (eval BN is per row)."""
    import torch
    model, _ = make_model(data_parallel=False, max_batch=BATCH)
    R = max(1, -(-args.steps // args.launch_steps))
    while args.steps % R:
        R += 1
    C = args.steps // R
    rng = np.random.default_rng(100 + rank)
    X = torch.from_numpy(rng.standard_normal((args.steps, BATCH, IN)).astype(np.float32)).cuda()
    Y = torch.empty((args.steps, BATCH, OUT), dtype=torch.float32, device="cuda")
    xs = [X[i * C:(i + 1) * C].reshape(C * BATCH, IN) for i in range(R)]
    ys = [Y[i * C:(i + 1) * C].reshape(C * BATCH, OUT) for i in range(R)]

    # the launches with their argument checks done once (LinearModel.serve_launcher)
    launch = [model.serve_launcher(xs[i], ys[i]) for i in range(R)]

    def run(k):
        for i in range(k):
            launch[i % R]()

    # untimed warmup: the W steps, and at least 5 launches (~30 ms) so the timed launches
    # run at the clock the chip holds under this load (the first launches ran 3-17 % slower:
    # profiles/r01_v14_serve_launches.json)
    wl = max(5, -(-args.warmup // C))
    run(wl)
    model.serve_check()
    # serve_check's device read runs on another queue; one more launch + synchronize puts the
    # compute queue back in the state every timed launch starts from (the first launch after
    # the read measured ~25 us slower than the median launch + synchronize round trip)
    # pre-warm: the chip's clock keeps ramping under this load for ~200 launches (~25 ms): in the
    # round-6 rocprof trace of this command the launches ran 123 us (#30), 107 (#90), 105 (#110,
    # where the timed region then sat), 102.5 (#140), 99-100 (#175-190)
    # (profiles/r06_v1_serve_launches.json); 400 launches (~45 ms) put the timed region on the plateau
    prewarm = int(os.environ.get("P3D_BENCH_PREWARM", "400"))
    run(prewarm)
    # and the timed region's own code, untimed (the first pass through it measured ~10 us
    # slower than every later one: host-side first-use costs, not GPU work)
    for _ in range(3):
        barrier_sync(world)
        run(R)
        barrier_sync(world)
    # the timed region, repeated (one sample of a ~130 us region is noise-dominated):
    # each repeat is exactly the K steps bracketed by barrier + synchronize, max over ranks; the
    # reported time is the MEDIAN repeat
    nrep = int(os.environ.get("P3D_BENCH_REPEATS", "9"))
    samples = []
    # Each repeat: barrier + synchronize, t0, the K steps, this rank's synchronize, t1, then the
    # closing barrier + synchronize; the repeat's time is the MAX over ranks of t1 - t0.  (At N > 1
    # the closing barrier is an NCCL all-reduce whose own latency -- tens of us at 8 ranks, against
    # a ~110 us region -- would otherwise sit inside every rank's interval; a slow rank still sets
    # the repeat's time through the max.  At N = 1 both orders time the same interval.)
    import torch
    for _ in range(max(1, nrep)):
        barrier_sync(world)
        t0 = time.perf_counter()
        run(R)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        barrier_sync(world)
        samples.append(max_over_ranks(t1 - t0, world))
    dt = sorted(samples)[len(samples) // 2]
    model.serve_check()
    value = world * args.steps * BATCH / dt
    # where the wall time of a launch goes (diagnostic, untimed): host enqueue of one launch,
    # one launch + synchronize round trip, synchronize of an idle device (medians)
    import torch
    def med(fn, n=30):
        ts = []
        for _ in range(n):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        return round(1e6 * sorted(ts)[len(ts) // 2], 2), [round(1e6 * v, 1) for v in ts[:3]]
    reps = [round(1e6 * v, 1) for v in samples]     # every timed repeat (value: their median)
    host = {"enqueue_us": med(lambda: run(1)), "launch_sync_us": med(lambda: (run(1), torch.cuda.synchronize())),
            "idle_sync_us": med(torch.cuda.synchronize), "timed_region_repeats_us": reps}
    if world == 1:
        host["accounting"] = serve_region_accounting(model, run, R, nrep, world)
    # dominant (only) kernel, timed live: launches carrying a start/stop event pair attached to
    # their dispatch (hipExtLaunchKernel).  avg_us = the median over the accounting's 9 paired
    # repeats of the timed region (the kernel in the timed region's own context, R launches each);
    # one more event-timed launch after them is reported beside it
    prof = profile_kernels(model, lambda: run(R))
    paired = host.get("accounting", {}).get("serve_paired")
    cnt, avg_us = (9 * R, paired["device_us"] / R) if paired else (prof["serve"][0], prof["serve"][1])
    flop = float(C * BATCH * flops_per_pose())
    achieved = flop / (avg_us * 1e-6) / 1e12
    kname = kernel_name(model, 3)
    traffic = args.traffic if args.traffic is not None else \
        _committed_traffic(kname, {"mode": "infer", "steps_per_launch": C})
    roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
            "kernel": kname + " (persistent: %d batch-64 steps per launch, whole network per XCD, fp32 MFMA 16x16x4)" % C,
            "flop_per_launch": int(flop), "steps_per_launch": C, "warmup_launches": wl, "prewarm_launches": prewarm,
            "avg_us": round(avg_us, 3),
            "avg_us_from": "median of the event-timed launches of the 9 paired timed-region repeats" if paired else
                           "one event-timed launch",
            "launches_timed": cnt, "single_launch_event_us": round(prof["serve"][1], 3),
            "rocprof_cross_check": _committed_serve_launches(kname, C, flop),
            "event_pair_avg_us": {k: round(v[1], 3) for k, v in prof.items()}, "host_us": host}
    model.close()
    return value, dt, roof


def serve_region_accounting(model, run, R, nrep, world):
    """Where the headline's timed region goes beyond its kernel, untimed.
    (a) Paired repeats: the timed region exactly as timed (barrier + synchronize, R launches,
        barrier + synchronize), each launch carrying its dispatch-attached event pair, so every
        repeat yields its region time AND its kernel's device time; gap = region - kernel.
    (b) The same round trip of an EMPTY kernel (256 workgroups, p3d_empty_launch, the same ctypes
        launch path): its region time and its own device time; overhead = region - device.
    residual = gap - overhead: what the region pays that a launch + completion of an empty kernel
    does not (0 if the headline's gap is the launch/completion round trip itself)."""
    import ctypes
    import torch
    import _p3d
    lib = _p3d.lib()
    buf = ctypes.create_string_buffer(1 << 12)

    def paired(fn, tag):
        regions, devs = [], []
        for _ in range(max(3, nrep)):
            _p3d.check(lib.p3d_profile_start(model._h, 8), "p3d_profile_start")
            barrier_sync(world)
            t0 = time.perf_counter()
            fn()
            barrier_sync(world)
            regions.append(1e6 * (time.perf_counter() - t0))
            _p3d.check(lib.p3d_profile_stop(model._h, buf, len(buf)), "p3d_profile_stop")
            tot = 0.0
            for line in buf.value.decode().strip().splitlines():
                t, cnt, us = line.split("\t")[:3]
                if t == tag:
                    tot += float(us)
            devs.append(tot)
        gaps = sorted(r - d for r, d in zip(regions, devs))
        m = lambda v: sorted(v)[len(v) // 2]   # noqa: E731
        return {"region_us": round(m(regions), 2), "device_us": round(m(devs), 2), "gap_us": round(gaps[len(gaps) // 2], 2),
                "regions_us": [round(v, 1) for v in regions], "devices_us": [round(v, 2) for v in devs]}

    empty = lambda: _p3d.check(lib.p3d_empty_launch(model._h, 256, _p3d.stream_handle()), "p3d_empty_launch")  # noqa: E731
    for _ in range(20):
        empty()
    torch.cuda.synchronize()
    e = paired(empty, "empty")
    run(3)
    torch.cuda.synchronize()
    k = paired(lambda: run(R), "serve")

    def plain(fn):   # the same region without the event pair (the headline's own form)
        regions = []
        for _ in range(max(3, nrep)):
            barrier_sync(world)
            t0 = time.perf_counter()
            fn()
            barrier_sync(world)
            regions.append(1e6 * (time.perf_counter() - t0))
        return round(sorted(regions)[len(regions) // 2], 2), [round(v, 1) for v in regions]
    eu, eus = plain(empty)
    su, sus = plain(lambda: run(R))
    # without events: timed region = kernel + (empty region - empty kernel) + residual, with both
    # kernels' device times from the paired repeats
    return {"serve_paired": k, "empty_kernel": e,
            "launch_completion_overhead_us": round(e["gap_us"], 2),
            "residual_us": round(k["gap_us"] - e["gap_us"], 2),
            "unpaired": {"serve_region_us": su, "serve_regions_us": sus, "empty_region_us": eu, "empty_regions_us": eus,
                         "launch_completion_overhead_us": round(eu - e["device_us"], 2),
                         "residual_us": round((su - k["device_us"]) - (eu - e["device_us"]), 2)},
            "note": "gap = timed region - the kernel's event-timed device time, per repeat (median); the empty "
                    "kernel's gap is the launch + completion round trip with no work; residual = serve gap - empty gap; "
                    "'unpaired' repeats both regions without the event pair (the headline's form) and subtracts the "
                    "paired repeats' device times"}


def bench_latency_b64(reps=300):
    """Launch-to-result latency of ONE batch-64 request (the reference's per-batch
    step(isTraining=False), src/linear_model.py:239-245, device-resident input): host wall time
    of issue + completion (torch.cuda.synchronize) per request, median over `reps`, and the
    device time of the kernels (dispatch-attached events), for (a) p3d_serve at B = 64 (one
    persistent launch, k_serve6 on 64 rows) and (b) the six-launch chain (p3d_forward, B = 64),
    eager and as one replayed HIP graph."""
    import torch
    model, _ = make_model(data_parallel=False, max_batch=BATCH)
    x = torch.from_numpy(np.random.default_rng(11).standard_normal((BATCH, IN)).astype(np.float32)).cuda()
    y = torch.empty((BATCH, OUT), dtype=torch.float32, device="cuda")
    flop = float(BATCH * flops_per_pose())
    serve = model.serve_launcher(x, y)
    chain = lambda: model.forward_device(x, False, 1.0, out=y, ctr=0)   # noqa: E731
    chain()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=s0):
        chain()
    torch.cuda.current_stream().wait_stream(s0)
    out = {"workload": "one batch-64 request (cfg2, BN eval, keep 1), input resident in HBM, launch to result",
           "flop_per_request": int(flop)}
    for name, fn in (("serve", serve), ("chain", chain), ("chain_graph", g.replay)):
        for _ in range(30):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        prof = profile_kernels(model, lambda: [fn() for _ in range(50)]) if name != "chain_graph" else {}
        dev = sum(v[0] * v[1] for v in prof.values()) / 50.0 if prof else None
        ent = {"median_us": round(1e6 * ts[len(ts) // 2], 2), "p10_us": round(1e6 * ts[len(ts) // 10], 2),
               "p90_us": round(1e6 * ts[(9 * len(ts)) // 10], 2)}
        if dev:
            ach = flop / (dev * 1e-6) / 1e12
            ent["device_us"] = round(dev, 2)
            ent["kernels_us"] = {k: round(v[1], 3) for k, v in prof.items()}
            ent["roofline"] = {"bound": "mfma", "achieved": round(ach, 2), "peak": FP32_PEAK_TFLOPS,
                               "unit": "TFLOP/s", "frac": round(ach / FP32_PEAK_TFLOPS, 4)}
        out[name] = ent
    out["serve"]["kernel"] = kernel_name(model, 3)
    model.serve_check()
    del g
    model.close()
    return out


def bench_infer(args, rank, world):
    """K forward steps of one 64-pose batch each.  S streams (one per hardware queue) each
    replay their own HIP graph of G/S steps over a disjoint workspace slot
    (p3d_forward_ex ws_row), so independent batches overlap on the GPU; every batch still
    runs its own six layer kernels at M = 64 and is bit-identical to a sequential
    p3d_forward.  The single-stream rate is measured too (``single_stream``)."""
    import torch
    S = args.streams
    model, _ = make_model(data_parallel=False, max_batch=BATCH * S)
    # R replay rounds of G = K / R steps (G <= --graph-steps), the G steps of a round split
    # over the S streams as evenly as possible: exactly K timed steps for any K and S
    R = max(1, -(-args.steps // args.graph_steps))
    while args.steps % R:
        R += 1
    G = args.steps // R
    rng = np.random.default_rng(100 + rank)
    X = torch.from_numpy(rng.standard_normal((G, BATCH, IN)).astype(np.float32)).cuda()
    Y = torch.empty((G, BATCH, OUT), dtype=torch.float32, device="cuda")

    def steps_eager(k, base=0):
        for i in range(k):
            model.forward_device(X[(base + i) % G], False, 1.0, out=Y[(base + i) % G], ctr=0)

    # HIP binds a stream to one of GPU_MAX_HW_QUEUES (=4) hardware queues on first use,
    # round robin; the first pool streams share queues with torch's own, so one round of
    # streams is touched first and the batch streams land on 4 distinct idle queues
    # (tools/streams_probe.py: 3.8 -> 5.6 M poses/s at 4 streams).
    if args.queue_probe:
        pool = distinct_queue_streams(S)
    else:
        spare = [torch.cuda.Stream() for _ in range(int(os.environ.get("GPU_MAX_HW_QUEUES", "4")))]
        for st in spare:
            with torch.cuda.stream(st):
                torch.zeros(16, device="cuda").add_(1)
        torch.cuda.synchronize()
        pool = None

    def capture(nstreams):
        streams = pool[:nstreams] if pool is not None else [torch.cuda.Stream() for _ in range(nstreams)]
        counts = [G // nstreams + (1 if j < G % nstreams else 0) for j in range(nstreams)]
        first = [sum(counts[:j]) for j in range(nstreams)]
        graphs = []
        for j, st in enumerate(streams):
            def body(j=j):
                for i in range(first[j], first[j] + counts[j]):
                    model.forward_device(X[i], False, 1.0, out=Y[i], ctr=0, ws_row=BATCH * j)
            with torch.cuda.stream(st):
                body()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                body()
            graphs.append(g)
        torch.cuda.synchronize()

        def replay():
            for j, st in enumerate(streams):
                with torch.cuda.stream(st):
                    graphs[j].replay()
        return replay

    def timed(fn, steps):
        for _ in range(max(1, args.warmup // G)):
            fn()
        barrier_sync(world)
        t0 = time.perf_counter()
        for _ in range(R):
            fn()
        barrier_sync(world)
        return max_over_ranks(time.perf_counter() - t0, world)

    dt = timed(capture(S), args.steps)
    value = world * args.steps * BATCH / dt
    single = None
    if S > 1:
        dt1 = timed(capture(1), args.steps)
        single = {"value": round(world * args.steps * BATCH / dt1, 1), "ms_per_step": round(1000.0 * dt1 / args.steps, 5)}

    # dominant kernel, timed live: every hidden-layer launch (k_fwd<...,1>) of 100 steps
    # issued on the model's stream in step order (the layers rotate through their weights as
    # in the timed region), each carrying a start/stop event pair attached to its dispatch
    # (hipExtLaunchKernel: the packet's own begin/end timestamps, the interval rocprofv3
    # reports).  isolated_avg_us: one layer relaunched 200x with its weights hot, for reference.
    import _p3d
    prof = profile_kernels(model, lambda: steps_eager(min(args.steps, 100)))
    cnt, avg_us = prof["fwd_hidden"][0], prof["fwd_hidden"][1]
    lay = lambda n: _p3d.check(_p3d.lib().p3d_time_layer(model._h, 1, BATCH, n, model.stream()), "p3d_time_layer")
    lay(20)
    iso_us = profile_kernels(model, lambda: lay(200))["fwd_hidden"][1]
    flop = 2.0 * BATCH * L * L          # one hidden-layer launch: [64,1024] x [1024,1024]
    achieved = flop / (avg_us * 1e-6) / 1e12
    kname = kernel_name(model, 0)
    traffic = _committed_traffic(kname, {"mode": "chain", "batch": BATCH})
    roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
            "kernel": kname + " (hidden Linear+BN+ReLU+residual, fp32 MFMA 16x16x4)",
            "flop_per_launch": int(flop), "avg_us": round(avg_us, 3), "launches_timed": cnt,
            "isolated_avg_us": round(iso_us, 3),
            "event_pair_avg_us": {k: round(v[1], 3) for k, v in prof.items()}}
    model.close()
    return value, dt, roof, single


def bench_train(args, rank, world, steps=None, warmup=None, bucket_mb=None, dp=None):
    """cfg3: K training steps (fwd + MSE + bwd + [all-reduce] + TF1 Adam/re-pack) of 64 poses
    per GPU, captured in HIP graphs (all step state is device-resident: dropout counter, lr
    decay, beta powers).  Single GPU: the fused step (Adam inside the weight-gradient launch),
    G steps per graph.  Data parallel over RCCL: G whole DP steps per graph -- the bucketed
    all-reduce(AVG) of the 17.17 MB flat gradient (buckets of ``bucket_mb``, one weight-gradient
    launch each, overlapping the rest of the backward; 0: one all-reduce after it) captured on
    the comm stream; over gloo (rehearsal: several ranks on one GPU) per-step graphs around the
    host-staged all-reduce (LinearModel.train_step_graph).  ``dp`` forces the data-parallel
    form (e.g. on a 1-rank RCCL group: the DP step's compute beside the fused single-GPU step)."""
    import torch
    import torch.distributed as dist
    steps = steps or args.steps
    warmup = warmup if warmup is not None else args.warmup
    dp = (world > 1) if dp is None else dp
    model, _ = make_model(data_parallel=dp)
    if dp:
        model.dp_buckets(args.dp_bucket_mb if bucket_mb is None else bucket_mb)
    rng = np.random.default_rng(200 + rank)
    G = 16
    while steps % G:
        G -= 1
    X = torch.from_numpy(rng.standard_normal((G, BATCH, IN)).astype(np.float32)).cuda()
    T = torch.from_numpy(rng.standard_normal((G, BATCH, OUT)).astype(np.float32)).cuda()
    Y = torch.empty((BATCH, OUT), dtype=torch.float32, device="cuda")

    def run(k):
        for i in range(k):
            model.train_step_device(X[i % G], T[i % G], args.keep, out=Y)

    gloo = dp and dist.is_initialized() and dist.get_backend() != "nccl"
    use_graph = not args.train_eager
    run(max(2, warmup // 4))
    torch.cuda.synchronize()
    mode = "eager"
    if use_graph and gloo:
        # host-staged all-reduce between a forward+backward graph and an optimizer graph per step
        steps_g = [model.train_step_graph(X[i], T[i], args.keep, out=Y) for i in range(G)]
        fn, per, mode = (lambda: [f() for f in steps_g]), G, "graph"
    elif use_graph:
        s0 = torch.cuda.Stream()
        s0.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s0):
            run(G)
        torch.cuda.current_stream().wait_stream(s0)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            run(G)
        model._step_host -= G
        fn, per, mode = graph.replay, G, "graph"
    else:
        fn, per = (lambda: run(G)), G
    for _ in range(max(1, warmup // per)):
        fn()
    barrier_sync(world)
    t0 = time.perf_counter()
    for _ in range(steps // per):
        fn()
    barrier_sync(world)
    dt = max_over_ranks(time.perf_counter() - t0, world)
    value = world * steps * BATCH / dt
    prof = profile_kernels(model, lambda: run(min(steps, 32)))
    # dominant HBM kernel: fused Adam + re-pack over the 4,291,632 trainables:
    # p, m, v read+write, g read (7 x 4 B) + Wf, Wd written (2 x 4 B per weight element)
    n_params = sum(n for _, n, k, _ in model.param_table if k == 0)
    n_w = sum(n for nm, n, k, _ in model.param_table if k == 0 and nm.split("/")[-1][0] == "w")
    if "adam_bucket" in prof:   # data parallel: each bucket's optimizer behind its all-reduce
        cnt, avg_us, _, _ = prof["adam_bucket"]
        nb = len(model._buckets or ()) or 1
        byts = 7 * 4 * n_params + 2 * 4 * n_w       # the whole model's, over the step's nb launches
        achieved = byts / (nb * avg_us * 1e-6) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": "k_adam_pack per gradient bucket (TF1 Adam + Wf/Wd re-pack, on the comm stream behind "
                          "the bucket's all-reduce, overlapping the rest of the backward), %d per step" % nb,
                "bytes_per_step": byts, "avg_us": round(avg_us, 3), "launches_timed": cnt}
    elif "adam_pack" in prof:   # data parallel: separate optimizer pass after the all-reduce
        cnt, avg_us, _, _ = prof["adam_pack"]
        byts = 7 * 4 * n_params + 2 * 4 * n_w
        achieved = byts / (avg_us * 1e-6) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": _committed_traffic("k_adam_pack", {"mode": "train", "batch": BATCH}),
                "kernel": "k_adam_pack (TF1 Adam + Wf/Wd re-pack + step advance, after the all-reduce)",
                "bytes_per_launch": byts, "avg_us": round(avg_us, 3)}
    else:
        # single GPU (p3d_train_step): Adam runs inside the weight-gradient kernels; per step
        # they read X and dZ, read m, v and W, write m, v, Wf, Wd (4 B each) -- and the TF-layout
        # master W only when the library's optimizers write it (p3d_kernel_name 6: "master", i.e.
        # --max_norm or P3D_W_MASTER=1; "packed": W is read from Wd and the master is re-derived on
        # demand, 28 B per weight element instead of 32) -- and update the biases and the previous
        # layer's BN gamma/beta (read+write w, m, v)
        w_bytes = 32 if kernel_name(model, 6) == "master" else 28
        shapes = [(IN, L)] + [(L, L)] * (2 * NBLK) + [(L, OUT)]
        byts = sum(4 * (BATCH * K + BATCH * N) + w_bytes * K * N + 4 * 6 * N for K, N in shapes)
        byts += 4 * 12 * L * (2 * NBLK + 1)          # gamma, beta of every BN layer
        multi = "wgrad_multi" in prof            # all layers in one launch
        cnt, avg_us, _, _ = prof["wgrad_multi" if multi else "wgrad"]
        per_step = 1 if multi else len(shapes)
        kname = ("k_wgrad_multi (fused TF1 Adam + Wf/Wd re-pack), all %d layers in one launch" % len(shapes)
                 if multi else "k_wgrad (fused TF1 Adam + Wf/Wd re-pack), all %d layers" % per_step)
        traffic = _committed_traffic("k_wgrad_multi" if multi else "k_wgrad", {"mode": "train", "batch": BATCH})
        achieved = byts / (per_step * avg_us * 1e-6) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kname,
                "bytes_per_step": int(byts), "weight_bytes_per_element": w_bytes,
                "avg_us": round(avg_us, 3), "launches_timed": cnt}
    roof["event_pair_avg_us"] = {k: round(v[1], 3) for k, v in prof.items()}
    # the whole step against HBM: SURVEY 8d's algorithmic bytes of one cfg3 step (parameters,
    # gradients, both Adam slots read and written: 8 x 17.17 MB) over the measured step time
    step_bytes = 8 * 4 * n_params
    ms = 1000.0 * dt / steps
    roof["step"] = {"bytes_per_step": step_bytes, "ms_per_step": round(ms, 5),
                    "achieved": round(step_bytes / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(step_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    model.close()
    return value, dt, roof, mode


def bench_eval(args, rank, world):
    """cfg4: evaluateActionWise sweep (src/predict_3dpose.py:274-298) over a synthetic
    H3.6M-shaped test set: 15 actions, N_a ~ U[20000, 40000] frames (seed 4), the
    reference's per-action n % 64 tail drop, each action's batches split contiguously
    across ranks.  One sweep = forward (BN eval, keep 1) + MSE loss + fused MPJPE of
    every batch, then one all-reduce of the [15, 19] fp64 per-action table and its copy
    to the host (the per-action numbers the reference prints).  Inputs are resident in
    HBM; independent batches are submitted --eval-chunk rows per launch."""
    import torch
    import data_utils
    import dist_utils
    import predict_3dpose
    chunk = args.eval_chunk
    model, _ = make_model(data_parallel=False, max_batch=chunk)
    rng = np.random.default_rng(4)
    nb = [int(n) // BATCH for n in rng.integers(20000, 40001, 15)]
    shares = [dist_utils.shard_range(b, rank, world) for b in nb]
    rows = [(hi - lo) * BATCH for lo, hi in shares]
    g = np.random.default_rng(40 + rank)
    X = torch.from_numpy(g.standard_normal((sum(rows), IN)).astype(np.float32)).cuda()
    Y = torch.from_numpy(g.standard_normal((sum(rows), OUT)).astype(np.float32)).cuda()
    use3, _ = data_utils.dimension_sets(3)
    sr = np.random.default_rng(3)
    mean3, std3 = np.zeros(96), np.zeros(96)
    mean3[use3] = sr.uniform(-500, 500, len(use3))
    std3[use3] = sr.uniform(50, 300, len(use3))
    accs = [predict_3dpose.MPJPE(model, mean3, std3, use3, procrustes=args.procrustes) for _ in nb]
    table = torch.zeros((len(nb), 19), dtype=torch.float64, device="cuda")

    def sweep():
        off = 0
        for a, acc in enumerate(accs):
            acc.reset()
            if rows[a]:
                predict_3dpose.run_eval_rows(model, acc, X[off:off + rows[a]], Y[off:off + rows[a]], BATCH,
                                             chunk_rows=chunk)
            off += rows[a]
            table[a, :17] = acc.joint_sum
            table[a, 17] = float(acc.frames)
            table[a, 18] = acc.loss_sum(BATCH)[0]
        dist_utils.allreduce_sum_(table)
        return table.cpu().numpy()

    for _ in range(2):
        sweep()
    reps = max(1, args.eval_reps)
    barrier_sync(world)
    t0 = time.perf_counter()
    for _ in range(reps):
        t = sweep()
    barrier_sync(world)
    dt = max_over_ranks(time.perf_counter() - t0, world) / reps
    frames = sum(nb) * BATCH
    assert int(round(t[:, 17].sum())) == frames, (t[:, 17].sum(), frames)
    errs = t[:, :17].sum(1) / (t[:, 17] * 17)
    # dominant kernel of the sweep: the large-M hidden layers (k_gemm_f32) of one whole
    # sweep, each launch timed with dispatch-attached events; FLOPs from the chunk sizes
    big_m = int(os.environ.get("P3D_BIG_M", "256"))
    prof = profile_kernels(model, sweep)
    big_rows = 0
    for r in rows:
        for s0 in range(0, r, chunk):
            n = min(chunk, r - s0)
            big_rows += n if n >= big_m else 0
    tag = "fwd_hidden_big"
    if tag in prof and big_rows:
        cnt, avg_us = prof[tag][0], prof[tag][1]
        flop = 2.0 * 2 * NBLK * big_rows * L * L        # 2N hidden layers per chunk
        ach = flop / (cnt * avg_us * 1e-6) / 1e12
        roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / FP32_PEAK_TFLOPS, 4),
                "kernel": kernel_name(model, 1) + " (hidden layers, %d-row launches)" % chunk,
                "traffic": _committed_traffic(kernel_name(model, 1), {"mode": "eval", "chunk": chunk}),
                "flop_per_launch": int(flop / cnt), "avg_us": round(avg_us, 3), "launches_timed": cnt}
    else:
        roof = None
    model.close()
    return {"workload": "cfg4 evaluateActionWise sweep: 15 actions, %d frames (tail-dropped), %s, "
                        "%d-row launches, sharded over %d rank(s)"
                        % (frames, "Protocol #2 (Procrustes)" if args.procrustes else "Protocol #1", chunk, world),
            "value": round(frames / dt, 1), "unit": "frames/s", "ms_per_sweep": round(1000.0 * dt, 3),
            "average_mm": round(float(np.mean(errs)), 6), "roofline": roof}


def bench_api(args, rank, world, n_infer=300, n_train=100):
    """API-level rates: LinearModel.step() fed numpy batches of 64 exactly as the
    reference's session.run path is (float64 host arrays -> H2D, outputs D2H, loss to host
    every step), eval and train.  Includes every host round trip; the device-resident rates
    are the headline and "train"."""
    import torch
    model, _ = make_model(data_parallel=world > 1)
    rng = np.random.default_rng(500 + rank)
    xs = [rng.standard_normal((BATCH, IN)) for _ in range(8)]
    ts = [rng.standard_normal((BATCH, OUT)) for _ in range(8)]
    out = {}
    for name, n, train, keep in (("eval", n_infer, False, 1.0), ("train", n_train, True, 0.5)):
        for i in range(10):
            model.step(None, xs[i % 8], ts[i % 8], keep, isTraining=train)
        barrier_sync(world)
        t0 = time.perf_counter()
        for i in range(n):
            model.step(None, xs[i % 8], ts[i % 8], keep, isTraining=train)
        barrier_sync(world)
        dt = max_over_ranks(time.perf_counter() - t0, world)
        out[name] = {"value": round(world * n * BATCH / dt, 1), "unit": "poses/s", "ms_per_step": round(1000.0 * dt / n, 4)}
    out["eval"]["note"] = ("one p3d_serve_mse_sync call per step: the kernel reads x / t from pinned memory, writes y and the "
                           "fused loss there and stores a completion word the host waits on")
    out["train"]["note"] = ("one step: %s" % ("the data-parallel step (eager, RCCL all-reduce), a stream synchronize"
                                               if world > 1 else
                                               "the captured step (x / t read from pinned memory, y / loss written to "
                                               "coherent host memory) replayed, its last node a host signal the host "
                                               "waits on"))
    # the OpenPose front end's per-frame call (src/openpose_3dpose_sandbox.py:317-356): B = 1
    x1, t1 = xs[0][:1], np.zeros((1, OUT))
    for i in range(20):
        model.step(None, x1, t1, 1.0, isTraining=False)
    t0 = time.perf_counter()
    n1 = 2 * n_infer
    for i in range(n1):
        model.step(None, x1, t1, 1.0, isTraining=False)
    dt = time.perf_counter() - t0
    out["eval_b1"] = {"us_per_call": round(1e6 * dt / n1, 2), "unit": "us",
                      "note": "LinearModel.step() at batch 1 from numpy: one p3d_serve_mse_sync call -- the persistent "
                              "batch-1 forward (k_gemv_chain) reads x / t from pinned memory, writes y there, its last "
                              "output workgroup reduces the loss (k_mse's order) and stores a completion word the host "
                              "waits on"}
    # device time of the batch-1 forward itself (k_gemv layers): a HIP graph of 50 forwards
    # replayed back to back (kernels + the dependent boundaries between them), and the hidden
    # layer's dispatch-attached duration against its weight stream
    x1d = torch.from_numpy(xs[0][:1].astype(np.float32)).cuda()
    y1d = torch.empty((1, OUT), dtype=torch.float32, device="cuda")
    fwd1 = lambda: model.forward_device(x1d, False, 1.0, out=y1d, ctr=0)   # noqa: E731
    for _ in range(20):
        fwd1()
    torch.cuda.synchronize()
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        for _ in range(50):
            fwd1()
    for _ in range(5):
        g1.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g1.replay()
    e1.record()
    torch.cuda.synchronize()
    dev_us = 1000.0 * e0.elapsed_time(e1) / 500
    prof = profile_kernels(model, lambda: [fwd1() for _ in range(100)])
    if "gemv_chain" in prof:   # the whole forward in one launch: every layer's weights per launch
        H = 2 * NBLK
        hb = 4 * (H * (L * L + 5 * L) + (IN * L + 5 * L) + (L * OUT + OUT)) + 4 * (IN + OUT)
        h_us, kname = prof["gemv_chain"][1], "k_gemv_chain<4, 4> (whole batch-1 forward, one launch)"
    else:
        hb = 4 * (L * L + 5 * L) + 4 * 3 * L          # weights + bias/BN vectors + x, residual, y
        h_us, kname = prof["gemv_hidden"][1], kernel_name(model, 4) + " (hidden layer, batch 1)"
    out["forward_b1"] = {
        "us_per_forward": round(dev_us, 2), "unit": "us",
        "launches": sum(v[0] for v in prof.values()) // 100,
        "note": "device time of one batch-1 forward (k_gemv_chain: the whole network in one persistent launch, "
                "every hidden layer's weight slices requested at kernel start, layer outputs handed over as "
                "data-tagged granules), graph of 50 replayed back to back",
        "layers_us": {k: round(v[1], 3) for k, v in prof.items()},
        "roofline": {"bound": "hbm", "kernel": kname,
                     "bytes_per_launch": hb, "avg_us": round(h_us, 3),
                     "achieved": round(hb / (h_us * 1e-6) / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(hb / (h_us * 1e-6) / 1e9 / 8000.0, 4), "traffic": None}}
    # the front end's whole per-frame path as one graph (openpose_frontend.FrameLifter):
    # pinned H2D of the mapped frame, normalise, 6 layers, unNormalizeData, D2H
    import data_utils
    import openpose_frontend
    rng2 = np.random.default_rng(600)
    use2, _ = data_utils.dimension_sets(2)
    _, ign3 = data_utils.dimension_sets(3)
    fl = openpose_frontend.FrameLifter(model, rng2.uniform(200, 600, 64), rng2.uniform(50, 150, 64), use2,
                                       rng2.uniform(-400, 400, 96), rng2.uniform(30, 300, 96), ign3, batch=1)
    e = openpose_frontend.map_frames(rng2.uniform(100, 900, (1, 36)))
    for i in range(20):
        fl.lift_mapped(e)
    t0 = time.perf_counter()
    for i in range(n1):
        fl.lift_mapped(e)
    dt = time.perf_counter() - t0
    raw = rng2.uniform(100, 900, (1, 36))     # an OpenPose frame: the joint mapping included
    for i in range(20):
        fl.lift(raw)
    t0 = time.perf_counter()
    for i in range(n1):
        fl.lift(raw)
    dt_op = time.perf_counter() - t0
    out["frontend_b1"] = {"us_per_frame": round(1e6 * dt / n1, 2), "unit": "us",
                          "us_per_frame_from_openpose_frame": round(1e6 * dt_op / n1, 2),
                          "note": "openpose_frontend.FrameLifter.lift_mapped: one p3d_lift_sync call per frame "
                                  "(normalise, the 6 layers as one persistent k_gemv_chain, unNormalizeData; the "
                                  "pinned frame rows read and the pinned output rows written by the kernel, which "
                                  "stores a completion word the host waits on); from_openpose_frame: lift() of a "
                                  "raw OpenPose frame, the joint mapping included"}
    del fl
    model.close()
    return out


def bench_stress(args, rank, world, steps=None, warmup=None):
    """cfg5: L=4096, 4 residual blocks, bf16 weights/activations with fp32 accumulate and
    fp32 BN, batch 1024, inference.  One step = one forward of one batch of 1024 poses."""
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    import torch
    import _p3d
    import linear_model
    Ls, Ns, Bs = 4096, 4, 1024
    model = linear_model.LinearModel(Ls, Ns, True, True, False, Bs, 1e-3, "/tmp/p3d_bench", dtype="bfloat16",
                                     seed=7, max_batch=Bs, data_parallel=False)
    rng = np.random.default_rng(2)
    bn = {}
    for name, numel, kind, _ in model.param_table:
        if name.endswith("/gamma"):
            bn[name] = rng.uniform(0.5, 1.5, numel)
        elif name.endswith("/beta") or name.endswith("/moving_mean"):
            bn[name] = rng.normal(0.0, 0.1, numel)
        elif name.endswith("/moving_variance"):
            bn[name] = rng.uniform(0.5, 2.0, numel)
    model.set_weights(bn)
    G = 8
    X = torch.from_numpy(np.random.default_rng(300 + rank).standard_normal((G, Bs, IN)).astype(np.float32)).cuda()
    Y = torch.empty((G, Bs, OUT), dtype=torch.float32, device="cuda")

    def run(k):
        for i in range(k):
            model.forward_device(X[i % G], False, 1.0, out=Y[i % G])

    run(G)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        run(G)
    steps = max(G, steps // G * G)
    for _ in range(max(1, warmup // G)):
        graph.replay()
    barrier_sync(world)
    t0 = time.perf_counter()
    for _ in range(steps // G):
        graph.replay()
    barrier_sync(world)
    dt = max_over_ranks(time.perf_counter() - t0, world)
    value = world * steps * Bs / dt
    # hidden-layer launches of 8 steps in step order (32 MB of bf16 weights per layer,
    # rotating), dispatch-attached events; isolated: one layer relaunched with hot weights
    prof = profile_kernels(model, lambda: run(G))
    reps, avg_us = prof["bf16_hidden"][0], prof["bf16_hidden"][1]
    lay = lambda n: _p3d.check(_p3d.lib().p3d_time_layer(model._h, 1, Bs, n, model.stream()), "p3d_time_layer")
    lay(5)
    iso_us = profile_kernels(model, lambda: lay(50))["bf16_hidden"][1]
    flop = 2.0 * Bs * Ls * Ls
    achieved = flop / (avg_us * 1e-6) / 1e12
    kname = kernel_name(model, 5)
    roof = {"bound": "mfma", "achieved": round(achieved, 1), "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / BF16_PEAK_TFLOPS, 4), "traffic": _committed_traffic(kname, {"mode": "stress", "batch": Bs}),
            "kernel": kname + " (hidden [1024,4096]x[4096,4096] bf16 MFMA 16x16x32 + BN/ReLU/residual)",
            "flop_per_launch": int(flop), "avg_us": round(avg_us, 3), "launches_timed": reps,
            "isolated_avg_us": round(iso_us, 3)}
    model.close()
    return value, dt, roof, steps


def bench_data(args, rank, world):
    """The H3.6M training-set preprocessing of create_2d_data / read_3d_data
    (src/data_utils.py:395-471) on the GPU: world poses of 5 subjects x 150 sequences
    (390,000 frames, H3.6M's train-set size) -> 2D projections into 4 cameras, their
    mean/std and normalisation; camera-frame 3D, root-centring, mean/std, normalisation.
    Float64 like the reference, inputs resident in HBM; every rank runs the whole set
    (replicas)."""
    import torch
    import data_pipeline as dp
    import data_utils
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from synth_cameras import synth_cameras, synth_world_poses
    rng = np.random.default_rng(77)
    subjects = (1, 5, 6, 7, 8)
    frames = args.data_frames // len(subjects)
    cams, packed, _ = synth_cameras(rng, subjects)
    W = [dp.as_device(synth_world_poses(rng, frames)).reshape(-1, 3) for _ in subjects]
    C = [dp.as_device(packed[i]) for i in range(len(subjects))]
    use2 = torch.from_numpy(data_utils.dimension_sets(2)[0].astype(np.int32)).cuda()
    use3 = torch.from_numpy(data_utils.dimension_sets(3)[0].astype(np.int32)).cuda()
    S, n = len(subjects), frames * 32
    p2 = torch.empty((S, 4, n, 2), dtype=torch.float64, device="cuda")
    c3 = torch.empty((S, 4, n, 3), dtype=torch.float64, device="cuda")
    ev = {}

    def mark(tag):
        if ev is not None and tag in ev:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev[tag].append(e)

    def step():
        mark("project0")
        for i in range(S):
            dp.project(W[i], C[i], out=p2[i])
        mark("project1")
        x2 = p2.reshape(-1, 64)
        mark("moments2_0")
        m2, s2 = dp.moments(x2)
        mark("moments2_1")
        mark("normalize2_0")
        n2 = dp.normalize(x2, m2, s2, use2)
        mark("normalize2_1")
        mark("transform0")
        for i in range(S):
            dp.world_to_camera(W[i], C[i], out=c3[i])
        mark("transform1")
        cen, root = dp.root_center(c3.reshape(-1, 96))
        mark("moments3_0")
        m3, s3 = dp.moments(cen)
        mark("moments3_1")
        n3 = dp.normalize(cen, m3, s3, use3)
        return n2, n3

    ev = None
    step()
    torch.cuda.synchronize()
    reps = args.data_reps
    barrier_sync(world)
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    barrier_sync(world)
    dt = max_over_ranks(time.perf_counter() - t0, world) / reps
    # stage timing (one instrumented pass): which kernel dominates
    ev = {k: [] for k in ("project0", "project1", "moments2_0", "moments2_1", "normalize2_0", "normalize2_1",
                          "transform0", "transform1", "moments3_0", "moments3_1")}
    step()
    torch.cuda.synchronize()
    ms = lambda a, b: ev[a][0].elapsed_time(ev[b][0])   # noqa: E731
    F2 = S * 4 * frames
    stages = {
        # algorithmic bytes: inputs read once, outputs written once
        "k_cam_points<2> (project, 5 launches)": (ms("project0", "project1"), S * (n * 24 + 4 * n * 16)),
        "k_cam_points<0> (world->camera, 5 launches)": (ms("transform0", "transform1"), S * (n * 24 + 4 * n * 24)),
        "k_col_partial x2 + k_col_final x2 (moments 3D)": (ms("moments3_0", "moments3_1"), 2 * F2 * 96 * 8),
        "k_normalize (2D)": (ms("normalize2_0", "normalize2_1"), F2 * 64 * 8 + F2 * 32 * 8),
    }
    stages["k_col_partial x2 + k_col_final x2 (moments 2D)"] = (ms("moments2_0", "moments2_1"), 2 * F2 * 64 * 8)
    # dominant kernel: k_col_partial (the longest single launch), averaged over its four launches
    # per pass (pass 1 and 2 over the 2D and the 3D matrices); the two tiny k_col_final folds
    # (D workgroups) inside the timed spans are charged to it
    name = "k_col_partial<1,2> (np.mean / np.std column sums)"
    nbytes = (2 * F2 * 64 * 8 + 2 * F2 * 96 * 8) / 4
    t_ms = (ms("moments2_0", "moments2_1") + ms("moments3_0", "moments3_1")) / 4
    ach = nbytes / (t_ms * 1e-3) / 1e9
    traffic = _committed_traffic_avg("k_col_partial", {"mode": "data", "frames": S * frames})
    out = {"workload": "H3.6M train-set preprocessing (create_2d_data + read_3d_data numerics), "
                       "%d world frames x 4 cameras, float64" % (S * frames),
           "value": round(F2 / dt, 1), "unit": "camera-poses/s", "ms_per_pass": round(1000.0 * dt, 3),
           "reps": reps,
           "stages_ms": {k: round(v[0], 4) for k, v in stages.items()},
           "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": 8000.0, "unit": "GB/s",
                        "frac": round(ach / 8000.0, 4), "traffic": traffic, "kernel": name,
                        "bytes_per_launch": int(nbytes), "avg_us": round(1000.0 * t_ms, 2),
                        "stages_ms": {k: round(v[0], 4) for k, v in stages.items()}}}
    if rank == 0 and not args.no_cpu:
        out["cpu_baseline"] = cpu_data_baseline(args.cpu_seconds / 2)
    return out


def cpu_data_baseline(seconds):
    """The oracle's numpy pipeline (oracle/ref_data.py) on sequences of one subject, as many
    as fit in ~seconds: camera-poses/s, one host core (numpy is single-threaded here)."""
    from oracle import ref_data
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from synth_cameras import synth_cameras, synth_world_poses
    rng = np.random.default_rng(78)
    cams, _, _ = synth_cameras(rng, (1,))
    seq = {(1, "Walking", "Walking %d.h5" % i): synth_world_poses(rng, 2600) for i in range(4)}
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        p2 = ref_data.project_to_cameras(seq, cams)
        x2 = np.vstack(list(p2.values()))
        m2, s2 = ref_data.moments(x2)
        use2 = np.flatnonzero(s2 > 0)
        _ = (x2[:, use2] - m2[use2]) / s2[use2]
        c3 = ref_data.transform_world_to_camera(seq, cams)
        cen, _ = ref_data.postprocess_3d(c3)
        x3 = np.vstack(list(cen.values()))
        m3, s3 = ref_data.moments(x3)
        use3 = np.flatnonzero(s3 > 0)
        _ = (x3[:, use3] - m3[use3]) / s3[use3]
        done += x2.shape[0]
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 1), "unit": "camera-poses/s", "cores": 1, "kind": "port",
            "sample": "%d camera-poses (4 sequences x 2600 frames x 4 cameras per pass), %.1f s" % (done, dt)}


def model_bucket_mb(args, world):
    """The gradient-bucket size a DP run uses: --dp-bucket-mb if given, else the library's policy
    (LinearModel.dp_buckets: none -- one all-reduce after the backward -- unless P3D_DP_BUCKET_MB)."""
    if args.dp_bucket_mb is not None:
        return args.dp_bucket_mb
    return float(os.environ.get("P3D_DP_BUCKET_MB", "0"))


def run_dp1_child(args, timeout=300):
    """Run the 1-rank data-parallel train leg as `bench.py --dp1-child` (a fresh process; the
    caller has not initialised the GPU) and return its JSON, or {"error": ...}."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--dp1-child", "--train-steps", str(args.train_steps),
           "--keep", str(args.keep)]
    if args.dp_bucket_mb is not None:
        cmd += ["--dp-bucket-mb", str(args.dp_bucket_mb)]
    if args.train_eager:
        cmd.append("--train-eager")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "dp1 child timed out after %d s" % timeout}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode == 0 and lines:
        try:
            return json.loads(lines[-1])
        except ValueError:
            pass
    return {"error": "dp1 child rc %d" % r.returncode, "stderr_tail": r.stderr[-1500:]}


def dp1_child(args, json_fd):
    """The 1-rank RCCL data-parallel step (bench_train(dp=True) on a world-1 process group): the
    whole DP step -- buckets, the library's RCCL all-reduce, per-bucket Adam -- as HIP graphs."""
    import torch.distributed as dist
    import dist_utils
    import torch
    torch.cuda.set_device(0)
    init_world1_group()
    dv, ddt, droof, dmode = bench_train(args, 0, 1, steps=args.train_steps, warmup=64, dp=True)
    bk = model_bucket_mb(args, 1)
    form = ("%g MB gradient buckets, one weight-gradient launch each, RCCL all-reduce from libp3d's own "
            "communicator on its comm stream, each bucket's TF1 Adam + re-pack behind its all-reduce on the "
            "compute stream" % bk) if bk > 0 else (
            "one gradient-only weight-gradient launch, the RCCL all-reduce of the flat gradient from libp3d's own "
            "communicator, TF1 Adam + re-pack behind it (the library's bucket policy on a 1-rank group: no "
            "buckets, nothing to overlap)")
    out = {"workload": "the data-parallel step (fwd + bwd, %s; step advance in the last launch; 1-rank group: the "
                       "reduction is the identity)" % form,
           "value": round(dv, 1), "unit": "poses/s", "mode": dmode,
           "ms_per_step": round(1000.0 * ddt / args.train_steps, 5),
           "event_pair_avg_us": droof.get("event_pair_avg_us")}
    # the forms a rank of an N > 1 run can execute (P3D_DP_FORCE_MULTI), forced on this
    # 1-rank group, so what they time is each form's per-rank cost without any xGMI transfer:
    #   n_gt_1_form (the default): one ncclAllReduce(ncclAvg) of the flat gradient on the compute
    #     stream after the backward, then one TF1 Adam + re-pack pass;
    #   n_gt_1_bucketed: 8 MB buckets, the comm-stream fork, one ncclAllReduce(ncclAvg) per bucket
    #     behind its gradient-ready event, the joins, each bucket's Adam on the compute stream
    if os.environ.get("P3D_DP_FORCE_MULTI") is None:
        os.environ["P3D_DP_FORCE_MULTI"] = "1"
        try:
            for key, bmb in (("n_gt_1_form", 0.0), ("n_gt_1_bucketed", 8.0)):
                mv, mdt, mroof, mmode = bench_train(args, 0, 1, steps=args.train_steps, warmup=64, dp=True,
                                                    bucket_mb=bmb)
                form = ("one ncclAllReduce(ncclAvg) of the flat gradient on the compute stream after the backward, "
                        "one TF1 Adam + re-pack pass (the default)" if bmb == 0 else
                        "%g MB buckets, comm-stream fork, per-bucket ncclAllReduce(ncclAvg) behind the gradient-ready "
                        "events, joins, per-bucket TF1 Adam on the compute stream" % bmb)
                out[key] = {
                    "workload": "the N > 1 data-parallel step forced on the 1-rank group (P3D_DP_FORCE_MULTI=1): "
                                "%s, one HIP graph" % form,
                    "value": round(mv, 1), "unit": "poses/s", "mode": mmode,
                    "ms_per_step": round(1000.0 * mdt / args.train_steps, 5),
                    "event_pair_avg_us": mroof.get("event_pair_avg_us")}
        finally:
            del os.environ["P3D_DP_FORCE_MULTI"]
    dist_utils.close_native_comms()
    dist.destroy_process_group()
    sys.stdout.flush()
    os.write(json_fd, (json.dumps(out) + "\n").encode())
    return 0


def build_arg_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--mode", choices=["infer", "train", "eval", "stress", "data"], default="infer")
    ap.add_argument("--graph-steps", type=int, default=240)
    ap.add_argument("--launch-steps", type=int, default=1000, help="batch-64 steps per persistent p3d_serve launch")
    ap.add_argument("--no-streams", action="store_true", help="skip the per-step kernel-chain sub-measurement")
    ap.add_argument("--streams", type=int, default=4, help="independent batch streams (inference)")
    ap.add_argument("--queue-probe", type=int, default=0,
                    help="pick the inference streams by observed hardware-queue concurrency")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--train-eager", action="store_true", help="train steps without HIP graphs")
    ap.add_argument("--no-dp1", action="store_true", help="skip the 1-rank data-parallel train form (infer mode)")
    ap.add_argument("--train-steps", type=int, default=400, help="train sub-measurement (infer mode)")
    ap.add_argument("--keep", type=float, default=0.5, help="dropout keep_prob of the train step")
    ap.add_argument("--dp-bucket-mb", type=float, default=None,
                    help="data-parallel gradient all-reduce bucket (MB) overlapping the backward; 0 = one all-reduce "
                         "after the backward (default: the library's policy, P3D_DP_BUCKET_MB or 0)")
    ap.add_argument("--eval-chunk", type=int, default=8192, help="rows per launch in the cfg4 sweep")
    ap.add_argument("--eval-reps", type=int, default=5)
    ap.add_argument("--no-eval", action="store_true", help="skip the cfg4 sweep sub-measurement (infer mode)")
    ap.add_argument("--no-api", action="store_true", help="skip the LinearModel.step() API-level rates (infer mode)")
    ap.add_argument("--procrustes", action="store_true", help="cfg4 sweep with Protocol #2 alignment")
    ap.add_argument("--no-data", action="store_true", help="skip the H3.6M preprocessing sub-measurement")
    ap.add_argument("--no-stress", action="store_true", help="skip the cfg5 bf16 sub-measurement (infer mode)")
    ap.add_argument("--stress-steps", type=int, default=64, help="cfg5 batches of 1024 timed (infer mode)")
    ap.add_argument("--data-frames", type=int, default=390000)
    ap.add_argument("--data-reps", type=int, default=10)
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes/launch of the dominant kernel from rocprofv3 PMC (profiles/)")
    ap.add_argument("--dp1-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="print the N-rank launch command --gpus N > 1 would run, and exit")
    return ap


def main():
    ap = build_arg_parser()
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start N fresh ranks and wait for them.  This process touches
        # no GPU (never re-exec a process that has initialised one).
        return launch_ranks(args.gpus, dry=args.launch_dry_run)
    if args.gpus != int(os.environ.get("WORLD_SIZE", "1")):
        raise SystemExit("bench.py: --gpus %d but the job has %s rank(s) (WORLD_SIZE)"
                         % (args.gpus, os.environ.get("WORLD_SIZE", "1")))
    # everything the libraries print (RCCL's banner at communicator creation, ...) goes to
    # stderr: stdout carries exactly the one JSON line
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if args.dp1_child:
        return dp1_child(args, json_fd)
    # the data-parallel step's form on a 1-rank RCCL group (what every rank runs at N > 1), in a
    # child process that runs BEFORE this one touches the GPU: whatever happens to it (a fault, an
    # abort from a runtime thread) cannot take the headline line with it
    dp1 = None
    if (args.mode == "infer" and int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_dp1
            and args.train_steps > 0):
        dp1 = run_dp1_child(args)
    rank, world, local = setup_dist()
    train = single = sweep = api = data = stress = lat = None
    chain = None
    if args.mode == "infer":
        value, dt, roof = bench_serve(args, rank, world)
        workload = ("cfg2 inference: L=1024, 2 residual blocks, BN(eval), keep=1; a step = one batch-64 request "
                    "(its own 64 poses); %d requests per persistent p3d_serve launch (%d rows, whole network "
                    "per XCD); one request alone: latency_b64" % (roof["steps_per_launch"], 64 * roof["steps_per_launch"]))
        try:
            lat = bench_latency_b64()
        except Exception as exc:
            lat = {"error": repr(exc)[:300]}
        if not args.no_streams:   # the per-step kernel chain (six launches per step), 4 streams
            try:
                cv, cdt, croof, single = bench_infer(args, rank, world)
                chain = {"workload": "same steps as six kernel launches each (p3d_forward_ex), %d stream(s) "
                                     "of HIP graphs" % args.streams,
                         "value": round(cv, 1), "unit": "poses/s", "ms_per_step": round(1000.0 * cdt / args.steps, 5),
                         "roofline": croof}
            except Exception as exc:
                chain = {"error": repr(exc)[:300]}
        if args.train_steps > 0:   # cfg3 beside the headline, same ranks (data parallel)
            try:
                tv, tdt, troof, tmode = bench_train(args, rank, world, steps=args.train_steps, warmup=64)
                train = {"workload": "cfg3 train step (fwd+bwd+TF1 Adam), batch 64/GPU, keep 0.5, dp%d" % world,
                         "value": round(tv, 1), "unit": "poses/s", "steps": args.train_steps,
                         "ms_per_step": round(1000.0 * tdt / args.train_steps, 5), "mode": tmode,
                         "roofline": troof}
            except Exception as exc:  # report, never lose the headline line
                train = {"error": repr(exc)[:300]}
            if dp1 is not None:
                train["dp_form_1rank"] = dp1
            if world > 1 and "error" not in train:
                # the other N > 1 form on the same ranks: 8 MB buckets overlapping the backward when
                # the run used one all-reduce after it (the default), else that single all-reduce
                alt = 8.0 if model_bucket_mb(args, world) == 0 else 0.0
                key = "bucketed_8mb" if alt else "single_allreduce"
                try:
                    sv, sdt, _, _ = bench_train(args, rank, world, steps=args.train_steps, warmup=64, bucket_mb=alt)
                    train["dp_bucket_mb"] = model_bucket_mb(args, world)
                    train[key] = {"value": round(sv, 1), "unit": "poses/s",
                                  "ms_per_step": round(1000.0 * sdt / args.train_steps, 5)}
                except Exception as exc:
                    train[key] = {"error": repr(exc)[:300]}
        if not args.no_eval:
            try:
                sweep = bench_eval(args, rank, world)
            except Exception as exc:
                sweep = {"error": repr(exc)[:300]}
        if not args.no_api:
            try:
                api = bench_api(args, rank, world)
            except Exception as exc:
                api = {"error": repr(exc)[:300]}
        if not args.no_data:
            try:
                data = bench_data(args, rank, world)
            except Exception as exc:
                data = {"error": repr(exc)[:300]}
        if not args.no_stress:   # cfg5 beside the headline (bf16 / fp32-accumulate stress config)
            try:
                sv, sdt, sroof, ssteps = bench_stress(args, rank, world, steps=args.stress_steps, warmup=32)
                stress = {"workload": "cfg5 inference: L=4096, 4 residual blocks, BN(eval), batch 1024 per step, "
                                      "bf16 weights/activations, fp32 accumulate", "value": round(sv, 1),
                          "unit": "poses/s", "steps": ssteps, "ms_per_step": round(1000.0 * sdt / ssteps, 5),
                          "dtype": "bf16", "roofline": sroof}
            except Exception as exc:
                stress = {"error": repr(exc)[:300]}
    elif args.mode == "eval":
        sweep = bench_eval(args, rank, world)
        value, dt, roof = sweep["value"], sweep["ms_per_sweep"] / 1000.0, sweep.pop("roofline")
        args.steps = 1
        workload = sweep["workload"]
    elif args.mode == "data":
        data = bench_data(args, rank, world)
        value, roof = data["value"], data.pop("roofline")
        args.steps = data["reps"]
        dt = data["ms_per_pass"] / 1000.0 * args.steps
        workload = data["workload"]
    elif args.mode == "stress":
        value, dt, roof, args.steps = bench_stress(args, rank, world)
        workload = "cfg5 inference: L=4096, 4 residual blocks, BN(eval), batch 1024 per step, bf16/fp32-acc"
    else:
        value, dt, roof, tmode = bench_train(args, rank, world)
        workload = ("cfg3 train step: L=1024, 2 residual blocks, BN, dropout keep 0.5, batch 64/GPU, TF1 Adam "
                    "(%s)" % tmode)
    if rank == 0:
        if args.mode == "data":
            cpu = data.pop("cpu_baseline", None)
        elif args.mode == "stress" or args.no_cpu:
            cpu = None
        else:
            cpu = cpu_baseline(args.mode, args.cpu_seconds)
        cfg1 = bench_cfg1() if (args.mode == "infer" and not args.no_cpu and world == 1) else None
        metric = {"stress": "poses/sec at batch 1024 (cfg5 bf16 stress)",
                  "eval": "frames/sec, evaluateActionWise MPJPE sweep (cfg4)",
                  "data": "camera-poses/sec, H3.6M train-set preprocessing (float64)"}.get(
                      args.mode, "poses/sec at batch 64 (H3.6M 16-joint)")
        unit = {"eval": "frames/s", "data": "camera-poses/s"}.get(args.mode, "poses/s")
        line = {"metric": metric, "value": round(value, 1), "unit": unit,
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(1000.0 * dt / args.steps, 5), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None,
                "dtype": {"stress": "bf16", "data": "f64"}.get(args.mode, "f32"),
                "data": "synthetic",
                "config": ({"workload": workload, "global_batch": BATCH * world, "linear_size": L,
                            "num_layers": NBLK, "parallelism": "dp%d" % world} if args.mode != "stress" else
                           {"workload": workload, "global_batch": 1024 * world, "linear_size": 4096,
                            "num_layers": 4, "parallelism": "dp%d" % world}),
                "roofline": roof, "cpu_baseline": cpu}
        if lat is not None:
            line["latency_b64"] = lat
        if chain is not None:
            line["stream_chain"] = chain
        if single is not None:
            line["single_stream"] = single
        if train is not None:
            line["train"] = train
        if sweep is not None and args.mode != "eval":
            line["eval_sweep"] = sweep
        if api is not None:
            line["api_step"] = api
        if data is not None and args.mode != "data":
            line["data_pipeline"] = data
        if stress is not None:
            line["stress"] = stress
        if cfg1 is not None:
            line["cfg1"] = cfg1
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    if world > 1:
        import torch.distributed as dist
        import dist_utils
        dist_utils.close_native_comms()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
