"""Where the drop-in API's host time goes, on the GPU box:

  python tools/api_probe.py

(1) LinearModel.step(isTraining=False) at B = 64 from numpy, as shipped; (2) its pieces; (3) eager
alternatives: p3d_serve reading x straight from pinned host memory and writing y there (zero-copy),
p3d_mse on the pinned buffers, one synchronize; the same with device buffers and explicit copies;
(4) FrameLifter as shipped (p3d_lift_sync), from mapped rows and from an OpenPose frame, vs p3d_lift
on the pinned buffers + a stream synchronize.  Prints JSON."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)


def med(fn, n=400, warm=50):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(1e6 * ts[len(ts) // 2], 2)


def main():
    import torch
    import _p3d
    import bench
    lib = _p3d.lib()
    torch.cuda.set_device(0)
    model, _ = bench.make_model(data_parallel=False, max_batch=64)
    rng = np.random.default_rng(3)
    x = rng.standard_normal((64, 32))
    t = rng.standard_normal((64, 48))
    out = {}
    out["step_eval_b64"] = med(lambda: model.step(None, x, t, 1.0, isTraining=False))
    x1, t1 = x[:1], t[:1]
    out["step_eval_b1"] = med(lambda: model.step(None, x1, t1, 1.0, isTraining=False))
    st = model._host_step_state(False, 64, 1.0)

    def replay_sync(st_):
        st_["graph"].replay()
        if st_.get("signal"):     # (a graph ending in p3d_host_signal: keep the model's count in step)
            model._hsig = (model._hsig + 1) & 0xffffffff
        torch.cuda.current_stream().synchronize()
    out["pieces"] = {
        "copyto_x_t": med(lambda: (np.copyto(st["hx_np"], x, casting="unsafe"), np.copyto(st["ht_np"], t, casting="unsafe"))),
        "graph_replay_sync": med(lambda: replay_sync(st)),
        "check_errors": med(model.check_errors),
        "out_copy": med(lambda: st["hy_np"].copy()),
        "sync_idle": med(lambda: torch.cuda.current_stream().synchronize()),
    }
    f32 = torch.float32
    hx = torch.empty((64, 32), dtype=f32, pin_memory=True)
    ht = torch.empty((64, 48), dtype=f32, pin_memory=True)
    hy = torch.empty((64, 48), dtype=f32, pin_memory=True)
    hl = torch.empty((4,), dtype=f32, pin_memory=True)
    hx.numpy()[:] = x
    ht.numpy()[:] = t
    dx = torch.empty((64, 32), dtype=f32, device="cuda")
    dt_ = torch.empty((64, 48), dtype=f32, device="cuda")
    dy = torch.empty((64, 48), dtype=f32, device="cuda")
    dl = torch.empty((4,), dtype=f32, device="cuda")
    h = model._h
    sh = _p3d.stream_handle

    def zc():
        _p3d.check(lib.p3d_serve(h, hx.data_ptr(), 64, hy.data_ptr(), sh()), "serve")
        _p3d.check(lib.p3d_mse(hy.data_ptr(), ht.data_ptr(), 64, 48, hl.data_ptr(), 0, sh()), "mse")
        torch.cuda.current_stream().synchronize()

    def zc_dev_y():
        _p3d.check(lib.p3d_serve(h, hx.data_ptr(), 64, dy.data_ptr(), sh()), "serve")
        _p3d.check(lib.p3d_mse(dy.data_ptr(), ht.data_ptr(), 64, 48, hl.data_ptr(), 0, sh()), "mse")
        hy.copy_(dy, non_blocking=True)
        torch.cuda.current_stream().synchronize()

    def copies():
        dx.copy_(hx, non_blocking=True)
        dt_.copy_(ht, non_blocking=True)
        _p3d.check(lib.p3d_serve(h, dx.data_ptr(), 64, dy.data_ptr(), sh()), "serve")
        _p3d.check(lib.p3d_mse(dy.data_ptr(), dt_.data_ptr(), 64, 48, dl.data_ptr(), 0, sh()), "mse")
        hy.copy_(dy, non_blocking=True)
        hl.copy_(dl, non_blocking=True)
        torch.cuda.current_stream().synchronize()

    def serve_only_zc():
        _p3d.check(lib.p3d_serve(h, hx.data_ptr(), 64, hy.data_ptr(), sh()), "serve")
        torch.cuda.current_stream().synchronize()

    def serve_only_dev():
        _p3d.check(lib.p3d_serve(h, dx.data_ptr(), 64, dy.data_ptr(), sh()), "serve")
        torch.cuda.current_stream().synchronize()

    ss = model._serve_step_state(64)
    if ss is not None:
        np.copyto(ss["hx_np"], x, casting="unsafe")
        np.copyto(ss["ht_np"], t, casting="unsafe")
        # the step's launch as shipped (p3d_serve_mse_sync: returns with the results in host memory)
        out["serve_mse_sync_call"] = med(ss["launch"])
        args = (h, hx.data_ptr(), 64, hy.data_ptr(), ht.data_ptr(), hl.data_ptr())
        out["serve_mse_launch_stream_sync"] = med(lambda: (lib.p3d_serve_mse(*args, sh()),
                                                           torch.cuda.current_stream().synchronize()))
    out["device_ctx"] = med(lambda: torch.cuda.device(model.device).__enter__())
    out["current_stream_sync_call"] = med(lambda: torch.cuda.current_stream(model.device).synchronize())
    ref = model.step(None, x, t, 1.0, isTraining=False)
    zc()
    a_zc = hy.numpy().copy()
    copies()
    out["eager"] = {"zero_copy_serve_mse": med(zc), "zero_copy_x_dev_y": med(zc_dev_y), "copies_serve_mse": med(copies),
                    "serve_only_zero_copy": med(serve_only_zc), "serve_only_device": med(serve_only_dev)}
    out["agree"] = {"zc_vs_copies_bitwise": bool(np.array_equal(a_zc, hy.numpy())),
                    "zc_vs_step_maxabs": float(np.abs(a_zc - ref[2]).max()),
                    "loss_zc": float(hl.numpy()[0]), "loss_step": float(ref[0])}
    # FrameLifter
    import data_utils
    import openpose_frontend
    rng2 = np.random.default_rng(600)
    use2, _ = data_utils.dimension_sets(2)
    _, ign3 = data_utils.dimension_sets(3)
    stats = (rng2.uniform(200, 600, 64), rng2.uniform(50, 150, 64), use2, rng2.uniform(-400, 400, 96),
             rng2.uniform(30, 300, 96), ign3)
    fl = openpose_frontend.FrameLifter(model, *stats, batch=1)
    e = openpose_frontend.map_frames(rng2.uniform(100, 900, (1, 36)))
    out["frontend_lift_mapped"] = med(lambda: fl.lift_mapped(e))
    # its pieces: the C call (launch + wait for the completion word), the Python around it, and the
    # same call on device-resident rows (no PCIe reads / writes inside the kernel)
    out["frontend_pieces"] = {
        "lift_sync_call": med(fl._launch),
        "asarray_store_rows": med(lambda: fl.hin_np.__setitem__(slice(0, 1), np.asarray(e, np.float64))),
        "out_copy": med(lambda: fl.hout_np[:1].copy()),
        "stream_handle": med(sh),
    }
    dargs = (h, fl.din.data_ptr(), 1, 64, fl.m2.data_ptr(), fl.s2.data_ptr(), fl.u2.data_ptr(), fl.u2.numel(),
             fl.m3.data_ptr(), fl.s3.data_ptr(), fl.u3.data_ptr(), fl.u3.numel(), 96, fl.p3.data_ptr())
    out["frontend_pieces"]["lift_sync_device_rows"] = med(lambda: lib.p3d_lift_sync(*dargs, sh()))
    out["frontend_pieces"]["lift_device_rows_stream_sync"] = med(lambda: (lib.p3d_lift(*dargs, sh()),
                                                                          torch.cuda.current_stream().synchronize()))
    raw = rng2.uniform(100, 900, (1, 36))
    out["frontend_lift_from_openpose_frame"] = med(lambda: fl.lift(raw))
    r_graph = fl.lift_mapped(e)

    def eager_lift():
        fl.hin_np[:1] = e
        openpose_frontend.lift(model, fl.hin, fl.m2, fl.s2, fl.u2, fl.m3, fl.s3, fl.u3, out=fl.hout)
        torch.cuda.current_stream().synchronize()
        return fl.hout_np[:1].copy()
    out["frontend_eager_zero_copy"] = med(eager_lift)
    out["frontend_eager_agree_bitwise"] = bool(np.array_equal(eager_lift(), r_graph))
    # host enqueue cost alone (the launch call returns before the kernel runs; synchronize untimed):
    # the empty kernel, p3d_serve at B = 64 and the headline's 1280 rows, and a trivial ABI call
    def enq(fn, n=300, warm=30):
        ts = []
        for k in range(n + warm):
            torch.cuda.current_stream().synchronize()
            t0 = time.perf_counter()
            fn()
            if k >= warm:
                ts.append(time.perf_counter() - t0)
        torch.cuda.current_stream().synchronize()
        ts.sort()
        return round(1e6 * ts[len(ts) // 2], 2)
    import ctypes
    flg = ctypes.c_int32()
    x1280 = torch.zeros((1280, 32), dtype=f32, device="cuda")
    y1280 = torch.empty((1280, 48), dtype=f32, device="cuda")
    out["enqueue"] = {"empty_kernel": enq(lambda: lib.p3d_empty_launch(h, 256, sh())),
                      "serve_b64": enq(model.serve_launcher(dx, dy)),
                      "serve_b1280": enq(model.serve_launcher(x1280, y1280)),
                      "abi_call_no_launch": enq(lambda: lib.p3d_error_flags(h, ctypes.byref(flg), 0))}
    # the training step from numpy (the captured step without copy nodes, waited on its signal word)
    xtr, ttr = rng.standard_normal((64, 32)), rng.standard_normal((64, 48))
    out["step_train_b64"] = med(lambda: model.step(None, xtr, ttr, 0.5, isTraining=True), n=200, warm=20)
    sttr = model._host_step_state(True, 64, 0.5)
    if sttr.get("signal"):
        def replay_then_wait(timed):
            t0 = time.perf_counter()
            sttr["graph"].replay()
            t1 = time.perf_counter()
            model._hsig = (model._hsig + 1) & 0xffffffff
            _p3d.check(lib.p3d_host_wait(h, model._hsig, sh()), "p3d_host_wait")
            t2 = time.perf_counter()
            model._step_host += 1
            timed.append((t1 - t0, t2 - t0))
        tt = []
        for _ in range(220):
            replay_then_wait(tt)
        tt = tt[20:]
        out["train_pieces"] = {"graph_replay_call": round(1e6 * sorted(a for a, _ in tt)[len(tt) // 2], 2),
                               "replay_to_signal": round(1e6 * sorted(b for _, b in tt)[len(tt) // 2], 2),
                               "params_changed": med(lambda: lib.p3d_params_changed(h))}
    # the same step's calls issued eagerly each step (P3D_STEP_GRAPH=0), with the signal
    os.environ["P3D_STEP_GRAPH"] = "0"
    torch.cuda.synchronize()
    model._host_steps.clear()
    out["step_train_b64_eager_signal"] = med(lambda: model.step(None, xtr, ttr, 0.5, isTraining=True), n=200, warm=20)
    del os.environ["P3D_STEP_GRAPH"]
    print(json.dumps(out), flush=True)
    model.close()


if __name__ == "__main__":
    main()
