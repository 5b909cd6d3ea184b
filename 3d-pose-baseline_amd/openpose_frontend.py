"""Per-frame lifting of the OpenPose front end, on the GPU.

src/openpose_3dpose_sandbox.py:317-356 lifts one frame at a time: map the OpenPose joints into
the 64-wide H3.6M 2D vector (``order`` of :25 plus the derived Hip / Neck-Nose / Thorax,
:336-342), normalise it with the 2D training statistics (:347-350), ``model.step`` at batch 1
(:353) and ``unNormalizeData`` of the 3D output (:356).

``FrameLifter`` runs everything after the joint mapping as ONE HIP graph per call: pinned H2D
of the mapped frame(s) -> ``p3d_lift`` (normalise, the float32 placeholder cast, the forward,
unNormalizeData: one persistent launch at batch <= 4, else ``p3d_normalize`` + the layer kernels +
``p3d_unnormalize``, the same bits) -> pinned D2H of the [B, 96] millimetre pose(s).  The mapping is
a host-side index shuffle of the OpenPose JSON values (as in the reference).  The plotting,
axis swap and Maya export that follow in the sandbox are out of scope.
"""
from __future__ import annotations

import os

import numpy as np

import data_pipeline as dp

ORDER = [15, 12, 25, 26, 27, 17, 18, 19, 1, 2, 3, 6, 7, 8]   # src/openpose_3dpose_sandbox.py:25
# the per-joint copies of the mapping as one gather: H3.6M columns 2h, 2h+1 <- OpenPose 2i, 2i+1
_SRC = np.array([2 * i + k for i in range(len(ORDER)) for k in (0, 1)])
_DST = np.array([2 * h + k for h in ORDER for k in (0, 1)])


def map_frames(frames_xy):
    """OpenPose frames [N, >= 28] (x/y interleaved) -> H3.6M 2D vectors [N, 64] float64."""
    xy = np.asarray(frames_xy, np.float64)
    if xy.ndim == 1:
        xy = xy[None, :]
    if xy.ndim != 2 or xy.shape[1] < 2 * len(ORDER):
        raise ValueError("expected OpenPose frames [N, >= %d], got %s" % (2 * len(ORDER), xy.shape))
    e = np.zeros((xy.shape[0], 64))
    e[:, _DST] = xy[:, _SRC]
    e[:, 0:2] = (e[:, 2:4] + e[:, 12:14]) / 2            # Hip = mean(RHip, LHip)
    e[:, 28:30] = (e[:, 30:32] + e[:, 24:26]) / 2        # Neck/Nose = mean(Head, Spine)
    e[:, 26:28] = 2 * e[:, 24:26] - e[:, 28:30]          # Thorax = 2 Spine - Neck/Nose
    return e


def lift(model, raw, mean2, std2, use2, mean3, std3, use3, out):
    """Device rows raw [B, 64] float64 (mapped frames) -> out [B, D3] float64 millimetres:
    normalize_data, the float32 cast, the eval forward, unNormalizeData (p3d_lift).  mean/std:
    device float64; use2/use3: device int32 dimension sets (data_pipeline._dims)."""
    import _p3d
    p = lambda t: t.data_ptr()   # noqa: E731
    _p3d.check(_p3d.lib().p3d_lift(model._h, p(raw), raw.shape[0], raw.shape[1], p(mean2), p(std2), p(use2),
                                   use2.numel(), p(mean3), p(std3), p(use3), use3.numel(), out.shape[1], p(out),
                                   model.stream()), "p3d_lift")
    return out


class FrameLifter:
    """Lift mapped OpenPose frames to 3D (mm) with a LinearModel: one p3d_lift launch per call on
    pinned host rows (fp32 models; bf16 models: one HIP graph of the three calls per call)."""

    def __init__(self, model, data_mean_2d, data_std_2d, dim_to_use_2d, data_mean_3d, data_std_3d,
                 dim_to_ignore_3d, batch=1):
        import torch
        self.torch, self.model, self.B = torch, model, int(batch)
        if self.B < 1 or self.B > model.max_batch:
            raise ValueError("batch must be in [1, max_batch=%d]" % model.max_batch)
        dev = model.device
        D3 = int(np.asarray(data_mean_3d).shape[0])
        use3 = np.setdiff1d(np.arange(D3), np.asarray(dim_to_ignore_3d, np.int64))
        if len(use3) != model.output_size or len(dim_to_use_2d) != model.input_size:
            raise ValueError("statistics do not match the model's %d inputs / %d outputs"
                             % (model.input_size, model.output_size))
        with torch.cuda.device(dev):
            self.m2, self.s2 = dp.as_device(data_mean_2d), dp.as_device(data_std_2d)
            self.m3, self.s3 = dp.as_device(data_mean_3d), dp.as_device(data_std_3d)
            self.u2 = dp._dims(dim_to_use_2d, 64, "FrameLifter")
            self.u3 = dp._dims(use3, D3, "FrameLifter")
            f32, f64 = torch.float32, torch.float64
            self.hin = torch.empty((self.B, 64), dtype=f64, pin_memory=True)
            self.hout = torch.empty((self.B, D3), dtype=f64, pin_memory=True)
            self.din = torch.empty((self.B, 64), dtype=f64, device=dev)
            self.x = torch.empty((self.B, model.input_size), dtype=f32, device=dev)
            self.y = torch.empty((self.B, model.output_size), dtype=f32, device=dev)
            self.p3 = torch.empty((self.B, D3), dtype=f64, device=dev)
            self.hin.zero_()
            self.graph, self._launch, self._host_wait = None, None, False
            if not model.bf16 and os.environ.get("P3D_LIFT_EAGER", "1") != "0":
                # fp32 (round 6): ONE p3d_lift launch per call that reads the pinned frame rows and
                # writes the pinned millimetre rows itself (mapped host memory), its ctypes
                # arguments bound once -- a graph replay costs more than the launch it would save
                import ctypes
                import _p3d
                c = ctypes.c_void_p
                args = (model._h, c(self.hin.data_ptr()), self.B, 64, c(self.m2.data_ptr()), c(self.s2.data_ptr()),
                        c(self.u2.data_ptr()), self.u2.numel(), c(self.m3.data_ptr()), c(self.s3.data_ptr()),
                        c(self.u3.data_ptr()), self.u3.numel(), D3, c(self.hout.data_ptr()))
                # p3d_lift_sync returns once the rows are in hout (the launch's output workgroups
                # store a completion word the host waits on); env P3D_HOST_WAIT=0: p3d_lift + a
                # stream synchronize
                self._host_wait = os.environ.get("P3D_HOST_WAIT", "1") != "0"
                fn, sh = (_p3d.lib().p3d_lift_sync if self._host_wait else _p3d.lib().p3d_lift), _p3d.stream_handle
                self._launch = lambda: fn(*args, c(sh()))   # noqa: E731
                _p3d.check(self._launch(), "p3d_lift")
                torch.cuda.current_stream(dev).synchronize()
            else:
                side = torch.cuda.Stream(dev)
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    self._body()                           # eager warm-up (no side effects)
                torch.cuda.current_stream(dev).wait_stream(side)
                self.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph, stream=side):
                    self._body()
        self.hin_np, self.hout_np = self.hin.numpy(), self.hout.numpy()

    def _body(self):
        self.din.copy_(self.hin, non_blocking=True)
        if self.model.bf16:
            # p3d_lift is float32-only: the three calls it folds (the same arithmetic)
            dp.normalize(self.din, self.m2, self.s2, self.u2, out_dtype=self.torch.float32, out=self.x)
            self.model.forward_device(self.x, False, 1.0, out=self.y, ctr=0)
            dp.unnormalize(self.y, self.m3, self.s3, self.u3, self.p3.shape[1], out=self.p3)
        else:
            lift(self.model, self.din, self.m2, self.s2, self.u2, self.m3, self.s3, self.u3, out=self.p3)
        self.hout.copy_(self.p3, non_blocking=True)

    def lift_mapped(self, enc_in64):
        """Mapped H3.6M 2D vectors [n <= batch, 64] -> 3D poses [n, 96] (mm, float64)."""
        e = np.asarray(enc_in64, np.float64)
        n = e.shape[0]
        if e.ndim != 2 or e.shape[1] != 64 or not 1 <= n <= self.B:
            raise ValueError("expected [1..%d, 64] mapped frames, got %s" % (self.B, e.shape))
        self.hin_np[:n] = e
        if n < self.B:
            self.hin_np[n:] = 0.0
        if self._launch is not None:
            rc = self._launch()
            if rc:
                import _p3d
                self.model.check_errors()         # (raises with the kernels' own report, if any)
                _p3d.check(rc, "p3d_lift")
            if not self._host_wait:
                self.torch.cuda.current_stream(self.model.device).synchronize()
        else:
            self.graph.replay()
            self.torch.cuda.current_stream(self.model.device).synchronize()
        return self.hout_np[:n].copy()

    def lift(self, frames_xy):
        """OpenPose frames [N, >= 28] -> 3D poses [N, 96] (mm), in calls of `batch` frames."""
        e = map_frames(frames_xy)
        if e.shape[0] <= self.B:          # (the sandbox's per-frame call: one batch)
            return self.lift_mapped(e)
        return np.concatenate([self.lift_mapped(e[i:i + self.B]) for i in range(0, e.shape[0], self.B)])
