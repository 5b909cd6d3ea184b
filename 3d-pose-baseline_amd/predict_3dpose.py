"""Driver / API of src/predict_3dpose.py on the MI355X-native model.

Keeps: ``FLAGS`` (same flag names and defaults, src/predict_3dpose.py:31-107),
the hyper-parameter-encoded ``train_dir`` (:110-123), ``create_model`` (:131-186),
the epoch ``train`` loop (:188-334), ``get_action_subset`` (:337-349) and
``evaluate_batches`` (:352-444).  Differences, all documented in DESIGN.md:

* flags are parsed in ``main`` (the reference parses argv at import time); an
  importable ``FLAGS`` object holds the defaults so front ends can import it;
* the per-frame MPJPE (un-normalize, 17 joints, per-joint L2) runs on the GPU in
  one fused kernel, accumulating fp64 per-joint sums on the device;
* ``evaluate_action_wise`` shards each action's batches across the ranks of a
  ``torch.distributed`` job and combines per-action sums with one RCCL
  all-reduce;
* the H3.6M tree and cameras.h5 are read as the reference's HDF5 files (h5py) or as .npz
  archives of the same datasets under the same paths (``load_data``); ``--synthetic`` feeds
  data of the reference's shapes without files.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

import _p3d
import cameras
import data_utils
import dist_utils
import linear_model
from _p3d import check, lib, ptr


def build_parser():
    p = argparse.ArgumentParser()
    p.add_argument("--learning_rate", type=float, default=1.0, help="Learning rate")
    p.add_argument("--dropout", type=float, default=1, help="Dropout keep probability. 1 means no dropout")
    p.add_argument("--batch_size", type=int, default=64, help="Batch size to use during training")
    p.add_argument("--epochs", type=int, default=200, help="How many epochs we should train for")
    p.add_argument("--camera_frame", action='store_true', default=False, help="Convert 3d poses to camera coordinates")
    p.add_argument("--max_norm", action='store_true', default=False, help="Apply maxnorm constraint to the weights")
    p.add_argument("--batch_norm", action='store_true', default=False, help="Use batch_normalization")
    p.add_argument("--predict_14", action='store_true', default=False, help="predict 14 joints")
    p.add_argument("--use_sh", action='store_true', default=False, help="Use 2d pose predictions from StackedHourglass")
    p.add_argument("--action", type=str, default="All", help="The action to train on. 'All' means all the actions")
    p.add_argument("--linear_size", type=int, default=1024, help="Size of each model layer.")
    p.add_argument("--num_layers", type=int, default=2, help="Number of layers in the model.")
    p.add_argument("--residual", action='store_true', default=False, help="Whether to add a residual connection every 2 layers")
    p.add_argument("--procrustes", action='store_true', default=False, help="Apply procrustes analysis at test time")
    p.add_argument("--evaluateActionWise", action='store_true', default=False, help="The dataset to use either h36m or heva")
    p.add_argument("--cameras_path", type=str, default="data/h36m/cameras.h5", help="Directory to load camera parameters")
    p.add_argument("--data_dir", type=str, default="data/h36m/", help="Data directory")
    p.add_argument("--train_dir", type=str, default="experiments", help="Training directory.")
    # openpose front ends (src/predict_3dpose.py:76-91; read by src/openpose_3dpose_sandbox.py:240-446)
    p.add_argument("--pose_estimation_json", type=str, default="/tmp/",
                   help="pose estimation json output directory, openpose or tf-pose-estimation")
    p.add_argument("--interpolation", action='store_true', default=False, help="interpolate openpose json")
    p.add_argument("--multiplier", type=float, default=0.1, help="interpolation frame range")
    p.add_argument("--write_gif", action='store_true', default=False, help="write final anim gif")
    p.add_argument("--gif_fps", type=int, default=30, help="output gif framerate")
    p.add_argument("--verbose", type=int, default=2, help="0:Error, 1:Warning, 2:INFO*(default), 3:debug")
    p.add_argument("--cache_on_fail", action='store_true', default=True,
                   help="caching last valid frame on invalid frame")
    p.add_argument("--sample", action='store_true', default=False, help="Set to True for sampling.")
    p.add_argument("--use_cpu", action='store_true', default=False, help="Whether to use the CPU")
    p.add_argument("--load", type=int, default=0, help="Try to load a previous checkpoint.")
    p.add_argument("--use_fp16", action='store_true', default=False, help="Train using fp16 instead of fp32.")
    # build-specific
    p.add_argument("--synthetic", action='store_true', default=False,
                   help="Use synthetic H3.6M-shaped data (the dataset is not part of this build)")
    p.add_argument("--seed", type=int, default=0, help="Weight / dropout seed")
    p.add_argument("--max_batch", type=int, default=8192,
                   help="rows the device workspaces hold (evaluation submits up to this many rows per "
                        "launch); front ends stepping single frames can pass their batch size")
    p.add_argument("--device_loop", type=int, default=1,
                   help="1: stage each epoch in HBM and train without per-step host round trips; "
                        "0: the reference's per-batch step() loop")
    return p


FLAGS = build_parser().parse_args([])   # defaults; main() re-parses argv


def train_dir_for(flags):
    """Hyper-parameter-encoded train_dir (src/predict_3dpose.py:110-123)."""
    return os.path.join(flags.train_dir, flags.action, 'dropout_{0}'.format(flags.dropout),
                        'epochs_{0}'.format(flags.epochs) if flags.epochs > 0 else '',
                        'lr_{0}'.format(flags.learning_rate),
                        'residual' if flags.residual else 'not_residual',
                        'depth_{0}'.format(flags.num_layers), 'linear_size{0}'.format(flags.linear_size),
                        'batch_size_{0}'.format(flags.batch_size),
                        'procrustes' if flags.procrustes else 'no_procrustes',
                        'maxnorm' if flags.max_norm else 'no_maxnorm',
                        'batch_normalization' if flags.batch_norm else 'no_batch_normalization',
                        'use_stacked_hourglass' if flags.use_sh else 'not_stacked_hourglass',
                        'predict_14' if flags.predict_14 else 'predict_17')


class Session:
    """Minimal stand-in for tf.Session: a context manager whose ``run`` evaluates the
    few graph handles callers fetch outside ``step`` (err_mm_summary)."""

    def __init__(self, *args, **kwargs):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def run(self, fetches, feed_dict=None):
        feed_dict = feed_dict or {}
        if isinstance(fetches, tuple) and fetches and fetches[0] == "summary":
            val = next(iter(feed_dict.values()))
            return linear_model.Summary(fetches[1], val)
        if hasattr(fetches, "eval"):
            return fetches.eval()
        raise NotImplementedError("Session.run: unsupported fetch %r" % (fetches,))


def create_model(session, actions, batch_size, flags=None, load_exact=False):
    """src/predict_3dpose.py:131-186: build the model, init fresh or restore --load."""
    flags = flags or FLAGS
    tdir = train_dir_for(flags)
    if flags.use_fp16:
        raise ValueError("--use_fp16 is not supported by this build (fp32 graph)")
    model = linear_model.LinearModel(flags.linear_size, flags.num_layers, flags.residual, flags.batch_norm,
                                     flags.max_norm, batch_size, flags.learning_rate,
                                     os.path.join(tdir, "log"), flags.predict_14, seed=flags.seed,
                                     max_batch=max(batch_size, getattr(flags, "max_batch", 8192)))
    if flags.load <= 0:
        print("Creating model with fresh parameters.")
        return model
    # src/predict_3dpose.py:163-181, including its behaviour: --load N checks that
    # checkpoint-N.index exists, then restores the checkpoint the directory's `checkpoint` file
    # names as the latest (ckpt.model_checkpoint_path, :180) -- not necessarily N.  Pass
    # load_exact=True (a keyword of this build) to restore checkpoint-N itself.
    # A directory of an earlier build's checkpoint-N.npz files has no `checkpoint` state file:
    # there N itself is restored.
    import tf_bundle
    latest = tf_bundle.read_checkpoint_state(tdir)
    ck = os.path.join(tdir, "checkpoint-{0}".format(flags.load))
    have = os.path.isfile(ck + ".index") or os.path.isfile(ck + ".npz")
    if latest is None and not have:
        raise ValueError("Checkpoint directory {0} does not seem to hold a checkpoint".format(tdir))
    if not have:
        raise ValueError("Asked to load checkpoint {0}, but it does not seem to exist".format(flags.load))
    path = ck if (load_exact or latest is None) else latest
    print("Loading model {0}".format(os.path.basename(ck)))
    model.saver.restore(session, path)
    return model


def get_action_subset(poses_set, action):
    """src/predict_3dpose.py:337-349."""
    return {k: v for k, v in poses_set.items() if k[1] == action}


class MPJPE:
    """Device accumulator of per-joint L2 sums (p3d_mpjpe_accum_ex), fp64.

    17-joint protocol (root prepended, 48 used dims) or --predict_14 (14 joints, 42 dims);
    --procrustes aligns every predicted frame to its target first (Protocol #2,
    src/predict_3dpose.py:413-421)."""

    def __init__(self, model, data_mean_3d, data_std_3d, dim_to_use_3d, predict_14=False, procrustes=False):
        import torch
        self.torch = torch
        self.model = model
        self.J = 14 if predict_14 else 17
        self.D = 3 * self.J if predict_14 else 3 * (self.J - 1)
        self.procrustes = bool(procrustes)
        dev = model.device
        self.mean = torch.as_tensor(np.asarray(data_mean_3d, np.float64), device=dev)
        self.std = torch.as_tensor(np.asarray(data_std_3d, np.float64), device=dev)
        self.dims = torch.as_tensor(np.asarray(dim_to_use_3d, np.int32), device=dev)
        if self.mean.numel() != 96 or self.std.numel() != 96 or self.dims.numel() != self.D:
            raise ValueError("MPJPE expects 96-d mean/std and %d used dims" % self.D)
        if model.output_size != self.D:
            raise ValueError("model predicts %d dims, the %d-joint protocol needs %d"
                             % (model.output_size, self.J, self.D))
        # [0:J] per-joint L2 sums (mm), [J] sum of squared normalized errors (the loss
        # numerator of src/linear_model.py:129), both fp64, accumulated by the kernel
        self.sums = torch.zeros(self.J + 1, dtype=torch.float64, device=dev)
        self.joint_sum = self.sums[:self.J]
        self.sq_sum = self.sums[self.J:]
        self.frames = 0
        self.batches = 0

    def reset(self):
        self.sums.zero_()
        self.frames = 0
        self.batches = 0

    def add(self, pred, gt, nbatches=None):
        """Accumulate one device batch of B frames (B = nbatches * batch_size rows)."""
        B = pred.shape[0]
        check(lib().p3d_mpjpe_accum_ex(ptr(pred), ptr(gt), self.D, ptr(self.mean), ptr(self.std), ptr(self.dims),
                                       B, self.J, int(self.procrustes), ptr(self.joint_sum), ptr(self.sq_sum),
                                       self.model.stream()), "p3d_mpjpe_accum_ex")
        self.frames += B
        self.batches += 1 if nbatches is None else nbatches

    def loss_sum(self, batch_size):
        """Device scalar: sum over batches of the per-batch loss mean((y - t)^2)."""
        return self.sq_sum / float(batch_size * self.D)


def _stack(batches, width):
    if len(batches) == 0:
        return np.zeros((0, width), np.float32)
    return np.ascontiguousarray(np.vstack(batches), dtype=np.float32)


def run_eval_rows(model, acc, X, Y, batch_size, chunk_rows=8192):
    """Forward + fused MPJPE over whole batches of device rows X/Y (no host sync).

    Inference rows are independent (BN uses moving statistics), so consecutive
    batches are submitted together in chunks of up to ``chunk_rows``.
    """
    n = X.shape[0]
    chunk = max(batch_size, (min(chunk_rows, model.max_batch) // batch_size) * batch_size)
    out = model.torch.empty((min(chunk, max(n, 1)), model.output_size), dtype=model.torch.float32,
                            device=model.device)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        y = model.forward_device(X[s:e], False, 1.0, out=out[:e - s])
        acc.add(y, Y[s:e], (e - s) // batch_size)


def evaluate_batches(sess, model, data_mean_3d, data_std_3d, dim_to_use_3d, dim_to_ignore_3d,
                     data_mean_2d, data_std_2d, dim_to_use_2d, dim_to_ignore_2d,
                     current_step, encoder_inputs, decoder_outputs, current_epoch=0, flags=None):
    """src/predict_3dpose.py:352-444 -> (total_err, joint_err, step_time, loss)."""
    flags = flags or FLAGS
    torch = model.torch
    nbatches = len(encoder_inputs)
    for b in encoder_inputs:
        if b.shape[0] != model.batch_size:
            raise AssertionError("batch of %d != batch_size %d" % (b.shape[0], model.batch_size))
    start = time.time()
    acc = MPJPE(model, data_mean_3d, data_std_3d, dim_to_use_3d, flags.predict_14, flags.procrustes)
    with torch.cuda.device(model.device):
        X = torch.from_numpy(_stack(encoder_inputs, model.input_size)).to(model.device)
        Y = torch.from_numpy(_stack(decoder_outputs, model.output_size)).to(model.device)
        run_eval_rows(model, acc, X, Y, model.batch_size)
        js = acc.joint_sum.cpu().numpy()
        loss = float(acc.loss_sum(model.batch_size).item())
        model.check_errors()
    step_time = (time.time() - start) / max(nbatches, 1)
    n = max(acc.frames, 1)
    joint_err = js / n
    total_err = float(np.sum(js) / (n * acc.J))
    return total_err, joint_err, step_time, loss / max(nbatches, 1)


def evaluate_action_wise(model, test_set_2d, test_set_3d, data_mean_3d, data_std_3d, dim_to_use_3d,
                         actions, camera_frame=True, flags=None):
    """Per-action MPJPE sweep (src/predict_3dpose.py:274-298), frame-sharded.

    Each action's batch list (after the reference's per-action n % B tail drop) is
    split contiguously across the ranks of the current torch.distributed job; every
    rank accumulates fp64 per-joint sums, frame counts and loss sums on its GPU and
    one all-reduce over a [n_actions, J+2] fp64 tensor combines them.  Returns
    ({action: mm}, average_mm) with the reference's unweighted Average.
    """
    import torch
    flags = flags or FLAGS
    _, rank, world = dist_utils.dist_state()
    J = 14 if flags.predict_14 else 17
    table = torch.zeros((len(actions), J + 2), dtype=torch.float64, device=model.device)
    with torch.cuda.device(model.device):
        for ai, action in enumerate(actions):
            enc, dec = model.get_all_batches(get_action_subset(test_set_2d, action),
                                             get_action_subset(test_set_3d, action), camera_frame,
                                             training=False)
            lo, hi = dist_utils.shard_range(len(enc), rank, world)
            acc = MPJPE(model, data_mean_3d, data_std_3d, dim_to_use_3d, flags.predict_14, flags.procrustes)
            if hi > lo:
                X = torch.from_numpy(_stack(enc[lo:hi], model.input_size)).to(model.device)
                Y = torch.from_numpy(_stack(dec[lo:hi], model.output_size)).to(model.device)
                run_eval_rows(model, acc, X, Y, model.batch_size)
            table[ai, :J] = acc.joint_sum
            table[ai, J] = float(acc.frames)
            table[ai, J + 1] = acc.loss_sum(model.batch_size)[0]
        dist_utils.allreduce_sum_(table)
        t = table.cpu().numpy()
        model.check_errors()
    errs = {}
    for ai, action in enumerate(actions):
        n = max(t[ai, J], 1.0)
        errs[action] = float(np.sum(t[ai, :J]) / (n * J))
    return errs, float(np.mean([errs[a] for a in actions]))


def synthetic_h36m(n_train=20000, n_test=4000, seed=0, out_dim=48):
    """Normalized H3.6M-shaped data (keys (subject, action, seqname)) and stats."""
    rng = np.random.default_rng(seed)
    actions = data_utils.define_actions("All")
    use3, ign3 = data_utils.dimension_sets(3, out_dim == 42)
    use2, ign2 = data_utils.dimension_sets(2)
    mean3 = np.zeros(96)
    std3 = np.zeros(96)
    mean3[use3] = rng.uniform(-500, 500, len(use3))
    std3[use3] = rng.uniform(50, 300, len(use3))
    mean2 = np.zeros(64)
    std2 = np.ones(64)
    mean2[use2] = rng.uniform(200, 800, len(use2))
    std2[use2] = rng.uniform(20, 120, len(use2))
    proj = rng.standard_normal((32, out_dim)) / np.sqrt(32)

    def make(subjects, n):
        s2, s3 = {}, {}
        for a in actions:
            for j, subj in enumerate(subjects):
                k = max(1, n // (len(actions) * len(subjects)))
                x = rng.standard_normal((k + j * 7, 32))
                y = np.tanh(x @ proj) + 0.1 * rng.standard_normal((len(x), out_dim))
                # H3.6M key shapes: 2D (and camera-frame 3D) "<seq>.<camera>.h5", world-frame
                # 3D "<seq>.h5" -- get_all_batches derives the 3D key from the 2D one
                # (src/linear_model.py:272-273); one camera per sequence, so both resolve
                seq = "%s %d" % (a, j)
                s2[(subj, a, "%s.54138969.h5" % seq)] = x
                s3[(subj, a, "%s.54138969.h5" % seq)] = y
                s3[(subj, a, "%s.h5" % seq)] = y
        return s2, s3

    tr2, tr3 = make(data_utils.TRAIN_SUBJECTS, n_train)
    te2, te3 = make(data_utils.TEST_SUBJECTS, n_test)
    return dict(train_set_2d=tr2, train_set_3d=tr3, test_set_2d=te2, test_set_3d=te3, data_mean_3d=mean3,
                data_std_3d=std3, dim_to_use_3d=use3, dim_to_ignore_3d=ign3, data_mean_2d=mean2,
                data_std_2d=std2, dim_to_use_2d=use2, dim_to_ignore_2d=ign2)


def dp_epoch_share(enc, dec, rank, world):
    """This rank's batches of a data-parallel epoch: equal contiguous shares of the
    (identically permuted) batch list, so every replica runs the same number of steps."""
    per = len(enc) // world
    return enc[rank * per:(rank + 1) * per], dec[rank * per:(rank + 1) * per]


SUBJECT_IDS = [1, 5, 6, 7, 8, 9, 11]


def load_data(flags):
    """The training / test sets and their statistics (src/predict_3dpose.py:194-208): cameras,
    3D poses (camera frame, root-centred, normalised) and the 2D inputs -- ground-truth
    projections or Stacked Hourglass detections.  ``--data_dir`` / ``--cameras_path`` name the
    H3.6M tree and cameras.h5 or their .npz archives (data_utils, cameras); ``--synthetic``
    skips the files."""
    if flags.synthetic:
        return synthetic_h36m(out_dim=42 if flags.predict_14 else 48, seed=flags.seed)
    actions = data_utils.define_actions(flags.action)
    rcams = cameras.load_cameras(flags.cameras_path, SUBJECT_IDS)
    (train_set_3d, test_set_3d, data_mean_3d, data_std_3d, dim_to_ignore_3d, dim_to_use_3d, _,
     _) = data_utils.read_3d_data(actions, flags.data_dir, flags.camera_frame, rcams, flags.predict_14)
    if flags.use_sh:
        two = data_utils.read_2d_predictions(actions, flags.data_dir)
    else:
        two = data_utils.create_2d_data(actions, flags.data_dir, rcams)
    train_set_2d, test_set_2d, data_mean_2d, data_std_2d, dim_to_ignore_2d, dim_to_use_2d = two
    return dict(train_set_2d=train_set_2d, train_set_3d=train_set_3d, test_set_2d=test_set_2d,
                test_set_3d=test_set_3d, data_mean_3d=data_mean_3d, data_std_3d=data_std_3d,
                dim_to_use_3d=dim_to_use_3d, dim_to_ignore_3d=dim_to_ignore_3d, data_mean_2d=data_mean_2d,
                data_std_2d=data_std_2d, dim_to_use_2d=dim_to_use_2d, dim_to_ignore_2d=dim_to_ignore_2d)


def train(flags=None):
    """Epoch loop of src/predict_3dpose.py:188-334 on the MI355X model."""
    flags = flags or FLAGS
    actions = data_utils.define_actions(flags.action)
    d = load_data(flags)
    tdir = train_dir_for(flags)
    os.makedirs(os.path.join(tdir, "log"), exist_ok=True)
    with Session() as sess:
        print("Creating %d bi-layers of %d units." % (flags.num_layers, flags.linear_size))
        model = create_model(sess, actions, flags.batch_size, flags)
        print("Model created")
        current_step = 0 if flags.load <= 0 else flags.load + 1
        log_every_n_batches = 100
        for epoch in range(1, flags.epochs + 1):
            if model.data_parallel:
                # one epoch covers the training set once over all replicas: every rank draws the
                # same permutation and trains on its own equal share of the batches (the global
                # batch is world x batch_size; a remainder of < world batches is dropped, like
                # the reference's n % batch_size tail)
                np.random.seed((flags.seed * 1000003 + epoch) % (2 ** 32))
            enc, dec = model.get_all_batches(d["train_set_2d"], d["train_set_3d"], flags.camera_frame,
                                             training=True)
            if model.data_parallel:
                enc, dec = dp_epoch_share(enc, dec, model.rank, model.world)
            nbatches = len(enc)
            print("There are {0} train batches".format(nbatches))
            start_time, loss = time.time(), 0.
            if flags.device_loop:
                # the epoch's batches staged in HBM once; per-step losses land in a device
                # vector (no host round trip per step; one sync per logging interval)
                import torch
                B = flags.batch_size
                with torch.cuda.device(model.device):
                    X = torch.from_numpy(_stack(enc, model.input_size)).to(model.device)
                    T = torch.from_numpy(_stack(dec, model.output_size)).to(model.device)
                    losses = torch.zeros(max(nbatches, 1), dtype=torch.float32, device=model.device)
                    for i in range(nbatches):
                        lr = linear_model.exponential_decay(model.lr0, model._step_host)
                        model.train_step_device(X[i * B:(i + 1) * B], T[i * B:(i + 1) * B], flags.dropout,
                                                loss_out=losses[i:i + 1])
                        if (i + 1) % log_every_n_batches == 0:
                            step_loss = float(losses[i].item())
                            model.check_errors()     # (after the sync the loss read made)
                            model.train_writer.add_summary(linear_model.Summary("loss/loss", step_loss), current_step)
                            model.train_writer.add_summary(
                                linear_model.Summary("learning_rate/learning_rate", lr), current_step)
                            step_time = time.time() - start_time
                            start_time = time.time()
                            print("Working on epoch {0}, batch {1} / {2}... done in {3:.2f} ms".format(
                                epoch, i + 1, nbatches, 1000 * step_time / log_every_n_batches))
                        current_step += 1
                    loss = float(losses[:nbatches].double().sum().item())
                    model.check_errors()
            else:
                for i in range(nbatches):
                    step_loss, loss_summary, lr_summary, _ = model.step(sess, enc[i], dec[i], flags.dropout,
                                                                        isTraining=True)
                    if (i + 1) % log_every_n_batches == 0:
                        model.train_writer.add_summary(loss_summary, current_step)
                        model.train_writer.add_summary(lr_summary, current_step)
                        step_time = time.time() - start_time
                        start_time = time.time()
                        print("Working on epoch {0}, batch {1} / {2}... done in {3:.2f} ms".format(
                            epoch, i + 1, nbatches, 1000 * step_time / log_every_n_batches))
                    loss += step_loss
                    current_step += 1
            loss = loss / max(nbatches, 1)
            print("=============================\n"
                  "Global step:         %d\n"
                  "Learning rate:       %.2e\n"
                  "Train loss avg:      %.4f\n"
                  "=============================" % (model.global_step.eval(), model.learning_rate.eval(), loss))
            model.sync_moving_stats()   # data parallel: evaluate with the replicas' mean statistics
            if flags.evaluateActionWise:
                print("{0:=^12} {1:=^6}".format("Action", "mm"))
                errs, avg = evaluate_action_wise(model, d["test_set_2d"], d["test_set_3d"], d["data_mean_3d"],
                                                 d["data_std_3d"], d["dim_to_use_3d"], actions,
                                                 flags.camera_frame, flags)
                for a in actions:
                    print("{0:<12} {1:>6.2f}".format(a, errs[a]))
                model.test_writer.add_summary(sess.run(model.err_mm_summary, {model.err_mm: avg}), current_step)
                print("{0:<12} {1:>6.2f}".format("Average", avg))
                print("{0:=^19}".format(''))
            else:
                enc, dec = model.get_all_batches(d["test_set_2d"], d["test_set_3d"], flags.camera_frame,
                                                 training=False)
                total_err, joint_err, step_time, vloss = evaluate_batches(
                    sess, model, d["data_mean_3d"], d["data_std_3d"], d["dim_to_use_3d"], d["dim_to_ignore_3d"],
                    d["data_mean_2d"], d["data_std_2d"], d["dim_to_use_2d"], d["dim_to_ignore_2d"],
                    current_step, enc, dec, epoch, flags)
                print("=============================\n"
                      "Step-time (ms):      %.4f\n"
                      "Val loss avg:        %.4f\n"
                      "Val error avg (mm):  %.2f\n"
                      "=============================" % (1000 * step_time, vloss, total_err))
                for i in range(17 if not flags.predict_14 else 14):
                    print("Error in joint {0:02d} (mm): {1:>5.2f}".format(i + 1, joint_err[i]))
                model.test_writer.add_summary(sess.run(model.err_mm_summary, {model.err_mm: total_err}),
                                              current_step)
            print("Saving the model... ", end="")
            t0 = time.time()
            model.saver.save(sess, os.path.join(tdir, 'checkpoint'), global_step=current_step)
            print("done in {0:.2f} ms".format(1000 * (time.time() - t0)))
            sys.stdout.flush()
    return model


def main(argv=None):
    global FLAGS
    FLAGS = build_parser().parse_args(argv)
    if FLAGS.sample:
        raise NotImplementedError("sample() is matplotlib visualisation (out of scope for this build)")
    try:
        return train(FLAGS)
    finally:
        dist_utils.close_native_comms()   # data parallel over RCCL: detach the model, free the comm


if __name__ == "__main__":
    main()
