"""Checkpoint interop with the reference's TF1 variables.

* Variable names and order: ``tf.global_variables()`` of ``src/linear_model.py`` --
  ``learning_rate`` and ``global_step`` (:84-85), then each layer's variables in creation
  order (``w1``, ``b1``, the BN ``gamma``/``beta``/``moving_mean``/``moving_variance``, ...,
  ``w4``, ``b4``; :103-193), then ``AdamOptimizer``'s ``beta1_power``/``beta2_power`` and the
  ``<var>/Adam``, ``<var>/Adam_1`` slots of every trainable (TF1 ``_create_slots``).
  ``tf.trainable_variables()`` is the trainable subset in the same order.
* The npy-dump format of the reference's weight export (``src/predict_3dpose.py:548-568``):
  one file per variable, ``"%04d - %s.npy" % (idx, var.name.replace('/', '-'))`` with TF's
  ``":0"`` output suffix, e.g. ``0000 - linear_model-w1:0.npy`` (trainable dump) or the
  global-variable dump of the same shape.

Files are read with ``np.load(allow_pickle=False)`` only.
"""
from __future__ import annotations

import os
import re

import numpy as np

_DUMP_RE = re.compile(r"^(\d{4}) - (.+):0\.npy$")


def trainable_order(param_table):
    """tf.trainable_variables() names (param_table rows: (name, numel, kind, offset))."""
    return [n for n, _, kind, _ in param_table if kind == 0]


def global_order(param_table):
    """tf.global_variables() names of the reference graph, in creation order.

    ``tf.layers.batch_normalization`` creates gamma, beta, moving_mean, moving_variance in
    that order inside its scope (src/linear_model.py:112,181,193), so each BN scope's moving
    statistics follow its beta -- whatever order the param table (p3d_create lists every
    moving statistic after all trainables) uses."""
    moving = {}
    for n, _, kind, _ in param_table:
        if kind != 0:
            moving.setdefault(n.rsplit("/", 1)[0], []).append(n)
    names = ["learning_rate", "global_step"]
    for n in trainable_order(param_table):
        names.append(n)
        if n.endswith("/beta"):
            names += moving.pop(n.rsplit("/", 1)[0], [])
    for rest in moving.values():       # moving statistics of a scope without beta (none in TF1)
        names += rest
    names += ["beta1_power", "beta2_power"]
    for n in trainable_order(param_table):
        names += [n + "/Adam", n + "/Adam_1"]
    return names


def dump_filename(idx: int, name: str) -> str:
    return "%04d - %s.npy" % (idx, (name + ":0").replace("/", "-"))


def parse_dump_filename(fname: str):
    """(index, TF variable name) of a dump file name, or None."""
    m = _DUMP_RE.match(os.path.basename(fname))
    if not m:
        return None
    return int(m.group(1)), m.group(2).replace("-", "/")


def export_npy_dump(model, directory: str, all_variables: bool = False):
    """Write the model's variables in the reference's npy-dump format; returns the paths."""
    os.makedirs(directory, exist_ok=True)
    state = model.get_state()
    names = global_order(model.param_table) if all_variables else trainable_order(model.param_table)
    paths = []
    for idx, name in enumerate(names):
        val = np.asarray(state[name])
        if name == "global_step":
            val = val.astype(np.int64)
        elif val.dtype != np.int64:
            val = val.astype(np.float32)
        path = os.path.join(directory, dump_filename(idx, name))
        with open(path, "wb") as f:
            np.save(f, val)
        paths.append(path)
    return paths


def read_npy_dump(directory: str):
    """{TF name: array} from a directory of dump files (trainable or global dump)."""
    out = {}
    for fname in sorted(os.listdir(directory)):
        parsed = parse_dump_filename(fname)
        if parsed is None:
            continue
        out[parsed[1]] = np.load(os.path.join(directory, fname), allow_pickle=False)
    if not out:
        raise ValueError("no '%%04d - <name>:0.npy' variable dumps in %s" % directory)
    return out


def check_state(model, state):
    """TF1 ``Saver.restore`` semantics (the Saver of src/linear_model.py:151 lists every global
    variable): every variable of the model must be in the checkpoint (TF raises NotFoundError
    otherwise), variables the model does not have are ignored, a shape mismatch is an error
    (InvalidArgumentError).  Returns the checkpoint restricted to the model's variables."""
    names = global_order(model.param_table)
    missing = [n for n in names if n not in state]
    if missing:
        raise ValueError("checkpoint lacks variables of this model: %s" % ", ".join(missing[:8]))
    shapes = model._shapes
    out = {}
    for name in names:
        val = state[name]
        want = shapes.get(name[:-len("/Adam_1")] if name.endswith("/Adam_1") else
                          name[:-len("/Adam")] if name.endswith("/Adam") else name)
        if want is not None and tuple(np.shape(val)) != tuple(want):
            raise ValueError("%s: checkpoint shape %s, model shape %s" % (name, np.shape(val), tuple(want)))
        out[name] = val
    return out


def import_npy_dump(model, directory: str):
    """Load a trainable or global npy dump into the model (unknown names are rejected)."""
    state = read_npy_dump(directory)
    known = set(global_order(model.param_table))
    unknown = sorted(set(state) - known)
    if unknown:
        raise ValueError("dump variables not in this model: %s" % ", ".join(unknown[:8]))
    shapes = model._shapes
    for name, val in state.items():
        if name in shapes and tuple(val.shape) != tuple(shapes[name]):
            raise ValueError("%s: dump shape %s, model shape %s" % (name, val.shape, tuple(shapes[name])))
    model.set_state(state)
    return sorted(state)
