"""Diagnostic: the 1-rank RCCL data-parallel step, eager then graph-captured, with a Python
traceback on a crash (faulthandler).   python tools/dp_rccl_probe.py [eager|graph]"""
import faulthandler
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)
faulthandler.enable()


def main(what):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29731")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import linear_model
    rng = np.random.default_rng(90)
    xs = torch.from_numpy(rng.standard_normal((3, 64, 32)).astype(np.float32)).cuda()
    ts = torch.from_numpy(rng.standard_normal((3, 64, 48)).astype(np.float32)).cuda()
    m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_dpr", seed=4, data_parallel=True)
    m.initialize(seed=13)
    m.dp_buckets(8)
    print("buckets", m._buckets, flush=True)
    variant = os.environ.get("PROBE_VARIANT", "")
    if variant == "noop_after":      # comm stream behind each bucket's all-reduce, no optimizer there
        import dist_utils
        orig = m._allreduce_grads

        def ar(bucket_adam=False):
            def wait(k, handle):
                linear_model.check(linear_model.lib().p3d_stream_wait_grad(m._h, k, handle), "wait")
            dist_utils.allreduce_mean_buckets_(m.flat["grads"], m._buckets, wait, m._comm,
                                               after=lambda k, h: None)
            if bucket_adam:
                for k in range(len(m._buckets)):
                    linear_model.check(linear_model.lib().p3d_adam_apply_bucket(m._h, k, m.stream()), "adam")
        m._allreduce_grads = ar
    m.train_step_device(xs[0], ts[0], 0.5)
    torch.cuda.synchronize()
    print("eager step 0 ok", flush=True)
    if what == "graph":
        step = m.train_step_graph(xs[1].clone(), ts[1].clone(), 0.5)
        print("captured", flush=True)
        step()
        torch.cuda.synchronize()
        print("replay ok", flush=True)
    else:
        m.train_step_device(xs[1], ts[1], 0.5)
        torch.cuda.synchronize()
        print("eager step 1 ok", flush=True)
    m.check_errors()
    m.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "eager")
