"""Dev tool: the data-parallel step's form on a 1-rank RCCL group (what each rank runs at
N > 1) over bucket sizes and optimizer placements, beside the fused single-GPU step.

    python tools/dp1_sweep.py [steps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 320
    args = bench.build_arg_parser().parse_args([])
    own = bench.init_world1_group()
    v, dt, roof, mode = bench.bench_train(args, 0, 1, steps=steps, warmup=64, dp=False)
    print(json.dumps({"form": "fused single-GPU", "us_per_step": round(1e6 * dt / steps, 2), "mode": mode,
                      "ev": roof.get("event_pair_avg_us")}), flush=True)
    if os.environ.get("FUSED_ONLY"):
        return
    for mb in (8.0, 4.0, 2.0, 0.0):
        for badam in ("1", "0"):
            if mb == 0.0 and badam == "1":
                continue
            os.environ["P3D_DP_BUCKET_ADAM"] = badam
            v, dt, roof, mode = bench.bench_train(args, 0, 1, steps=steps, warmup=64, bucket_mb=mb, dp=True)
            print(json.dumps({"bucket_mb": mb, "bucket_adam": badam, "us_per_step": round(1e6 * dt / steps, 2),
                              "mode": mode, "ev": roof.get("event_pair_avg_us")}), flush=True)
    if own:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
