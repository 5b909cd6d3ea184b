"""bench.py's N-rank entry point (host logic, no GPU): `--gpus N` outside a launcher starts
N ranks under torch.distributed.run itself; inside a launcher the rank count must match."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=e, timeout=120)


def test_gpus_n_starts_n_ranks():
    r = run(["--gpus", "4", "--steps", "20", "--warmup", "5", "--launch-dry-run"])
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])["launch"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[-6:] == ["--gpus", "4", "--steps", "20", "--warmup", "5"]


def test_rank_count_mismatch_fails():
    r = run(["--gpus", "8"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 8 but the job has 2 rank(s)" in r.stderr
