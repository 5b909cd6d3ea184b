"""Dev tool: A/B of two environment settings on one box (e.g. a kernel-form knob read at
p3d_create).  Runs `script` under env A and env B alternately, `rounds` times each.
Usage: python tools/env_ab.py 'K=V[,K=V]' 'K=V[,K=V]' <rounds> <script.py> [args...]
('-' for no variables)."""
import json
import os
import subprocess
import sys


def parse(s):
    return {} if s == "-" else dict(kv.split("=", 1) for kv in s.split(","))


def main():
    a, b, rounds, script = parse(sys.argv[1]), parse(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    rest = sys.argv[5:]
    out = {"A": a, "B": b, "runs": []}
    for r in range(rounds):
        for tag, ev in (("A", a), ("B", b)):
            env = dict(os.environ, **ev)
            p = subprocess.run([sys.executable, script] + rest, env=env, stdout=subprocess.PIPE,
                               stderr=subprocess.PIPE, text=True, timeout=300)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            res = json.loads(line[-1]) if (p.returncode == 0 and line) else {"rc": p.returncode, "err": p.stderr[-500:]}
            out["runs"].append({"round": r, "env": tag, **res})
            print(json.dumps(out["runs"][-1]), flush=True)
            if "rc" in res:   # a failed run (a GPU fault among the causes): run nothing more on the GPU
                print(json.dumps(out))
                sys.exit(2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
