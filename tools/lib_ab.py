"""Dev tool: A/B of two builds of libp3d.so on one box.  Runs `cmd` (a tools/ script printing one
JSON line) under P3D_LIB=A and P3D_LIB=B alternately, `rounds` times each, and prints every
result.  Usage: python tools/lib_ab.py <libA> <libB> <rounds> <script.py> [args...]"""
import json
import os
import subprocess
import sys


def main():
    a, b, rounds, script = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    rest = sys.argv[5:]
    out = {"A": a, "B": b, "runs": []}
    for r in range(rounds):
        for tag, lib in (("A", a), ("B", b)):
            env = dict(os.environ, P3D_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, script] + rest, env=env, stdout=subprocess.PIPE,
                               stderr=subprocess.PIPE, text=True, timeout=300)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            res = json.loads(line[-1]) if (p.returncode == 0 and line) else {"rc": p.returncode, "err": p.stderr[-500:]}
            out["runs"].append({"round": r, "lib": tag, **res})
            print(json.dumps(out["runs"][-1]), flush=True)
            if "rc" in res:   # a failed run (a GPU fault among the causes): run nothing more on the GPU
                print(json.dumps(out))
                sys.exit(2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
