"""Same-box A/B of two builds of libpa_hip.so (layout changes a run-time
knob cannot switch): runs a measurement script once per library per round,
in alternating order, each in its own process (PA_HIP_LIB selects the
other build), and prints the per-library results of every round as JSON.

    python tools/ab_lib.py --base abl/libpa_hip_base.so --rounds 4 -- tools/c5_bench.py --dtypes f32,f64 --steps 30
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(lib, cmd):
    env = dict(os.environ)
    if lib:
        env["PA_HIP_LIB"] = os.path.abspath(lib)
    else:
        env.pop("PA_HIP_LIB", None)
    p = subprocess.run([sys.executable, "-u"] + cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    if p.returncode != 0:
        raise SystemExit(f"{cmd} with {lib or 'HEAD'} failed ({p.returncode}):\n{p.stderr[-2000:]}")
    return [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", required=True, help="the other build (A); B is the in-tree library")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    out = {"base": [], "head": []}
    for r in range(a.rounds):
        order = [("base", a.base), ("head", None)] if r % 2 == 0 else [("head", None), ("base", a.base)]
        for name, lib in order:
            out[name].append(run(lib, cmd))
            print(json.dumps({"round": r, "lib": name, "result": out[name][-1]}), flush=True)
    print(json.dumps({"tool": "ab_lib", "base": a.base, "cmd": cmd, "rounds": a.rounds, "results": out}))


if __name__ == "__main__":
    main()
