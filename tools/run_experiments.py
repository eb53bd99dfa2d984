#!/usr/bin/env python3
"""Experiment harness for GpuSolve-cpu / GpuSolve-hip: the equivalent of the
reference's runExperiments.py:13-74 for this build.

Per (implementation, mode, resolution) it writes the reference's experiment config (10 V-cycles,
tol 10e-5, r^3 points, 3+3 smoothing, omega 0.8, gamma 1.0, the 7-point stencil;
runExperiments.py:15-26), runs the executable, and sums the "Took Nms" of every V-cycle / Newton
line (runExperiments.py:46-57). Differences, on purpose:
  * the residual field accepts exponents with '+' and nan/inf: the reference's regex
    `[\\d\\.e-]+` (runExperiments.py:46) skips lines like "residual: 2.1e+05", which a diverging
    power-of-two run prints; here such runs still count every cycle;
  * results also go to a JSON file (--json), with the final residual of each run;
  * implementations are given on the command line (name=path[:ENV=VAL,...]); by default the
    reference CPU build (oracle/_ref/GpuSolve-cpu, all cores and OMP_NUM_THREADS=1) when it exists
    and bin/GpuSolve-hip.

    python tools/run_experiments.py [--resolutions 63,127,255,511] [--modes 0,1,2] [--json out.json]
"""
import argparse
import itertools
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODE_NAMES = {0: "LINEAR", 1: "NON LINEAR", 2: "NEWTON"}
SHORT = {0: "lin", 1: "non", 2: "newton"}
# "iter: i residual: R Took Tms" and "newton iter: ..." (Timer.cpp:17-26 / CpuSolver.cpp:28)
ITER = re.compile(r"iter: (\d+) residual: (\S+) Took (\d+)ms")


def config_text(mode, resolution, maxiter=10, tol="10e-5", pre=3, post=3, omega=0.8, gamma=1.0):
    return (f"{maxiter}\n{tol}\n" + f"{resolution}\n" * 3 + f"{mode}\n{pre}\n{post}\n{omega}\n{gamma}\n"
            "6 -1 -1 -1 -1 -1 -1\n0 1 -1 0 0 0 0\n0 0 0 1 -1 0 0\n0 0 0 0 0 1 -1\n")


def parse_output(stdout):
    """(total ms, [(iter, residual)]) over every V-cycle / Newton iteration line."""
    rows = [(int(i), float(r), int(t)) for i, r, t in ITER.findall(stdout)]
    return sum(t for _, _, t in rows), [(i, r) for i, r, _ in rows]


def run_experiment(exe, mode, resolution, env_changes=None, timeout=3600):
    with tempfile.NamedTemporaryFile("w", suffix=".conf", delete=False) as f:
        f.write(config_text(mode, resolution))
        path = f.name
    env = dict(os.environ)
    env.update(env_changes or {})
    try:
        res = subprocess.run([exe, path], capture_output=True, text=True, env=env, timeout=timeout)
    finally:
        os.unlink(path)
    if res.returncode != 0:
        return {"ok": False, "stderr": res.stderr[-2000:], "stdout": res.stdout[-2000:]}
    total, iters = parse_output(res.stdout)
    if not iters:
        return {"ok": False, "stdout": res.stdout[-2000:]}
    return {"ok": True, "total_ms": total, "cycles": len(iters), "final_residual": iters[-1][1]}


def parse_impl(spec):
    name, _, rest = spec.partition("=")
    path, _, envs = rest.partition(":")
    env = dict(kv.split("=", 1) for kv in envs.split(",") if kv) if envs else {}
    return name, path, env


def default_impls():
    impls = []
    ref = os.path.join(REPO, "oracle", "_ref", "GpuSolve-cpu")
    if os.path.exists(ref):
        impls += [("GpuSolve-cpu", ref, {}), ("GpuSolve-cpu", ref, {"OMP_NUM_THREADS": "1"})]
    impls.append(("GpuSolve-hip", os.path.join(REPO, "gpu-solve_amd", "bin", "GpuSolve-hip"), {}))
    return impls


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", action="append", default=[], help="name=path[:ENV=VAL,...] (repeatable)")
    ap.add_argument("--resolutions", default="63,127,255,511")
    ap.add_argument("--modes", default="0,1,2")
    ap.add_argument("--no-warmup", action="store_true")
    ap.add_argument("--json", default="")
    a = ap.parse_args(argv)
    impls = [parse_impl(s) for s in a.impl] or default_impls()
    modes = [int(m) for m in a.modes.split(",")]
    resolutions = [int(r) for r in a.resolutions.split(",")]
    if not a.no_warmup:  # runExperiments.py:91-101
        for name, exe, env in impls:
            print(f"Warmup {name}", flush=True)
            run_experiment(exe, modes[0], resolutions[0], env)
    results = {}
    for (name, exe, env), mode, res in itertools.product(impls, modes, resolutions):
        r = run_experiment(exe, mode, res, env)
        key = f"{name}_{mode}_{res}_{env}"
        results[key] = dict(r, impl=name, env=env, mode=mode, resolution=res)
        if r["ok"]:
            print(f"{name} in mode {MODE_NAMES[mode]}{' with env ' + str(env) if env else ''} and {res} points: "
                  f"{r['total_ms']}ms ({r['cycles']} cycles, final residual {r['final_residual']:g})", flush=True)
        else:
            print(f"{name} in mode {MODE_NAMES[mode]} and {res} points: FAILED", flush=True)
    print("")
    for res in resolutions:  # the pgfplots lines of runExperiments.py:135-160
        print(f"Results for resolution {res}:")
        for name, exe, env in impls:
            coords = " ".join(f"({SHORT[m]},{results[f'{name}_{m}_{res}_{env}'].get('total_ms', 'nan')})"
                              for m in modes)
            print("\\addplot coordinates {" + coords + " }; %" + name + " " + str(env))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(results, f, indent=1)
    return 0 if all(r["ok"] for r in results.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
