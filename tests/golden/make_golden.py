#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs oracle/_ref/ref_probe and oracle/_ref/GpuSolve-cpu — both compiled by oracle/Makefile from
/root/reference/src/{main.cpp,Timer.cpp,cpu/*.cpp} where they lie (nothing copied) — and stores
only data: residual histories (17 significant digits), reference stdout transcripts, level tables,
right-hand sides and per-operator input/output fields on seeded random grids.

Outputs (all data, no reference source):
  histories.json        17-digit residual histories, keyed by case name (+ the case's config)
  large_histories.json  the BASELINE-size anchors (511^3/512^3), a few cycles each   (--large)
  stdout.json           6-digit reference stdout transcripts (timings stripped)
  paths.json            reference stdout/stderr/exit code for quoted/escaped and missing config paths
  levels.json           level dims + h for several grid shapes
  rhs.npz               level-0 f for linear / non-linear RHS on small grids
  ops.npz               per-operator fixtures (inputs + outputs, reference layout (Px,Py,Pz))
  dumps.json / .npz     Vector3::dump text of the level-0 solution after small solves, and the same
                        field as doubles (src/cpu/Vector3.cpp:56-78; the plotter.py input format)

Usage:  python tests/golden/make_golden.py [--large]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PROBE = os.path.join(REPO, "oracle", "_ref", "ref_probe")
REFEXE = os.path.join(REPO, "oracle", "_ref", "GpuSolve-cpu")
STENCIL = "6 -1 -1 -1 -1 -1 -1\n0 1 -1 0 0 0 0\n0 0 0 1 -1 0 0\n0 0 0 0 0 1 -1\n"


def config_text(c):
    return (f"{c['maxiter']}\n{c['tol']}\n{c['X']}\n{c['Y']}\n{c['Z']}\n{c['mode']}\n{c['pre']}\n"
            f"{c['post']}\n{c['omega']}\n{c['gamma']}\n" + c.get("stencil", STENCIL))


def case(X, Y=None, Z=None, mode=0, pre=2, post=2, maxiter=10, tol=0, omega=0.8, gamma=1.0, stencil=None):
    c = dict(X=X, Y=Y if Y is not None else X, Z=Z if Z is not None else X, mode=mode, pre=pre, post=post,
             maxiter=maxiter, tol=tol, omega=omega, gamma=gamma)
    if stencil:
        c["stencil"] = stencil
    return c


HIST_LINE = re.compile(r"^(Inital residual|Inital newton residual|iter: \d+ residual|newton iter: \d+ residual): (\S+)")


def run_history(c, exe=PROBE, args=("solve",)):
    with tempfile.NamedTemporaryFile("w", suffix=".conf", delete=False) as f:
        f.write(config_text(c))
        path = f.name
    try:
        out = subprocess.run([exe, *args, path], check=True, capture_output=True, text=True).stdout
    finally:
        os.unlink(path)
    return out


def parse_history(out):
    return [float(m.group(2)) for m in map(HIST_LINE.match, out.splitlines()) if m]


def small_cases():
    cases = {}
    for n in (7, 15, 16, 31, 32, 63, 127, 128):
        for mode in (0, 1, 2):
            cases[f"m{mode}_n{n}_2+2"] = case(n, mode=mode, maxiter=3 if mode == 2 else 10)
    for n in (31, 32):
        for mode in (0, 1, 2):
            for pre, post in ((1, 0), (3, 3), (0, 2)):
                cases[f"m{mode}_n{n}_{pre}+{post}"] = case(n, mode=mode, pre=pre, post=post,
                                                            maxiter=3 if mode == 2 else 6)
    for dims in ((17, 9, 12), (31, 32, 33), (20, 33, 15), (64, 48, 40), (9, 40, 23)):
        for mode in (0, 1, 2):
            cases[f"m{mode}_{dims[0]}x{dims[1]}x{dims[2]}_2+2"] = case(*dims, mode=mode,
                                                                        maxiter=3 if mode == 2 else 8)
    # relaxation / gamma variations and early exits through `tol`
    cases["m0_n63_w0.6"] = case(63, omega=0.6, maxiter=6)
    cases["m1_n63_g0.5"] = case(63, mode=1, gamma=0.5, maxiter=6)
    cases["m2_n63_g2.0"] = case(63, mode=2, gamma=2.0, maxiter=3)
    cases["m0_n63_tol1e-3"] = case(63, tol=1e-3, maxiter=20)
    cases["m1_n63_tol1e-4"] = case(63, mode=1, tol=1e-4, maxiter=20)
    cases["m2_n63_tol1e-6"] = case(63, mode=2, tol=1e-6, maxiter=10)
    # a permuted-order stencil (same operator, different summation order) and an anisotropic one
    cases["m0_n31_permuted"] = case(31, maxiter=5, stencil="-1 -1 6 -1 -1 -1 -1\n0 -1 0 0 1 0 0\n1 0 0 0 0 0 -1\n0 0 0 -1 0 1 0\n")
    cases["m0_n31_aniso"] = case(31, maxiter=5, stencil="4 -1 -1 -0.5 -0.5 -0.5 -0.5\n0 1 -1 0 0 0 0\n0 0 0 1 -1 0 0\n0 0 0 0 0 1 -1\n")
    # the reference's own example (Newton 127^3, 3+3, tol 1e-5)
    cases["example_data-2nd_order"] = case(127, mode=2, pre=3, post=3, maxiter=10, tol=1e-5)
    return cases


def large_cases():
    return {
        "m0_n511_2+2": case(511, maxiter=3),
        "m0_n512_2+2": case(512, maxiter=3),
        "m1_n511_2+2": case(511, mode=1, maxiter=2),
        "m1_n512_2+2": case(512, mode=1, maxiter=2),
        "m2_n511_2+2": case(511, mode=2, maxiter=2),
        "m2_n512_2+2": case(512, mode=2, maxiter=2),
    }


def config3_cases():
    """BASELINE config #3 as stated (10 V-cycles) and its converging companion, plus config #4's
    companion for more than two Newton iterations."""
    return {
        "m0_n511_2+2_x10": case(511, maxiter=10),
        "m0_n512_2+2_x10": case(512, maxiter=10),
        "m2_n511_2+2_x4": case(511, mode=2, maxiter=4),
    }


def huge_cases():
    """BASELINE config #5's grid (1024^3) and its companion 1023^3, two linear V-cycles each. The
    reference holds 6 arrays per level (src/cpu/CpuGridData.cpp:32-39): ~55 GiB at this size, so the
    probe runs under a virtual-memory cap (it fails with bad_alloc instead of waking the OOM killer)."""
    return {
        "m0_n1023_2+2": case(1023, maxiter=2),
        "m0_n1024_2+2": case(1024, maxiter=2),
    }


def huge10_cases():
    """Config #5's grid as the solver runs it: 1024^3 linear 2+2, TEN V-cycles (round-3 verdict: the
    2-cycle anchors pin little of a converging history)."""
    return {"m0_n1024_2+2_x10": case(1024, maxiter=10), "m0_n1023_2+2_x10": case(1023, maxiter=10)}


def gen_histories(cases, path, vmem_kb=None):
    res = {}
    if os.path.exists(path) and vmem_kb:  # resumable: the huge cases take minutes each
        with open(path) as f:
            res = json.load(f)
    for name, c in cases.items():
        if name in res:
            continue
        if vmem_kb:
            import resource

            def cap():
                resource.setrlimit(resource.RLIMIT_AS, (vmem_kb * 1024, vmem_kb * 1024))
            with tempfile.NamedTemporaryFile("w", suffix=".conf", delete=False) as f:
                f.write(config_text(c))
                conf = f.name
            try:
                out = subprocess.run([PROBE, "solve", conf], check=True, capture_output=True, text=True,
                                     preexec_fn=cap).stdout
            finally:
                os.unlink(conf)
            res[name] = {"config": c, "history": parse_history(out)}
            print(f"  {name}: {res[name]['history']}", flush=True)
            with open(path, "w") as f:
                json.dump(res, f, indent=1)
            continue
        out = run_history(c)
        res[name] = {"config": c, "history": parse_history(out)}
        print(f"  {name}: {len(res[name]['history'])} values", flush=True)
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


def gen_stdout(path):
    res = {}
    for name, c in {"example_data-2nd_order": case(127, mode=2, pre=3, post=3, maxiter=10, tol=1e-5),
                    "m0_n31_2+2": case(31, maxiter=5), "m1_n15_2+2": case(15, mode=1, maxiter=4),
                    "m0_n16_diverging": case(16, maxiter=10)}.items():
        out = run_history(c, exe=REFEXE, args=())
        lines = [re.sub(r"Took \d+ms", "Took <T>ms", l) for l in out.splitlines()]
        # the config path is a temp file name: keep the line shape only
        lines = [re.sub(r'^Using config file ".*"$', 'Using config file "<PATH>"', l) for l in lines]
        res[name] = {"config": c, "stdout": lines}
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


PATH_CASES = {
    # relative config paths (the executable runs with cwd = a scratch dir): std::filesystem::path's
    # operator<< goes through std::quoted, so '"' and '\\' come out escaped (src/main.cpp:24,28)
    "plain": "plain.conf",
    "space_backslash_quote": 'my conf\\dir "x".conf',
    "trailing_backslash": "end\\",
    "quotes_only": '""',
    "missing": 'no such\\"file.conf',
    "missing_dir": "nodir/",
}


def gen_paths(path):
    """Reference stdout/stderr/exit code for config paths with a space, backslash and double quote,
    and for missing paths (round-3 verdict item 1)."""
    res = {}
    c = case(7, maxiter=2)
    with tempfile.TemporaryDirectory() as td:
        for name, rel in PATH_CASES.items():
            if not name.startswith("missing"):
                with open(os.path.join(td, rel), "w") as f:
                    f.write(config_text(c))
            p = subprocess.run([REFEXE, rel], cwd=td, capture_output=True, text=True)
            res[name] = {"path": rel, "config": None if name.startswith("missing") else c,
                         "stdout": [re.sub(r"Took \d+ms", "Took <T>ms", l) for l in p.stdout.splitlines()],
                         "stderr": p.stderr.splitlines(), "returncode": p.returncode}
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


def gen_levels(path):
    res = {}
    for dims in ((7, 7, 7), (16, 16, 16), (127, 127, 127), (128, 128, 128), (512, 512, 512), (1024, 1024, 1024),
                 (17, 9, 12), (31, 32, 33), (1023, 1023, 1023)):
        out = subprocess.run([PROBE, "levels", *map(str, dims)], check=True, capture_output=True, text=True).stdout
        rows = [l.split() for l in out.splitlines()]
        res["x".join(map(str, dims))] = [[int(r[1]), int(r[2]), int(r[3]), float(r[4]), int(r[5])] for r in rows]
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


def load_field(path, dims):
    return np.fromfile(path, dtype="<f8").reshape(dims[0] + 2, dims[1] + 2, dims[2] + 2)


def gen_rhs(path):
    arrs = {}
    with tempfile.TemporaryDirectory() as td:
        for dims in ((9, 7, 8), (16, 16, 16), (5, 11, 6)):
            for mode, gamma in ((0, 1.0), (1, 1.0), (2, 1.0), (1, 0.5)):
                p = os.path.join(td, "f.bin")
                subprocess.run([PROBE, "rhs", *map(str, dims), str(mode), str(gamma), p], check=True)
                arrs[f"f_{'x'.join(map(str, dims))}_m{mode}_g{gamma}"] = load_field(p, dims)
    np.savez_compressed(path, **arrs)


def level_dims(dims, lvl):
    d = list(dims)
    for _ in range(lvl):
        d = [x // 2 for x in d]
    return d


def gen_ops(path):
    arrs = {}
    meta = {}
    seed = 20250227
    with tempfile.TemporaryDirectory() as td:
        def run(name, dims, mode, lvl, extra=()):
            nonlocal seed
            seed += 1
            for f in os.listdir(td):
                os.unlink(os.path.join(td, f))
            out = subprocess.run([PROBE, "op", name, *map(str, dims), str(mode), str(lvl), str(seed), td, *extra],
                                 check=True, capture_output=True, text=True).stdout
            key = f"{name}_{'x'.join(map(str, dims))}_m{mode}_l{lvl}" + ("_" + "_".join(extra) if extra else "")
            info = {"name": name, "dims": list(dims), "mode": mode, "level": lvl, "seed": seed, "extra": list(extra)}
            m = re.search(r"norm (\S+)", out)
            if m:
                info["norm"] = float(m.group(1))
            for fn in sorted(os.listdir(td)):
                base = fn[:-4]
                if name in ("restrict",) and base == "coarse":
                    d = level_dims(dims, lvl + 1)
                elif name == "interpolate" and base == "coarse":
                    d = level_dims(dims, lvl + 1)
                elif name == "vcycle" and base.startswith("newtonV"):
                    d = level_dims(dims, int(base[len("newtonV"):]))
                else:
                    d = level_dims(dims, lvl)
                arrs[f"{key}/{base}"] = load_field(os.path.join(td, fn), d)
            meta[key] = info

        for dims in ((9, 7, 8), (16, 16, 16), (13, 6, 10)):
            for mode in (0, 1, 2):
                run("residual", dims, mode, 0)
                run("jacobi", dims, mode, 0)
                run("jacobi", dims, mode, 0, ("0.8", "1.0", "3"))
            run("residual", dims, 0, 1)
            run("jacobi", dims, 1, 1, ("0.7", "0.5", "2"))
            run("restrict", dims, 0, 0)
            run("interpolate", dims, 0, 0)
            run("applyStencil", dims, 1, 0)
            run("applyStencil", dims, 1, 1)
            run("compF", dims, 2, 0)
        for dims in ((15, 15, 15), (16, 16, 16), (17, 9, 12)):
            for mode in (0, 1, 2):
                run("vcycle", dims, mode, 0)
        run("interpolate", (31, 32, 33), 0, 0)
        run("interpolate", (32, 31, 30), 0, 1)
        run("restrict", (31, 32, 33), 0, 0)
        run("restrict", (32, 31, 30), 0, 1)
    np.savez_compressed(path, **{k.replace("/", "__"): v for k, v in arrs.items()})
    with open(path.replace(".npz", ".json"), "w") as f:
        json.dump(meta, f, indent=1)


def dump_cases():
    return {"m0_n7_3": case(7, maxiter=3), "m1_9x5x7_3": case(9, 5, 7, mode=1, maxiter=3),
            "m2_n7_2": case(7, mode=2, maxiter=2), "m0_n15_4": case(15, maxiter=4)}


def gen_dumps(path):
    texts, arrs = {}, {}
    with tempfile.TemporaryDirectory() as td:
        for name, c in dump_cases().items():
            conf, txt, binf = (os.path.join(td, n) for n in ("c.conf", "v.txt", "v.bin"))
            with open(conf, "w") as f:
                f.write(config_text(c))
            subprocess.run([PROBE, "solve_dump", conf, txt, binf], check=True, capture_output=True)
            texts[name] = {"config": c, "text": open(txt).read()}
            arrs[name] = load_field(binf, (c["X"], c["Y"], c["Z"]))
    with open(path, "w") as f:
        json.dump(texts, f, indent=1)
    np.savez_compressed(path.replace(".json", ".npz"), **arrs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--large", action="store_true", help="also the 511^3/512^3 anchors (several minutes)")
    ap.add_argument("--only-large", action="store_true")
    ap.add_argument("--only-dumps", action="store_true")
    ap.add_argument("--config3", action="store_true", help="only the 10-cycle 511^3/512^3 anchors")
    ap.add_argument("--only-paths", action="store_true", help="only the config-path quoting transcripts")
    ap.add_argument("--huge", action="store_true", help="only the 1023^3/1024^3 anchors (~55 GiB of host RAM)")
    ap.add_argument("--huge10", action="store_true", help="only the 10-cycle 1024^3 anchor (~55 GiB, long)")
    a = ap.parse_args()
    if a.config3:
        gen_histories(config3_cases(), os.path.join(HERE, "config3_histories.json"), vmem_kb=60 << 20)
        return
    if a.huge:
        gen_histories(huge_cases(), os.path.join(HERE, "huge_histories.json"), vmem_kb=60 << 20)
        return
    if a.huge10:
        gen_histories(huge10_cases(), os.path.join(HERE, "huge10_histories.json"), vmem_kb=60 << 20)
        return
    for exe in (PROBE, REFEXE):
        if not os.path.exists(exe):
            sys.exit(f"{exe} missing: run `make -C oracle ref` (needs /root/reference)")
    if a.only_paths:
        gen_paths(os.path.join(HERE, "paths.json"))
        return
    if a.only_dumps:
        gen_dumps(os.path.join(HERE, "dumps.json"))
        return
    if not a.only_large:
        print("dumps ...", flush=True)
        gen_dumps(os.path.join(HERE, "dumps.json"))
        print("histories ...", flush=True)
        gen_histories(small_cases(), os.path.join(HERE, "histories.json"))
        print("stdout ...", flush=True)
        gen_stdout(os.path.join(HERE, "stdout.json"))
        gen_paths(os.path.join(HERE, "paths.json"))
        print("levels ...", flush=True)
        gen_levels(os.path.join(HERE, "levels.json"))
        print("rhs ...", flush=True)
        gen_rhs(os.path.join(HERE, "rhs.npz"))
        print("ops ...", flush=True)
        gen_ops(os.path.join(HERE, "ops.npz"))
    if a.large or a.only_large:
        print("large histories ...", flush=True)
        gen_histories(large_cases(), os.path.join(HERE, "large_histories.json"))


if __name__ == "__main__":
    main()
