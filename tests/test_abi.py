"""CPU-only checks of the drop-in boundary: both C-ABI libraries load, export every symbol their
headers declare, and the host-side logic (layout, config parsing, CLI errors) behaves like the
reference's — no GPU is touched here."""
import ctypes as C
import os
import re
import subprocess

import pytest

import gpusolve as gsv
from conftest import REPO

HEADERS = {
    os.path.join(REPO, "include", "gpusolve_hip.h"): gsv._abi.KERNEL_LIB,
    os.path.join(REPO, "include", "gpusolve_driver.h"): gsv._abi.DRIVER_LIB,
    os.path.join(REPO, "include", "gpusolve_diag.h"): gsv._abi.DIAG_LIB,
}
DECL = re.compile(r"^[A-Za-z_][\w \t\*]*?\b(gs_\w+)\s*\(", re.M)


def declared(header):
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(DECL.findall(text)))


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if l.strip()}


@pytest.mark.parametrize("header", sorted(HEADERS))
def test_every_declared_symbol_is_exported(header):
    lib = HEADERS[header]
    assert os.path.exists(lib), f"{lib} not built"
    names = declared(header)
    assert len(names) >= 10
    missing = [n for n in names if n not in exported(lib)]
    assert not missing, missing


def test_product_library_exports_exactly_its_header():
    """libgpusolve_hip.so exports include/gpusolve_hip.h's entry points and nothing else: the tuning
    variants, bandwidth probes and k_prr live in libgpusolve_diag.so (include/gpusolve_diag.h)."""
    names = set(declared(os.path.join(REPO, "include", "gpusolve_hip.h")))
    got = {n for n in exported(gsv._abi.KERNEL_LIB) if n.startswith("gs_")}
    assert got == names, got ^ names
    diag = set(declared(os.path.join(REPO, "include", "gpusolve_diag.h")))
    assert not (diag & names)
    assert {n for n in exported(gsv._abi.DIAG_LIB) if n.startswith("gs_")} == diag


def test_product_sources_read_no_environment_on_launch():
    """No getenv in the launchers or the device code (the A/B switches are read once at load time, into
    gs_device.hpp's Knobs; the driver's at grid creation), and no timing-only build macros."""
    csrc = os.path.join(REPO, "gpu-solve_amd", "csrc")
    kern = open(os.path.join(csrc, "gs_kernels.hip")).read()
    dev = open(os.path.join(csrc, "gs_device.hpp")).read()
    assert "getenv" not in kern
    body = dev[dev.index("struct Knobs"):]
    body = body[body.index("const Knobs kKnobs;"):]
    assert "getenv" not in body
    assert "GS_PRO_EXP" not in dev + kern and "GS_PRO_HALF" not in dev + kern
    grid = open(os.path.join(csrc, "gs_grid.cpp")).read()
    ctor_end = grid.index("HipGridData::~HipGridData()")
    # after the constructor only trace mode's stop switch (no device) reads the environment
    assert [l.strip() for l in grid[ctor_end:].splitlines() if "getenv" in l] == [
        'const char* e = std::getenv("GS_TRACE_STOP_AFTER"); // read per call: tests switch it']


def test_python_binding_covers_headers():
    names = set(declared(os.path.join(REPO, "include", "gpusolve_hip.h")))
    assert names == set(gsv._abi.KERNEL_API), names ^ set(gsv._abi.KERNEL_API)
    names = set(declared(os.path.join(REPO, "include", "gpusolve_diag.h")))
    assert names == set(gsv._abi.DIAG_API), names ^ set(gsv._abi.DIAG_API)
    names = set(declared(os.path.join(REPO, "include", "gpusolve_driver.h")))
    assert names == set(gsv._abi.DRIVER_API), names ^ set(gsv._abi.DRIVER_API)


def test_libraries_load_without_gpu():
    k = gsv.kernels()
    d = gsv.driver()
    assert b"gpusolve_hip" in k.gs_build_info()
    assert k.gs_strerror(0) == b"success"
    assert b"invalid argument" in k.gs_strerror(gsv._abi.GS_EINVAL)
    assert d.gs_last_error() is not None


@pytest.mark.parametrize("dims", [(1, 1, 1), (7, 7, 7), (126, 3, 2), (127, 127, 127), (512, 512, 512),
                                  (1024, 1024, 128), (1023, 5, 9)])
def test_field_layout(dims):
    nx, ny, nz = dims
    ldy, ldz, alloc, origin = gsv.field_layout(*dims)
    assert ldy >= nx + 2 and ldy % 16 == 0          # x=1 of every row 128-B aligned
    assert (origin + 1) % 16 == 0
    assert ldz == ldy * (ny + 2)
    assert alloc >= origin + ldz * (nz + 2)
    assert ldy - (nx + 2) < 16                       # at most one cache line of pitch padding


def test_parse_config_example():
    with open(os.path.join(REPO, "tests", "golden", "data-2nd_order.conf")) as f:
        p = gsv.parse_config(f.read())
    assert (p.maxiter, p.tol, p.gridDim, p.mode) == (10, 1e-5, (127, 127, 127), gsv.GS_NEWTON)
    assert (p.preSmoothing, p.postSmoothing, p.omega, p.gamma) == (3, 3, 0.8, 1.0)
    assert p.stencil.values == [6, -1, -1, -1, -1, -1, -1]
    assert p.stencil.offsets == gsv.CANONICAL_OFFSETS
    assert p.h == 1.0 / 128
    # round trip through our own writer
    assert gsv.parse_config(p.config_text()) == p


def test_parse_config_rejects():
    text = open(os.path.join(REPO, "tests", "golden", "data-2nd_order.conf")).read().splitlines()
    bad_mode = list(text)
    bad_mode[5] = "3"
    with pytest.raises(ValueError, match="Invalid mode"):
        gsv.parse_config("\n".join(bad_mode))
    bad_off = list(text)
    bad_off[11] = "0 2 -1 0 0 0 0"
    with pytest.raises(ValueError, match="stencil"):
        gsv.parse_config("\n".join(bad_off))


def test_executable_argument_errors(tmp_path):
    """src/main.cpp:17-26,53-56: exit 1 for a missing / non-file config and an invalid mode."""
    exe = gsv._abi.EXECUTABLE
    assert os.path.exists(exe)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 1 and "Missing config file" in r.stderr
    r = subprocess.run([exe, str(tmp_path / "nope.conf")], capture_output=True, text=True)
    assert r.returncode == 1 and "does not exist or is not a file" in r.stderr
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 1
    conf = tmp_path / "bad.conf"
    conf.write_text("10\n0\n7\n7\n7\n5\n2\n2\n0.8\n1.0\n6 -1 -1 -1 -1 -1 -1\n0 1 -1 0 0 0 0\n0 0 0 1 -1 0 0\n"
                    "0 0 0 0 0 1 -1\n")
    r = subprocess.run([exe, str(conf)], capture_output=True, text=True)
    assert r.returncode == 1 and "Invalid mode" in r.stderr
    assert r.stdout.startswith(f'Using config file "{conf}"')


def test_executable_config_path_quoting_without_gpu(tmp_path):
    """src/main.cpp:24,28 stream a std::filesystem::path, i.e. through std::quoted ('"' and '\\' escaped).
    Byte-for-byte against the reference executable's transcripts (tests/golden/paths.json) for the cases
    that end before any device work: missing paths, and the 'Using config file' line of every other
    path (checked here on an invalid-mode copy of the config, which exits before the solve)."""
    from conftest import load_json
    exe = gsv._abi.EXECUTABLE
    for name, case in load_json("paths.json").items():
        rel_path = case["path"]
        if case["config"] is None:
            r = subprocess.run([exe, rel_path], cwd=tmp_path, capture_output=True, text=True)
            assert r.returncode == case["returncode"], name
            assert r.stdout.splitlines() == case["stdout"], name
            assert r.stderr.splitlines() == case["stderr"], (name, r.stderr)
        else:
            (tmp_path / rel_path).write_text("1\n0\n7\n7\n7\n9\n")
            r = subprocess.run([exe, rel_path], cwd=tmp_path, capture_output=True, text=True)
            assert r.returncode == 1 and r.stderr == "Invalid mode\n", name
            assert r.stdout.splitlines() == case["stdout"][:1], (name, r.stdout)
            (tmp_path / rel_path).unlink()
