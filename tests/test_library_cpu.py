"""CPU: the C-ABI library builds, loads and exports every declared symbol; host-side
logic that needs no device (mesh loading) matches the fixtures."""
import ctypes
import shutil
import subprocess
import os
import re

import numpy as np
import pytest

import motionplanningtoolkit_amd as mpt
from motionplanningtoolkit_amd import _native, scenes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(REPO, "include", h) for h in ("mpt.h", "mpt_host.h")]
REF_MESHES = "/root/reference/mesh_models"


def declared_symbols():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(mpt_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_native.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 35
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the Python binding covers the same set
    assert set(syms) == set(_native.SIGNATURES), set(syms) ^ set(_native.SIGNATURES)


def test_library_targets_gfx950_only():
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    for other in (b"gfx942", b"gfx90a", b"gfx1100"):
        assert b"amdgcn-amd-amdhsa--" + other not in data


def test_version_and_error_plumbing():
    assert mpt.lib().mpt_version() == 100
    # invalid arguments are reported, not thrown/exited, even without a device
    st = mpt.lib().mpt_nn_create(0, 10, None)
    assert st != 0
    assert len(mpt.lib().mpt_last_error()) > 0


@pytest.mark.parametrize("name,which", [("agent_unit_box", "last"), ("agent_blimp", "all"),
                                        ("agent_blimp", "last"), ("env_model", "all"), ("env_corridor", "all")])
def test_cpp_loader_reads_obj_fixtures(name, which):
    a = mpt.load_mesh(scenes.mesh_path(name), which)
    b = scenes.read_obj(scenes.mesh_path(name), which)
    assert a.shape == b.shape
    assert np.array_equal(a, b)


def test_blimp_submesh_split():
    assert mpt.load_mesh(scenes.mesh_path("agent_blimp"), "all").shape[0] == 1355
    assert mpt.load_mesh(scenes.mesh_path("agent_blimp"), "last").shape[0] == 32  # Blimpmain1


@pytest.mark.skipif(not os.path.isdir(REF_MESHES), reason="reference meshes not present")
@pytest.mark.parametrize("rel,fixture", [
    ("agent_models/unit_box.dae", "agent_unit_box"),
    ("agent_models/blimp.3ds", "agent_blimp"),
    ("environment_models/model.dae", "env_model"),
    ("environment_models/unit_box.dae", "env_unit_box"),
])
def test_cpp_loader_reads_reference_formats(rel, fixture):
    """The C++ .dae/.3ds readers and the independent Python converter agree exactly."""
    a = mpt.load_mesh(os.path.join(REF_MESHES, rel), "all")
    b = scenes.read_obj(scenes.mesh_path(fixture), "all")
    assert np.array_equal(a, b)


@pytest.mark.skipif(not os.path.isdir(REF_MESHES), reason="reference meshes not present")
def test_cpp_loader_divider_dae():
    t = mpt.load_mesh(os.path.join(REF_MESHES, "environment_models/divider.dae"), "all")
    assert t.shape[0] > 1000 and np.isfinite(t).all()


def test_synthetic_envs():
    c = scenes.corridor_env(0)
    assert c.shape == (2664, 9)
    assert np.array_equal(c, scenes.corridor_env(0))
    r = scenes.rooms_env(3, 2)
    assert r.shape == (6 * 316, 9)


_SEG_PROBE = r"""
#define __HIP_PLATFORM_AMD__ 1
#include "fcl_math.h"
#include <cstdio>
#include <cstring>
#include <random>
using namespace mpt;
static bool same(v3 a, v3 b) { return !memcmp(&a.x, &b.x, 8) && !memcmp(&a.y, &b.y, 8) && !memcmp(&a.z, &b.z, 8); }
int main() {
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> U(-2, 2);
    long bad = 0;
    for (long it = 0; it < 2000000; ++it) {
        v3 P = mk(U(g), U(g), U(g)), A = mk(U(g), U(g), U(g)), Q = mk(U(g), U(g), U(g)), B = mk(U(g), U(g), U(g));
        switch (it % 8) {
            case 1: B = scale(A, U(g)); break;                                 // parallel
            case 2: A = mk(0, 0, 0); break;                                    // zero-length
            case 3: B = mk(0, 0, 0); break;
            case 4: Q = add(P, scale(A, U(g))); B = scale(A, U(g)); break;     // collinear
            case 5: Q = P; break;
            case 6: A = mk(1e-300, 0, 0); break;
            default: break;
        }
        v3 V1, X1, Y1, V2, X2, Y2;
        seg_points(P, A, Q, B, V1, X1, Y1);
        seg_points_sel(P, A, Q, B, V2, X2, Y2);
        if (!same(V1, V2) || !same(X1, X2) || !same(Y1, Y2)) ++bad;
    }
    printf("%ld\n", bad);
    return 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"), reason="needs g++ and HIP headers")
def test_seg_points_branch_free_matches_branchy(tmp_path):
    """k_distance's branch-free segPoints (fcl_math.h seg_points_sel) returns the branchy
    form's (seg_points, FCL's TriangleDistance::segPoints restated) points and direction bit for
    bit, on 2 M random segment pairs with parallel, collinear and zero-length cases (the header
    is host + device code; the host build checks the arithmetic, -ffp-contract=off as the
    device build)."""
    src, exe = tmp_path / "seg.cpp", tmp_path / "seg"
    src.write_text(_SEG_PROBE)
    csrc = os.path.join(REPO, "motionplanningtoolkit_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", csrc, "-I", "/opt/rocm/include", "-x",
                    "c++", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.strip()
    assert out == "0"


_HEAD_PROBE = r"""
#define __HIP_PLATFORM_AMD__ 1
#include "fcl_math.h"
#include <cstdio>
#include <cstring>
#include <random>
using namespace mpt;
template <int D, int NG>
static long check(std::mt19937_64 &g) {
    std::uniform_real_distribution<double> U(-50, 50);
    long bad = 0;
    double a[D], b[D];
    for (long it = 0; it < 300000; ++it) {
        for (int i = 0; i < D; ++i) {
            a[i] = U(g);
            b[i] = (it % 4 == 1 && i < 4 * NG) ? a[i] : U(g);  // head exactly zero
        }
        const double full = flann_l2<D>(a, b), head = flann_l2_head<NG>(a, b);
        const double rest = flann_l2_rest<D, NG>(a, b, head);
        if (memcmp(&full, &rest, 8) != 0 || head > full) ++bad;
    }
    return bad;
}
int main() {
    std::mt19937_64 g(11);
    printf("%ld\n", check<15, 1>(g) + check<15, 2>(g) + check<8, 1>(g) + check<8, 2>(g) + check<13, 3>(g));
    return 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"), reason="needs g++ and HIP headers")
def test_flann_l2_head_rest_split(tmp_path):
    """The NN run kernel's head screen (grid_nn.hip, long records): FLANN's L2 sum split into its
    first groups of four (fcl_math.h flann_l2_head) and the rest continued from them
    (flann_l2_rest) equals flann_l2 bit for bit, and the head never exceeds the full sum, so a
    point skipped because its head exceeds the best cannot be better."""
    src, exe = tmp_path / "head.cpp", tmp_path / "head"
    src.write_text(_HEAD_PROBE)
    csrc = os.path.join(REPO, "motionplanningtoolkit_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", csrc, "-I", "/opt/rocm/include", "-x",
                    "c++", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.strip()
    assert out == "0"


def test_mesh_dir_override(tmp_path):
    """MPT_MESH_DIR (the one path variable) redirects scenes.mesh_path."""
    code = "from motionplanningtoolkit_amd import scenes; print(scenes.mesh_path('env_model'))"
    env = dict(os.environ, MPT_MESH_DIR=str(tmp_path))
    out = subprocess.run(["python", "-c", code], cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().startswith(str(tmp_path))


def test_bench_line_fits_the_driver_tail():
    """bench.py prints a condensed line (the full one goes to --detail): for a full round-4 line
    with every leg (tests/golden/bench/full_line_r20.json, 17 KB) it stays under 8 KB -- the
    driver keeps the last 8 KB of stdout -- and keeps every leg's value, time and roofline."""
    import json
    import sys

    sys.path.insert(0, REPO)
    import bench

    full = json.load(open(os.path.join(REPO, "tests", "golden", "bench", "full_line_r20.json")))
    line = bench.compact_line(full, os.path.join(REPO, "gpurun_out", "bench_detail.json"))
    text = json.dumps(line)
    assert len(text) < 6000, len(text)
    assert line["value"] == full["value"] and line["roofline"]["frac"] == full["roofline"]["frac"]
    for name, leg in full["variants"].items():
        got = line["variants"][name]
        assert got["value"] == leg["value"] and got.get("ms_per_step") == leg.get("ms_per_step")
        assert got["roofline"]["frac"] == leg["roofline"]["frac"]
    assert line["variants"]["seeds=256"]["seeds_digest"] == full["variants"]["seeds=256"]["seeds_digest"]
    assert line["config5"]["per_gpu_ratio"] == full["config5"]["per_gpu_ratio"]


def test_bench_config5_keys_at_every_n():
    """The c5_* keys carry config 5 under one name at N = 1 (from the seeds=256 leg run beside
    config 2) and at N > 1 (the leg run in the same world), and survive the printed line; equal
    trees give equal c5_seeds_digest."""
    import copy
    import json
    import sys

    sys.path.insert(0, REPO)
    import bench

    full = json.load(open(os.path.join(REPO, "tests", "golden", "bench", "full_line_r20.json")))
    variants = full["variants"]
    one = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "scaling")}
    bench.attach_config5(one, None, variants)
    leg = variants["seeds=256"]
    two_leg = dict(copy.deepcopy(leg), world_size=2, n_gpus=2, value=2 * leg["value"])
    two = dict(one, n_gpus=2)
    for k in ("variants", "config5"):
        two.pop(k)
    bench.attach_config5(two, two_leg)
    for line, ws in ((one, 1), (two, 2)):
        printed = bench.compact_line(line, None)
        assert printed["c5_value"] == line["c5_value"] and printed["c5_world_size"] == ws
        assert printed["scaling_basis"] == bench.SCALING_BASIS and printed["c5_scaling"] == "strong"
        assert printed["c5_seeds_digest"] == leg["seeds_digest"] == printed["config5"]["seeds_digest"]
        assert printed["c5_ms_per_step"] == line["config5"]["ms_per_step"]
    assert two["c5_value"] == 2 * one["c5_value"]
    assert "per_gpu_ratio" in one["config5"] and "per_gpu_ratio" not in two["config5"]
    assert bench.c5_keys(None)["c5_value"] is None


def test_bench_gpus_must_match_world_size():
    """Under torchrun, --gpus N must equal WORLD_SIZE (checked before anything is imported)."""
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys_executable(), os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def sys_executable():
    import sys

    return sys.executable
