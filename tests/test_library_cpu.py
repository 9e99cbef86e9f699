"""CPU: the C-ABI library builds, loads and exports every declared symbol; host-side
logic that needs no device (mesh loading) matches the fixtures."""
import ctypes
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
