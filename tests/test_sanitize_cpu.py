"""CPU: AddressSanitizer + UndefinedBehaviorSanitizer builds.

* the oracle (oracle/mpt_oracle.c) driven through every entry point by
  oracle/sanitize_check.c, which also cross-checks the kd-tree against brute-force kNN and the
  AABB-tree collider against the all-pairs definition;
* the host mirror's device-free code (mesh readers, `.inst` parsing) on every mesh fixture, the
  reference's own mesh files when present, and truncated / byte-flipped copies of each.
Both builds use -fno-sanitize-recover, so any report fails the run."""
import glob
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_MESHES = "/root/reference/mesh_models"


def _make(directory, target):
    subprocess.run(["make", "-s", "-C", directory, target], check=True, capture_output=True, timeout=300)


@pytest.mark.timeout(600)
def test_oracle_under_asan_ubsan():
    _make(os.path.join(REPO, "oracle"), "sanitize")
    exe = os.path.join(REPO, "oracle", "_build", "sanitize_check")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize_check ok" in r.stdout


@pytest.mark.timeout(600)
def test_host_mirror_under_asan_ubsan():
    csrc = os.path.join(REPO, "motionplanningtoolkit_amd", "csrc")
    _make(csrc, "sanitize")
    exe = os.path.join(REPO, "motionplanningtoolkit_amd", "_lib", "sanitize_host")
    files = sorted(glob.glob(os.path.join(REPO, "tests", "golden", "meshes", "*.obj")))
    files += sorted(glob.glob(os.path.join(REPO, "instances", "*.inst")))
    if os.path.isdir(REF_MESHES):
        files += sorted(glob.glob(os.path.join(REF_MESHES, "*", "*.3ds")))
        files += sorted(glob.glob(os.path.join(REF_MESHES, "*", "*.dae")))
    r = subprocess.run([exe] + files, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("sanitize_host ok")
