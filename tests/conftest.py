"""Test configuration.

Markers:
  gpu  -- needs an MI355X (gfx950) and the built libmpt.so; parity tests proper, calling
          the product through its C ABI and checking it against the CPU oracle (oracle/).
Everything else runs on CPU: oracle self-checks against known answers / scipy / the
C++ standard library, host-side logic, and the C-ABI library's exported symbols.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libmpt.so")


@pytest.fixture(scope="session")
def mpt_gpu():
    """libmpt initialised on device 0 -- fails loudly (no CPU fallback) without a gfx950.
    torch's HIP runtime comes up first, as in bench.py, so tests that hand torch streams to
    the library (config 5's engines on streams) run in the same process layout."""
    import torch

    torch.cuda.init()
    import motionplanningtoolkit_amd as mpt

    mpt.init(0)
    return mpt


@pytest.fixture(scope="session")
def oracle():
    import oracle as orc

    orc.lib()
    return orc
