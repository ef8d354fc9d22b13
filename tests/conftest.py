"""Shared pytest setup.

Markers: ``gpu`` -- needs an MI355X (run with ``-m gpu`` on the GPU box); everything else runs on CPU.
The native libraries are built in-tree (glint_amd/build.py) before the session if they are stale.
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950)")
    config.addinivalue_line("markers", "slow: long-running")
    # by path: importing the glint_amd package loads libglint_gpu.so, which a fresh checkout lacks
    import importlib.util
    spec = importlib.util.spec_from_file_location("_glint_build", ROOT / "glint_amd" / "build.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.build_all()


@pytest.fixture(scope="session")
def kat():
    import json
    return json.loads((ROOT / "tests" / "golden" / "reference_kat.json").read_text())


@pytest.fixture(scope="session")
def gpu():
    """Device index used by GPU tests. Fails (never skips) when no GPU is visible: `-m gpu` runs are
    meant for the MI355X box, and a silent skip would hide a broken HIP path."""
    import glint_amd._native as N
    if N.load().glint_device_count() < 1:
        pytest.fail("no GPU visible to libglint_gpu.so")
    return int(os.environ.get("GLINT_TEST_DEVICE", "0"))


@pytest.fixture(autouse=True)
def _glint_env_knobs():
    """libglint_gpu.so caches its GLINT_* environment knobs; a test that sets one calls
    ``N.reload_env()``, and every test ends with a reload (after monkeypatch has restored the
    environment), so no knob leaks into the next test."""
    yield
    import glint_amd._native as N
    if N._lib is not None:
        N.reload_env()
