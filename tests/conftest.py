"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X); run with -m gpu")


@pytest.fixture(scope="session", autouse=True)
def built():
    """Build the library, CLI, generator and oracle once per session.  A GPU-box
    snapshot carries the prebuilt libraries and binaries but not `build/`
    (.gpurunignore): those are used as shipped, not rebuilt there."""
    shipped = [os.path.join(REPO, p) for p in
               ("grom_amd/lib/libgrom_amd.so", "grom_amd/bin/grom", "grom_amd/bin/grom_synth",
                "oracle/grom_oracle", "oracle/liboracle.so")]
    if not os.path.isdir(os.path.join(REPO, "build")) and all(os.path.exists(p) for p in shipped):
        return True
    r = subprocess.run(["make", "-j8", "all"], cwd=REPO, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("make failed:\n" + r.stdout[-4000:] + r.stderr[-4000:])
    return True


@pytest.fixture(scope="session")
def datadir(tmp_path_factory):
    return tmp_path_factory.mktemp("grom_data")
