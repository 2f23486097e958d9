"""Shared pytest setup.  GPU tests are marked ``gpu`` and run on an MI355X
with ``pytest -m gpu``; everything else runs on CPU (``-m "not gpu"``)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GAMMA = np.float32(0.95)


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs an MI355X GPU (run with -m gpu)")


def golden_map(name):
    return np.load(os.path.join(GOLDEN, "maps", name + ".npy"), allow_pickle=False)


def golden(kind, name):
    with np.load(os.path.join(GOLDEN, f"{kind}_{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def assert_rel_close(got, want, rel=1e-5, abs_floor=np.finfo(np.float32).tiny, msg=""):
    """|got - want| <= rel*|want| or <= abs_floor (FTZ floor), elementwise."""
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    err = np.abs(got - want)
    ok = (err <= rel * np.abs(want)) | (err <= abs_floor)
    if not ok.all():
        i = int(np.argmax(~ok.reshape(-1)))
        raise AssertionError(
            f"{msg}: {int((~ok).sum())} of {ok.size} elements differ; first at "
            f"{i}: got {got.reshape(-1)[i]!r} want {want.reshape(-1)[i]!r}")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O
