import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("hadoop-bam_amd", "oracle", "tools"):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhbam.so)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def genbam():
    import genbam as g
    g.lib()
    return g


@pytest.fixture(scope="session")
def small_bam(genbam):
    """Config #1 stand-in: committed fixture if present, else the same generator call."""
    path = os.path.join(GOLDEN, "small_pe.bam")
    if os.path.exists(path):
        return np.fromfile(path, dtype=np.uint8)
    return np.asarray(genbam.generate(**SMALL_PE_PARAMS))


# the committed fixture's generator parameters (tests/golden/make_golden.py)
SMALL_PE_PARAMS = dict(records=20000, seed=1, odd_every=211, long_every=7919,
                       mate_unmapped_permille=15, threads=4)


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch  # noqa: F401  (its HIP runtime opens the device before libhbam's)
    from hadoop_bam import _lib
    try:
        return _lib.Context(0)
    except _lib.HbamUnavailable as e:
        pytest.fail("GPU test without a usable HIP device/libhbam.so: %s" % e)
