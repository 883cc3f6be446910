import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libwpt.so's HIP kernels)")


@pytest.fixture(scope="session")
def wpt():
    import wpt_loader
    return wpt_loader.load()


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    return pyoracle


@pytest.fixture(scope="session")
def cloud_small(wpt):
    return wpt.scenes.triangle_cloud(3000, seed=0x5EED)


@pytest.fixture(scope="session")
def cloud_100k(wpt):
    path = os.path.join(GOLDEN, "cloud_100k.npy")
    if os.path.exists(path):
        return np.load(path, allow_pickle=False)
    return wpt.scenes.triangle_cloud(100000, seed=0x5EED)
