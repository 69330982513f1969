import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def port():
    import oracle
    return oracle.Port()


@pytest.fixture(scope="session")
def ff_golden():
    meta = json.load(open(os.path.join(GOLDEN, "ff_cases.json")))
    arrs = np.load(os.path.join(GOLDEN, "ff_cases.npz"), allow_pickle=False)
    return meta, arrs


@pytest.fixture(scope="session")
def scenario_golden():
    return json.load(open(os.path.join(GOLDEN, "scenarios.json")))


@pytest.fixture(scope="session")
def ctx():
    import torch
    from parameter_server_amd import filter as F
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = F.Context(0)
    yield c
    c.sync()
