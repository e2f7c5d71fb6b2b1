"""Shared test setup: import paths, the `gpu` marker, golden-fixture loaders.

`-m "not gpu"` tests run here (no GPU): oracle vs golden fixtures, host logic, C-ABI exports.
`-m gpu` tests run on the MI355X box and call the HIP library through the C ABI.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ldpc-neuralnetwork-decoder_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
CODES = os.path.join(ROOT, "codes")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and libldpc_amd.so")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def code_path(z):
    return os.path.join(CODES, f"NR_2_0_{z}.txt")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)
