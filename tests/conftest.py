"""Shared fixtures.  ``-m gpu`` tests call libpano through the C-ABI on a real MI355X;
``-m "not gpu"`` tests pin the oracle to the golden vectors and check host logic + ABI."""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs through libpano")
    config.addinivalue_line("markers", "slow: takes more than ~20 s on the CPU")


def digest(a) -> str:
    """SHA-256 over dtype, shape and bytes (same as tests/golden/make_golden.py)."""
    a = np.ascontiguousarray(a)
    h = hashlib.sha256()
    h.update(f"{a.dtype.str}{a.shape}".encode())
    h.update(a.tobytes())
    return h.hexdigest()


def load_json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def load_npz(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


@pytest.fixture(scope="session")
def gold_json():
    return load_json


@pytest.fixture(scope="session")
def gold_npz():
    return load_npz


@pytest.fixture(scope="session")
def parrington():
    from vfx_image_stitching_amd import data
    return data.load_set("parrington")


@pytest.fixture(scope="session")
def grail():
    from vfx_image_stitching_amd import data
    return data.load_set("grail")


@pytest.fixture(scope="session")
def outset():
    from vfx_image_stitching_amd import data
    return data.load_set("out")


@pytest.fixture(scope="session")
def parrington_cyl(parrington):
    """Oracle cylindrical frames (digest-checked against the reference in test_oracle)."""
    from oracle import stitch
    names, frames, focals, margin = parrington
    return [stitch.cylindrical(f, fl) for f, fl in zip(frames, focals)]


@pytest.fixture(scope="session")
def gpu():
    """The libpano context on cuda:0 -- fails loudly if the HIP path cannot run."""
    import torch
    from vfx_image_stitching_amd import _lib
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return _lib.context(0)
