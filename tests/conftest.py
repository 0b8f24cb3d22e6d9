"""Shared fixtures.  `-m "not gpu"` runs here (no GPU); `-m gpu` runs on the MI355X box.

The oracle (oracle/) is test infrastructure: it is imported only from tests, smoke() and bench.py's
cpu_baseline leg, always as the checker.
"""
import os
import sys

import pytest

# PyTorch-ROCm bundles its own HIP runtime under the same soname as /opt/rocm's; whichever is loaded
# first serves the whole process, and torch cannot start on the other one.  Load torch's first, as
# bench.py does, so that tests which move keys to the GPU with torch work in any selection.
try:
    import torch  # noqa: F401
except ImportError:
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "tfhe-aes-2_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

SEED = bytes(range(32))          # FHE key seed used by every parity test (recorded in DESIGN.md)
ENC_SEED = bytes([0xA5] * 32)    # not used by the product (it encrypts under the key's own seed)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running (full 10-round AES on the CPU oracle)")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def oracle_keys(oracle_mod):
    """Oracle key set for params_sqrd_lvl_64 generated from SEED (keygen spec)."""
    return oracle_mod.Keys(oracle_mod.PARAMS_SQRD_LVL_64, SEED, threads=min(8, os.cpu_count() or 1))


@pytest.fixture(scope="session")
def product_raw():
    """Product client key + standard-domain server keys from the same SEED (host only)."""
    import tfhe_aes
    return tfhe_aes.generate_keys_raw(tfhe_aes.PARAMS_SQRD_LVL_64, SEED, threads=min(16, os.cpu_count() or 1))


@pytest.fixture(scope="session")
def gpu_context(product_raw):
    import tfhe_aes
    if tfhe_aes.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    _, keys = product_raw
    return tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, keys, device=0)


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "aes_golden.json")) as fh:
        return json.load(fh)


# ---- 8-bit model (param set 4, shortint_woppbs_8bit.rs:39-86) ----
@pytest.fixture(scope="session")
def oracle_keys8(oracle_mod):
    return oracle_mod.Keys(oracle_mod.PARAMS_WOPPBS_8BIT, SEED, threads=min(16, os.cpu_count() or 1))


@pytest.fixture(scope="session")
def product_raw8():
    import tfhe_aes
    return tfhe_aes.generate_keys_raw(tfhe_aes.PARAMS_WOPPBS_8BIT, SEED, threads=min(16, os.cpu_count() or 1))


@pytest.fixture(scope="session")
def gpu_context8(product_raw8):
    import tfhe_aes
    if tfhe_aes.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    _, keys = product_raw8
    return tfhe_aes.context_from_raw(tfhe_aes.PARAMS_WOPPBS_8BIT, keys, device=0)
