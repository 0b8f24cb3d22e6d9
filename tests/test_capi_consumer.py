"""The C-ABI from plain C (tests/native/capi_consumer.c): the header compiles as strict C99
(gcc -std=c99 -pedantic -Werror), the program links the in-tree library by name, and
- on the CPU: host-only entry points work (parameters, the static noise schedule, client key, raw
  encrypt / decrypt, the index-range guard) and context creation fails with TAE_E_NODEV (no CPU fallback);
- on the GPU: FIPS-197 C.1 end to end through the C-ABI alone (FHE key schedule on the encrypted key,
  10 rounds of the GalMul driver), decrypted to the published ciphertext."""
import os
import subprocess

import pytest

from tests.conftest import PKG, ROOT

LIBDIR = os.path.join(PKG, "tfhe_aes")


def _build(tmp_path):
    exe = str(tmp_path / "capi_consumer")
    subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-O1",
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "native", "capi_consumer.c"),
                    "-L", LIBDIR, "-l:libtfhe_aes_amd.so", "-Wl,-rpath," + LIBDIR, "-o", exe], check=True)
    return exe


def test_c_consumer_host(tmp_path):
    r = subprocess.run([_build(tmp_path), "host"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK")


@pytest.mark.gpu
def test_c_consumer_fips197_on_gpu(tmp_path):
    r = subprocess.run([_build(tmp_path), "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "69c4e0d86a7b0430d8cdb78070b4c55a" in r.stdout
