"""Host-compiled checks of device helpers: the integer-only torus helpers of the blind-rotation kernels
(fft_device.hpp from_torus_bits, decompose16) against the CPU oracle's tfhe-rs restatement
(or_from_torus, or_decompose) on random and edge-case inputs (tests/native/torus_helpers_test.cpp), and
the K-layout PFKS slot plan (kslots.hpp, tests/native/kslots_test.cpp), and the fused-twiddle transforms'
constant tables of the product against the oracle's plans (tests/native/lf_tables_test.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_torus_helpers_match_oracle(tmp_path):
    exe = str(tmp_path / "torus_helpers_test")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950",
                    os.path.join(ROOT, "tests", "native", "torus_helpers_test.cpp"), "-x", "none",
                    os.path.join(ROOT, "oracle", "build", "liboracle.so"), "-o", exe,
                    "-Wl,-rpath," + os.path.join(ROOT, "oracle", "build")], check=True)
    r = subprocess.run([exe, "1000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


def test_pfks_slot_plan(tmp_path):
    """K-layout PFKS slot plan (csrc/kslots.hpp): digit ranges, exact limb split of every digit and the
    pre-shifted-key identity, on the base 2^16 x 2 and 2^12 x 3 shapes (tests/native/kslots_test.cpp)."""
    exe = str(tmp_path / "kslots_test")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "native", "kslots_test.cpp"), "-o", exe],
                   check=True)
    r = subprocess.run([exe, "2000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


def test_lf_tables_match_oracle(tmp_path):
    """The product's fused-transform tables (client.cpp make_lf512_table / make_lf1k_table, what the
    kernels stage) equal the oracle plans' constants bit for bit (tests/native/lf_tables_test.cpp; loads
    the product library, no GPU call)."""
    exe = str(tmp_path / "lf_tables_test")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tfhe-aes-2_amd")], check=True)
    lib = os.path.join(ROOT, "tfhe-aes-2_amd", "tfhe_aes")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "native", "lf_tables_test.cpp"),
                    os.path.join(ROOT, "oracle", "build", "liboracle.so"), os.path.join(lib, "libtfhe_aes_amd.so"),
                    "-o", exe, "-Wl,-rpath," + os.path.join(ROOT, "oracle", "build") + ":" + lib], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
