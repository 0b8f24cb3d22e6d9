"""LDS bank-conflict properties of the blind rotations' spectrum layouts, against the lane-group model of
MI355X_MICROARCH.md's LDS table (scripts/layout/): CPU only.

- br512x4 / br512lat: the slot tables SF, SG1, SG3 shipped in br512x4.hpp (parsed from the header) put
  256 distinct slots inside BUF_STRIDE and no two lanes of a ds_read_b128 / ds_write_b128 group on one
  bank for every access pattern of the kernel (passes A / B and their inverses, the MAC loads / stores).
- br1024 / br1024lat: the MAC's thread -> Fourier position map (mac_pos, mirrored from br1024.hpp and
  checked against the header's text) is a bijection of the 512 positions and conflict-free, and no
  sum-separable octal-digit table can make the pass-0 reads and pass-2 writes conflict-free together
  (b1k_sep_feasibility.c, exhaustive)."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts", "layout"))

import b1k_banks  # noqa: E402
import x4_banks  # noqa: E402


def _header(name):
    return open(os.path.join(ROOT, "tfhe-aes-2_amd", "csrc", name)).read()


def _table(src, name):
    m = re.search(r"\b%s\[\d+\]\s*=\s*\{([^}]*)\}" % name, src)
    return [int(x) for x in m.group(1).split(",")]


def test_br512x4_spectrum_layout_is_conflict_free():
    src = _header("br512x4.hpp")
    t = (_table(src, "SF"), _table(src, "SG1"), _table(src, "SG3"))
    stride = int(re.search(r"BUF_STRIDE\s*=\s*(\d+)", src).group(1))
    ok, span = x4_banks.valid(t)
    assert ok and span <= stride, (ok, span, stride)
    costs = x4_banks.cost(t, x4_banks.patterns())
    assert all(c == 0 for c in costs.values()), costs


def test_br1024_mac_positions():
    src = _header("br1024.hpp")
    body = re.search(r"int mac_pos\(int tid\) \{(.*?)\n\}", src, re.S).group(1)
    # the Python mirror checks the formula the header holds
    assert "const int j = (h & 8 ? 4 : 0) + ((o & 1) << 1) + (o >> 1);" in body
    assert "return 8 * ((h & 7) + 8 * j) + (tid & 7);" in body
    bijective, rd, wr = b1k_banks.mac_check()
    assert bijective and rd == 0 and wr == 0
    assert b1k_banks.mac_check(lambda t: t)[1] > 0  # consecutive positions do conflict


def test_br1024_separable_tables_cannot_be_conflict_free(tmp_path):
    exe = str(tmp_path / "sep")
    subprocess.run(["gcc", "-O2", os.path.join(ROOT, "scripts", "layout", "b1k_sep_feasibility.c"), "-o", exe],
                   check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300).stdout
    assert "found 0" in out


def test_fft_torus_1024_final_reads_conflict_free():
    import fft1k_banks
    src = _header("kernels.hip")
    assert _table(src, "kFftTau1k") == fft1k_banks.tau()
    t = fft1k_banks.tau()
    fs = sorted(128 * (c >> 1) + 32 * (c & 1) + t[u] for c in range(8) for u in range(64))
    assert fs == list(range(512))  # every output once
    # each read instruction stores whole 128-byte lines (8 complex values)
    for c in range(8):
        blocks = {}
        for u in range(64):
            f = 128 * (c >> 1) + 32 * (c & 1) + t[u]
            blocks.setdefault(f >> 3, set()).add(f & 7)
        assert all(len(v) == 8 for v in blocks.values())
    ex = fft1k_banks.extra_cycles()
    assert ex["final_read_lane_order"] > 0
    assert all(v == 0 for k, v in ex.items() if k != "final_read_lane_order"), ex
