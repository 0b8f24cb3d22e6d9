"""LDS bank-conflict model of br512p16 (16 points per lane, tfhe-aes-2_amd/csrc/br512p16.hpp) against the
lane-group model of MI355X_MICROARCH.md's LDS table.

Forward job regions (4096 B, one per FFT job) hold position P = a + 16 b at slot16(P) = 16 b + (a ^ b) (an XOR
swizzle: every access is a lane base XOR a compile-time constant, one VALU op, plus an immediate offset).
A wave runs four jobs (lanes 16 jj + u, jj = 0..3, u = 0..15), job regions 4 KiB apart:
  - pass A store: lane u of job jj writes P = u + 16 k (k fixed per instruction);
  - pass B load / store: lane kappa = u reads / writes P = lam + 16 kappa (lam fixed per instruction);
  - digits: job slots 1 KiB apart, layout [r][u][i] (16 B per (r, u)); the writer is the decomposition lane
    (u, r) = (l & 15, l >> 4) of a polynomial wave, the reader lane u of job jj reads r = 0..3;
  - MAC loads: thread lane l (wave block w4 = wave & 3) on position mac_pos(64 w4 + l), every job region;
  - MAC stores into the inverse regions, br512x4's sidx layout (x4_banks.sidx), same positions.
Read b128: bank group = 16-B unit mod 16 over the four 16-lane groups; write b128: unit mod 8 over 8-lane groups."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import x4_banks  # noqa: E402

RD, WR = x4_banks.RD, x4_banks.WR
X4_TABLES = ([-36, -45, -39, -38, -37, -30, -44, -31, -22, -55, -29, -20, -47, -28, -14, -53], [42, 78, 74, 46],
             [13, 81, 157, 225])


def slot16(P):
    a, b = P & 15, P >> 4
    return 16 * b + (a ^ b)


def mac_pos(t):
    """MAC thread t (0..255 within a 256-thread slot group) -> Fourier position (slot16(mac_pos(t)) = t)"""
    b = t >> 4
    return 16 * b + ((t & 15) ^ b)


def patterns():
    """(name, kind, lane -> 16-byte unit address)"""
    P = []
    job = lambda l: (l >> 4) * 256  # job regions 4096 B = 256 units apart
    for k in range(16):
        P.append((f"passA_st{k}", "w", lambda l, k=k: job(l) + slot16((l & 15) + 16 * k)))
    for lam in range(16):
        f = lambda l, lam=lam: job(l) + slot16(lam + 16 * (l & 15))
        P.append((f"passB_ld{lam}", "r", f))
        P.append((f"passB_st{lam}", "w", f))
    for r in range(4):  # digit reader: job jj's slot 64 units apart, [r][u][i] -> unit 16 r + u
        P.append((f"dig_ld{r}", "r", lambda l, r=r: (l >> 4) * 64 + 16 * r + (l & 15)))
    P.append(("dig_st", "w", lambda l: 16 * (l >> 4) + (l & 15)))  # writer lane (u, r): unit 16 r + u
    for w4 in range(4):
        P.append((f"mac_ld{w4}", "r", lambda l, w4=w4: slot16(mac_pos(64 * w4 + l))))
        P.append((f"mac_st{w4}", "w", lambda l, w4=w4: x4_banks.sidx(X4_TABLES, mac_pos(64 * w4 + l))))
    return P


def cost(P=None):
    out = {}
    for name, kind, f in P or patterns():
        groups, mod = (RD, 16) if kind == "r" else (WR, 8)
        c = 0
        for g in groups:
            cnt = {}
            for l in g:
                b = f(l) % mod
                cnt[b] = cnt.get(b, 0) + 1
            c += max(cnt.values()) - 1
        out[name] = c
    return out


def bijective():
    return sorted(slot16(P) for P in range(256)) == list(range(256)) and \
        sorted(mac_pos(t) for t in range(256)) == list(range(256))


if __name__ == "__main__":
    c = cost()
    print("bijective:", bijective())
    print({k: v for k, v in c.items() if v})
    print("total extra cycles per job-wave pattern set:", sum(c.values()))
