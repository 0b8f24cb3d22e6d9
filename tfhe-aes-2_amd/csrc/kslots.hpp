// Slot plan of the K-layout PFKS GEMM (ksgemm.hpp prep_digits_kl / prep_key_kl / gemm_g6<.., true>):
// which level and which 8-bit limb of its digit each of the S K-slots of a big-LWE coefficient
// carries.  Plain C++ so the host-side Engine header can hold one.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define TAE_KS_HD __host__ __device__
#else
#define TAE_KS_HD
#endif

namespace tae {
namespace ksgemm {

struct KSlots {
    int S = 0;        // slots per coefficient
    int lev[8];       // level index (0 = most significant) of slot s
    int limb[8];      // limb index of slot s (shift 8 limb)
    int nlimb[4];     // limbs of level l
    int first[4];     // first slot of level l
    int64_t off[4];   // digit offset c_l
    int clamp[4];     // 1: level l stores its rare digit +2^(B-1) as -2^(B-1) (see kslots_build)
};

// balanced n-byte range [-128 (256^n - 1) / 255, 127 (256^n - 1) / 255]: the fewest limbs n and the
// offset c that hold the digits [lo, hi] of a level
inline bool kslots_fit(int64_t lo, int64_t hi, int &n, int64_t &c) {
    for (n = 1; n <= 4; n++) {
        int64_t span = 0;
        for (int t = 0; t < n; t++) span = span * 256 + 1;  // (256^n - 1) / 255
        const int64_t mn = -128 * span, mx = 127 * span;
        c = hi - mx > 0 ? hi - mx : 0;
        if (lo - c >= mn) return true;
    }
    return false;
}

// The lower levels' balanced digits span [-2^(B-1), 2^(B-1)]: 2^B + 1 values, one more than B bits
// hold, and +2^(B-1) only comes up when a level's residue is exactly half the base and the carry rule
// keeps it (probability ~2^-(B+1) per digit).  With clamp allowed, such a level stores that digit as
// -2^(B-1) whenever this saves a limb (base 2^16: 2 limbs instead of 3, i.e. 4 slots per coefficient
// instead of 5 for params_sqrd_lvl_64), and the GEMM output is corrected afterwards by
// -2^B KEY[i][l][col] for every (ciphertext, i, l) it happened to (ksgemm.hpp pfks_clamp_fixup).
inline bool kslots_build(int base_log, int levels, KSlots &ks, bool allow_clamp = true) {
    if (levels > 4 || base_log > 30) return false;
    ks.S = 0;
    for (int l = 0; l < levels; l++) {
        const int64_t half = 1ll << (base_log - 1);
        const int64_t lo = l == 0 ? -half + 1 : -half, hi = half;  // the top level drops its carry
        int n, n2;
        int64_t c, c2;
        if (!kslots_fit(lo, hi, n, c)) return false;
        ks.clamp[l] = 0;
        if (allow_clamp && l > 0 && kslots_fit(lo, hi - 1, n2, c2) && n2 < n) {
            n = n2;
            c = c2;
            ks.clamp[l] = 1;
        }
        if (ks.S + n > 8) return false;
        ks.nlimb[l] = n;
        ks.first[l] = ks.S;
        ks.off[l] = c;
        for (int t = 0; t < n; t++) {
            ks.lev[ks.S] = l;
            ks.limb[ks.S] = t;
            ks.S++;
        }
    }
    return true;
}

// The balanced digits of x (tfhe-rs SignedDecomposer: closest representable, then the carry rule of
// decompose_one_level), least significant level first: f(lev, digit) for lev = levels .. 1.
template <class F>
TAE_KS_HD inline void kl_for_each_digit(uint64_t x, int base_log, int levels, F &&f) {
    const int nrb = 64 - base_log * levels;
    uint64_t s = x >> (nrb - 1);
    s += s & 1;
    s >>= 1;
    const uint64_t mask = (1ull << base_log) - 1;
    for (int lev = levels; lev >= 1; lev--) {
        const uint64_t res = s & mask;
        s >>= base_log;
        uint64_t carry = ((res - 1) | s) & res;
        carry >>= (base_log - 1);
        s += carry;
        f(lev, (int64_t)(res - (carry << base_log)));
    }
}

// The next signed 8-bit limb of an offset digit d (least significant first; the last limb takes the
// rest, which the slot plan keeps in [-128, 127]); d is left holding the limbs still to come.
TAE_KS_HD inline int64_t kl_next_limb(int64_t &d, bool last) {
    if (last) return d;
    const int64_t limb = ((d + 128) & 255) - 128;
    d = (d - limb) >> 8;
    return limb;
}

}  // namespace ksgemm
}  // namespace tae
