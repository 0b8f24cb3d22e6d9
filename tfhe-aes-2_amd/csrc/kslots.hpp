// Slot plan of the K-layout PFKS GEMM (ksgemm.hpp prep_digits_kl / prep_key_kl / gemm_g6<.., true>):
// which level and which 8-bit limb of its digit each of the S K-slots of a big-LWE coefficient
// carries.  Plain C++ so the host-side Engine header can hold one.
#pragma once
#include <cstdint>

namespace tae {
namespace ksgemm {

struct KSlots {
    int S = 0;        // slots per coefficient
    int lev[8];       // level index (0 = most significant) of slot s
    int limb[8];      // limb index of slot s (shift 8 limb)
    int nlimb[4];     // limbs of level l
    int first[4];     // first slot of level l
    int64_t off[4];   // digit offset c_l
};

// balanced n-byte range [-128 (256^n - 1) / 255, 127 (256^n - 1) / 255]
inline bool kslots_build(int base_log, int levels, KSlots &ks) {
    if (levels > 4 || base_log > 30) return false;
    ks.S = 0;
    for (int l = 0; l < levels; l++) {
        const int64_t half = 1ll << (base_log - 1);
        const int64_t lo = l == 0 ? -half + 1 : -half, hi = half;  // the top level drops its carry
        int n = 1;
        int64_t c = 0;
        for (;; n++) {
            if (n > 4) return false;
            int64_t span = 0;
            for (int t = 0; t < n; t++) span = span * 256 + 1;  // (256^n - 1) / 255
            const int64_t mn = -128 * span, mx = 127 * span;
            c = hi - mx > 0 ? hi - mx : 0;
            if (lo - c >= mn) break;
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

}  // namespace ksgemm
}  // namespace tae
