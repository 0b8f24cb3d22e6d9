// Host test of the K-layout PFKS slot plan (tfhe-aes-2_amd/csrc/kslots.hpp), the digit and limb code the
// prep_digits_kl kernel runs:
//   1. every digit the decomposer can produce (random inputs and edge patterns) lies in the level's
//      range the plan was sized for, and the digits recompose to the closest representable value;
//   2. for EVERY digit of that range, the offset digit splits into limbs in [-128, 127] that
//      recombine exactly;
//   3. with random u64 keys, sum_m limb_m (KEY << 8 m) + c KEY == digit KEY (mod 2^64), the identity
//      the GEMM (pre-shifted key rows) plus the per-column correction rely on; on a clamped level the
//      digit +2^(B-1) is stored as -2^(B-1) and the identity holds with pfks_clamp_fixup's extra
//      KEY << B term.  Both plans (clamping allowed, the default, and not: TAE_PFKS_LAYOUT=k5).
// Shapes: the MFMA PFKS sets, base 2^16 x 2 levels (params_sqrd_lvl_4 / _64) and 2^12 x 3 (lvl_256,
// the 8-bit model).  Usage: kslots_test [random inputs]; prints OK.
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../../tfhe-aes-2_amd/csrc/kslots.hpp"

using tae::ksgemm::KSlots;

static int fails = 0;
#define CHECK(c, ...)                          \
    do {                                       \
        if (!(c)) {                            \
            if (fails++ < 20) {                \
                std::printf("FAIL: " __VA_ARGS__); \
                std::printf("\n");             \
            }                                  \
        }                                      \
    } while (0)

static void run_shape(int base_log, int levels, long n_random, bool clamp) {
    KSlots ks;
    CHECK(tae::ksgemm::kslots_build(base_log, levels, ks, clamp), "plan for 2^%d x %d", base_log, levels);
    CHECK(ks.S <= 8, "S = %d", ks.S);
    const int64_t half = 1ll << (base_log - 1);
    std::mt19937_64 rng(base_log * 131 + levels);

    // 1. digit ranges and recomposition
    auto check_x = [&](uint64_t x) {
        int64_t d[4] = {0, 0, 0, 0};
        tae::ksgemm::kl_for_each_digit(x, base_log, levels, [&](int lev, int64_t v) { d[lev - 1] = v; });
        uint64_t rec = 0;
        for (int l = 0; l < levels; l++) {
            const int64_t lo = l == 0 ? -half + 1 : -half;
            CHECK(d[l] >= lo && d[l] <= half, "x %016llx level %d digit %lld outside [%lld, %lld]",
                  (unsigned long long)x, l + 1, (long long)d[l], (long long)lo, (long long)half);
            rec += (uint64_t)d[l] << (64 - base_log * (l + 1));
        }
        const int nrb = 64 - base_log * levels;
        const uint64_t closest = ((x >> (nrb - 1)) + 1) >> 1 << nrb;  // round half up, mod 2^64
        CHECK(rec == closest, "x %016llx recomposes to %016llx, closest %016llx", (unsigned long long)x,
              (unsigned long long)rec, (unsigned long long)closest);
    };
    for (long t = 0; t < n_random; t++) check_x(rng());
    const uint64_t edges[] = {0, ~0ull, 1ull << 63, (1ull << 63) - 1, 1, 0x8000800080008000ull,
                              0x7fff7fff7fff7fffull, 0x8008008008008000ull, 0x7ff7ff7ff7ff8000ull};
    for (uint64_t e : edges)
        for (int sh = 0; sh < 64; sh++) {
            check_x(e ^ (1ull << sh));
            check_x(e + (1ull << sh));
            check_x(e - (1ull << sh));
        }

    // 2 and 3. every digit of every level's range
    uint64_t key[4];
    for (auto &k : key) k = rng();
    for (int l = 0; l < levels; l++) {
        const int64_t lo = l == 0 ? -half + 1 : -half;
        const int n = ks.nlimb[l];
        for (int64_t digit = lo; digit <= half; digit++) {
            const bool clamped = ks.clamp[l] && digit == half;
            CHECK(!ks.clamp[l] || l > 0, "2^%d: the top level is never clamped", base_log);
            const int64_t stored = clamped ? -half : digit;
            int64_t d = stored - ks.off[l], back = 0, scale = 1;
            uint64_t prod = (uint64_t)ks.off[l] * key[l] + (clamped ? key[l] << base_log : 0);
            for (int m = 0; m < n; m++) {
                const int64_t limb = tae::ksgemm::kl_next_limb(d, m == n - 1);
                CHECK(limb >= -128 && limb <= 127, "2^%d level %d digit %lld limb %d = %lld", base_log, l + 1,
                      (long long)digit, m, (long long)limb);
                back += limb * scale;
                scale *= 256;
                prod += (uint64_t)limb * (key[l] << (8 * m));
            }
            CHECK(back == stored - ks.off[l], "2^%d level %d digit %lld recombines to %lld", base_log, l + 1,
                  (long long)digit, (long long)(back + ks.off[l]));
            CHECK(prod == (uint64_t)digit * key[l], "2^%d level %d digit %lld: limb products != digit * key",
                  base_log, l + 1, (long long)digit);
        }
    }
    std::printf("2^%d x %d%s: S = %d, limbs/level", base_log, levels, clamp ? "" : " (no clamp)", ks.S);
    for (int l = 0; l < levels; l++)
        std::printf(" %d (c = %lld%s)", ks.nlimb[l], (long long)ks.off[l], ks.clamp[l] ? ", clamped" : "");
    std::printf("\n");
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 1000000;
    for (bool clamp : {true, false}) {
        run_shape(16, 2, n, clamp);
        run_shape(12, 3, n, clamp);
    }
    if (fails) {
        std::printf("%d failures\n", fails);
        return 1;
    }
    std::printf("OK\n");
    return 0;
}
