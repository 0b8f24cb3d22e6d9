// Host-side check of the integer-only torus helpers the blind-rotation kernels use
// (fft_device.hpp: from_torus_bits, decompose16) against the CPU oracle's restatement of tfhe-rs
// (or_from_torus, or_decompose), on random and edge-case inputs. Built and run by
// tests/test_native_helpers.py (CPU only).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../tfhe-aes-2_amd/csrc/fft_device.hpp"

extern "C" {
uint64_t or_from_torus(double x);
void or_decompose(uint64_t x, int base_log, int levels, int64_t *digits);
}

static int fails = 0;

static void check_ft(double x) {
    const uint64_t a = tae::from_torus_bits(x), b = or_from_torus(x);
    if (a != b && fails++ < 10) printf("from_torus(%a): got %016llx want %016llx\n", x, (unsigned long long)a, (unsigned long long)b);
    // the kernels' fast path: acc + from_torus(x) whenever it accepts x (and it must accept every
    // |x| in [2^-12, 2^52))
    const uint64_t acc0 = 0x0123456789abcdefull ^ (uint64_t)(int64_t)(x * 7);
    bool ok;
    const uint64_t acc = tae::torus_add_fast(x, acc0, ok);
    const double ax = std::fabs(x);
    if (ok ? acc != acc0 + b : (ax >= 0x1p-12 && ax < 0x1p52)) {
        if (fails++ < 10) printf("torus_add_fast(%a): ok %d got %016llx want %016llx\n", x, (int)ok,
                                 (unsigned long long)(acc - acc0), (unsigned long long)b);
    }
    // the fused transform's conversion of y = x 2^8 (lf512.hpp: the untwist's exact 2^-8 folded into the
    // exponent) equals the conversion of x whenever it accepts y
    {
        const double y = x * 0x1p8;
        bool ok8;
        const uint64_t a8 = tae::torus_add_fast_sh<8>(y, acc0, ok8);
        if ((ok8 != ok || (ok8 && a8 != acc)) && fails++ < 10)
            printf("torus_add_fast_sh<8>(%a): ok %d got %016llx want %016llx\n", y, (int)ok8,
                   (unsigned long long)(a8 - acc0), (unsigned long long)b);
    }
    // ... and of y = x 2^9 (lf1k.hpp, N = 1024)
    {
        const double y = x * 0x1p9;
        bool ok9;
        const uint64_t a9 = tae::torus_add_fast_sh<9>(y, acc0, ok9);
        if ((ok9 != ok || (ok9 && a9 != acc)) && fails++ < 10)
            printf("torus_add_fast_sh<9>(%a): ok %d got %016llx want %016llx\n", y, (int)ok9,
                   (unsigned long long)(a9 - acc0), (unsigned long long)b);
    }
    // the kernels' fallback undoes the fast value (linear in acc) and adds the exact one
    bool d;
    if (acc - tae::torus_add_fast(x, 0, d) + b != acc0 + b && fails++ < 10)
        printf("torus_add_fast(%a) is not linear in acc\n", x);
}

template <int LEV, int B>
static void check_dect(uint64_t x) {
    uint32_t d[LEV];
    int64_t r[LEV];
    tae::decompose16t<LEV, B>(x, d);
    or_decompose(x, B, LEV, r);
    for (int l = 0; l < LEV; l++) {
        const int64_t got = (int16_t)(d[l] & 0xFFFF);
        if ((got != r[l] || (d[l] >> 16) != 0) && fails++ < 10)
            printf("decompose16t(%016llx, B=%d, L=%d) level %d: got %lld want %lld\n", (unsigned long long)x, B, LEV,
                   l + 1, (long long)got, (long long)r[l]);
    }
}

template <int LEV>
static void check_dec(uint64_t x, int B) {
    uint32_t d[LEV];
    int64_t r[LEV];
    tae::decompose16<LEV>(x, B, d);
    or_decompose(x, B, LEV, r);
    for (int l = 0; l < LEV; l++) {
        const int64_t got = (int16_t)(d[l] & 0xFFFF);
        if ((got != r[l] || (d[l] >> 16) != 0) && fails++ < 10)
            printf("decompose(%016llx, B=%d, L=%d) level %d: got %lld want %lld\n", (unsigned long long)x, B, LEV, l + 1,
                   (long long)got, (long long)r[l]);
    }
}

// level-by-level digit chain == the oracle's digits, finest level first
template <int LEV, int B>
static void check_chain(uint64_t x) {
    int64_t r[LEV];
    or_decompose(x, B, LEV, r);
    uint32_t st;
    int32_t got = tae::digit_first<LEV, B>(x, st);
    for (int l = LEV - 1; l >= 0; l--) {
        if (l < LEV - 1) got = tae::digit_next<B>(st);
        if (got != r[l] && fails++ < 10)
            printf("digit chain(%016llx, B=%d, L=%d) level %d: got %d want %lld\n", (unsigned long long)x, B, LEV, l + 1,
                   got, (long long)r[l]);
    }
}

// packed two-coefficient decomposition == decompose16 on each half
template <int LEV, int B>
static void check_decp(uint64_t x0, uint64_t x1) {
    uint32_t d[LEV], a[LEV], b[LEV];
    tae::decompose16p<LEV, B>(x0, x1, d);
    tae::decompose16t<LEV, B>(x0, a);
    tae::decompose16t<LEV, B>(x1, b);
    for (int l = 0; l < LEV; l++)
        if (d[l] != (a[l] | (b[l] << 16)) && fails++ < 10)
            printf("decompose16p(%016llx, %016llx, B=%d, L=%d) level %d: got %08x want %08x\n", (unsigned long long)x0,
                   (unsigned long long)x1, B, LEV, l + 1, d[l], a[l] | (b[l] << 16));
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    std::mt19937_64 rng(12345);
    // from_torus: magnitudes across every exponent that matters, exact halves, integers, zeros
    const double specials[] = {0.0, -0.0, 0.5, -0.5, 1.5, -1.5, 2.5, -2.5, 1.0, -1.0, 0x1p-64, -0x1p-64, 0x1p-65,
                               -0x1p-65, 0x1.8p-65, -0x1.8p-65, 0x1p-66, 0x1p52, -0x1p52, 0x1p53 + 2, 0x1p70, -0x1p70,
                               0x1p-1022, 0x1p-1074, 1e300, -1e300, 0.25, -0.25, 0x1.fffffffffffffp-2, -0x1.fffffffffffffp-2,
                               0x1p-12, -0x1p-12, 0x1.fffffffffffffp-13, -0x1.fffffffffffffp-13, 0x1.fffffffffffffp51,
                               -0x1.fffffffffffffp51, 0x1p51 + 0.5, -(0x1p51 + 0.5), -(0x1p40 + 0.5), -0.5 - 0x1p30,
                               -0x1p-64, 0x1.8p-12, -0x1.8p-12, 1.0 / 3.0, -1.0 / 3.0};
    for (double x : specials) check_ft(x);
    for (long i = 0; i < n; i++) {
        const uint64_t r = rng();
        const int ex = (int)(r % 100) - 75;  // |x| in [2^-75, 2^25)
        double x = std::ldexp((double)(rng() >> 11) * 0x1p-53, ex);
        if (r & (1ull << 40)) x = -x;
        check_ft(x);
        // exact halves at random integers and tiny values with ties below 2^-64
        if ((i & 15) == 0) {
            const double h = (double)(int64_t)(rng() % 100000) + 0.5;
            check_ft(h);
            check_ft(-h);
            const double t = std::ldexp((double)(2 * (rng() % 1000) + 1), -65 - (int)(rng() % 4));
            check_ft(t);
            check_ft(-t);
        }
    }
    // decompositions used by the kernels: PBS (B=12, L=3), CBS / VP (B=13, L=1), 8-bit set (B=7, L=6),
    // (B=6, L=4), plus edges around the rounding point and the top of the range
    const uint64_t edges[] = {0, 1, ~0ull, 1ull << 63, (1ull << 63) - 1, (1ull << 27), (1ull << 27) - 1, (1ull << 28) - 1,
                              0xFFFFFFFFF8000000ull, 0xFFFFFFFFF7FFFFFFull, 0x8008008000000000ull, 0x7FF7FF8000000000ull};
    for (uint64_t x : edges) {
        check_dec<3>(x, 12);
        check_dec<1>(x, 13);
        check_dec<6>(x, 5);
        check_dec<4>(x, 6);
        check_dec<2>(x, 15);
        check_dect<6, 7>(x);
        check_dect<4, 6>(x);
        check_dect<3, 12>(x);
        check_dect<4, 9>(x);
        check_chain<3, 12>(x);
        check_chain<1, 13>(x);
        check_chain<4, 6>(x);
        check_chain<2, 15>(x);
    }
    for (long i = 0; i < n; i++) {
        uint64_t x = rng();
        if (i & 1) x = (x & ~((1ull << 40) - 1)) | ((uint64_t)(rng() % 5) << 26);  // near-tie digits
        if ((i & 7) == 0) x = (x & 0xFFFFFFF000000000ull) | (0x800800800ull << 28 >> 28 << 28);
        check_dec<3>(x, 12);
        check_dec<1>(x, 13);
        check_dec<6>(x, 5);
        check_dec<4>(x, 6);
        check_dec<2>(x, 15);
        check_dect<6, 7>(x);
        check_dect<4, 6>(x);
        check_dect<3, 12>(x);
        check_dect<4, 9>(x);
        check_chain<3, 12>(x);
        check_chain<1, 13>(x);
        check_chain<4, 6>(x);
        check_chain<2, 15>(x);
        check_chain<3, 9>(x);
        const uint64_t y = (i & 2) ? rng() : (x ^ (rng() & 0xFFFFFFFull));
        check_decp<3, 12>(x, y);
        check_decp<1, 13>(x, y);
        check_decp<6, 7>(x, y);
        check_decp<4, 6>(x, y);
        check_decp<4, 9>(x, y);
        check_decp<2, 15>(x, y);
    }
    for (uint64_t x : edges)
        for (uint64_t y : edges) {
            check_decp<3, 12>(x, y);
            check_decp<1, 13>(x, y);
            check_decp<6, 7>(x, y);
        }
    printf("%s (%d mismatches)\n", fails ? "FAIL" : "OK", fails);
    return fails ? 1 : 0;
}
