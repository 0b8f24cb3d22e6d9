/*
 * tfhe_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker; see tfhe_oracle.h for the contract).
 *
 * A plain-C restatement of the reference's shortint_woppbs_1bit hot path and of the tfhe-rs
 * 0.11.2 routines it calls.  Reference citations are given per function.  Compiled with
 * -ffp-contract=off: every fused multiply-add below is an explicit fma() so that the f64 FFT
 * arithmetic is a fixed sequence of IEEE operations (the product's HIP kernels execute the same
 * sequence, which is what makes the GPU-vs-oracle comparison bit-exact).
 */
#include "tfhe_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_PI 3.14159265358979323846

/* ======================================================================================
 * Parameters: src/tfhe/shortint_woppbs_1bit/parameters.rs:29-205
 * ====================================================================================== */
int or_params_get(int id, or_params *o) {
    memset(o, 0, sizeof(*o));
    switch (id) {
    case 0: /* params_sqrd_lvl_1, parameters.rs:29-61 */
        *o = (or_params){671, 2, 1024, 2, 15, 4, 3, 1, 10, 1, 24,
                         4.7280002450549286e-05, 3.162026630747649e-16, 3.162026630747649e-16, 1};
        return 0;
    case 1: /* params_sqrd_lvl_4, parameters.rs:77-109 */
        *o = (or_params){679, 2, 1024, 2, 15, 4, 3, 1, 11, 2, 16,
                         4.7280002450549286e-05, 3.162026630747649e-16, 3.162026630747649e-16, 4};
        return 0;
    case 2: /* params_sqrd_lvl_64, parameters.rs:125-157 (default, main.rs:82-83) */
        *o = (or_params){677, 4, 512, 3, 12, 4, 3, 1, 13, 2, 16,
                         4.7280002450549286e-05, 0.00000000000000022148688116005568,
                         0.00000000000000022148688116005568, 64};
        return 0;
    case 3: /* params_sqrd_lvl_256, parameters.rs:173-205 */
        *o = (or_params){665, 2, 1024, 4, 9, 6, 2, 1, 14, 3, 12,
                         4.7280002450549286e-05, 3.162026630747649e-16, 3.162026630747649e-16, 256};
        return 0;
    case 4: /* shortint_woppbs_8bit params(), shortint_woppbs_8bit.rs:39-86; max_noise_sq holds the
             * shortint MaxNoiseLevel (11, additive levels), not a squared level */
        *o = (or_params){785, 2, 1024, 6, 7, 8, 2, 4, 6, 3, 12,
                         1.5140301927925663e-05, 0.00000000000000022148688116005568,
                         0.00000000000000022148688116005568, 11};
        return 0;
    case 5: /* shortint_1bit PARAMS, src/tfhe/shortint_1bit.rs:62-83 (ClassicPBSParameters "testing
             * parameters"; message modulus 2, carry 1, MaxNoiseLevel 11, EncryptionKeyChoice::Small).
             * The packing keyswitch key of generate_keys_with_params (:186-196) uses ks_base_log /
             * ks_level and the lwe noise: stored as (pfks_l, pfks_b, pfks_std). No CBS. */
        *o = (or_params){640, 4, 512, 7, 6, 2, 6, 0, 0, 2, 6,
                         4.728000245054929e-7, 2.845267479601915e-15, 4.728000245054929e-7, 11, 2};
        return 0;
    default:
        return -1;
    }
}

/* ======================================================================================
 * ChaCha20 (DJB variant, 64-bit counter + 64-bit nonce, as rand_chacha::ChaCha20Rng) -- the
 * reference's test seed generator (test_helper.rs:101-106) and our keygen randomness spec.
 * ====================================================================================== */
#define ROTL32(v, c) (((v) << (c)) | ((v) >> (32 - (c))))
#define QR(a, b, c, d)                                                                             \
    a += b; d ^= a; d = ROTL32(d, 16);                                                             \
    c += d; b ^= c; b = ROTL32(b, 12);                                                             \
    a += b; d ^= a; d = ROTL32(d, 8);                                                              \
    c += d; b ^= c; b = ROTL32(b, 7);

static uint32_t le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

void or_chacha20_block(const uint8_t key[32], uint64_t nonce, uint64_t counter, uint8_t out[64]) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865; s[1] = 0x3320646e; s[2] = 0x79622d32; s[3] = 0x6b206574;
    for (int i = 0; i < 8; i++) s[4 + i] = le32(key + 4 * i);
    s[12] = (uint32_t)counter; s[13] = (uint32_t)(counter >> 32);
    s[14] = (uint32_t)nonce; s[15] = (uint32_t)(nonce >> 32);
    memcpy(x, s, sizeof(s));
    for (int i = 0; i < 10; i++) {
        QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; i++) {
        uint32_t v = x[i] + s[i];
        out[4 * i] = (uint8_t)v; out[4 * i + 1] = (uint8_t)(v >> 8);
        out[4 * i + 2] = (uint8_t)(v >> 16); out[4 * i + 3] = (uint8_t)(v >> 24);
    }
}

void or_chacha20_stream(const uint8_t key[32], uint64_t nonce, uint64_t counter, uint8_t *out,
                        size_t len) {
    uint8_t blk[64];
    while (len) {
        or_chacha20_block(key, nonce, counter++, blk);
        size_t t = len < 64 ? len : 64;
        memcpy(out, blk, t);
        out += t;
        len -= t;
    }
}

typedef struct {
    uint8_t key[32];
    uint64_t nonce, ctr;
    uint8_t buf[64];
    int pos;
} rng_t;

static void rng_init(rng_t *r, const uint8_t key[32], uint64_t nonce, uint64_t ctr) {
    memcpy(r->key, key, 32);
    r->nonce = nonce;
    r->ctr = ctr;
    r->pos = 64;
}
static uint64_t rng_u64(rng_t *r) {
    if (r->pos == 64) {
        or_chacha20_block(r->key, r->nonce, r->ctr++, r->buf);
        r->pos = 0;
    }
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)r->buf[r->pos + i] << (8 * i);
    r->pos += 8;
    return v;
}
/* Box-Muller, one sample per two words; error = rint(z * sigma * 2^64) as a torus element */
static uint64_t rng_gauss_torus(rng_t *r, double sigma) {
    uint64_t w1 = rng_u64(r), w2 = rng_u64(r);
    double u1 = (double)((w1 >> 11) + 1) * 0x1p-53; /* (0, 1] */
    double u2 = (double)(w2 >> 11) * 0x1p-53;       /* [0, 1) */
    double rad = sqrt(-2.0 * log(u1));
    double z = rad * cos(2.0 * ORACLE_PI * u2);
    double v = rint(z * (sigma * 0x1p64));
    return (uint64_t)(int64_t)v;
}

/* keygen stream purposes (spec shared with the product client) */
enum { P_LWE_SK = 1, P_GLWE_SK = 2, P_KSK = 3, P_BSK = 4, P_PFPKSK = 5, P_ENCRYPT = 6, P_ENCRYPT_INT = 7 };
#define CT_STRIDE (1ull << 24)

/* ======================================================================================
 * Torus helpers -- tfhe-rs core_crypto::commons::math::decomposition (SignedDecomposer)
 * ====================================================================================== */
uint64_t or_closest_representable(uint64_t x, int base_log, int levels) {
    /* SignedDecomposer::closest_representable: round to the nearest multiple of 2^(64-B*L) */
    int nrb = 64 - base_log * levels;
    if (nrb <= 0) return x;
    uint64_t res = x >> (nrb - 1);
    res += res & 1;
    res >>= 1;
    return nrb == 64 ? 0 : res << nrb;
}

/* decompose_one_level + SignedDecompositionIter: balanced digits, least significant first */
void or_decompose(uint64_t x, int base_log, int levels, int64_t *digits) {
    uint64_t r = or_closest_representable(x, base_log, levels);
    int nrb = 64 - base_log * levels;
    uint64_t state = nrb >= 64 ? 0 : r >> nrb;
    uint64_t mask = (base_log == 64) ? ~0ull : ((1ull << base_log) - 1);
    for (int lev = levels; lev >= 1; lev--) {
        uint64_t res = state & mask;
        state >>= base_log;
        uint64_t carry = ((res - 1) | state) & res;
        carry >>= (base_log - 1);
        state += carry;
        digits[lev - 1] = (int64_t)(res - (carry << base_log));
    }
}

/* tfhe-rs UnsignedTorus::from_torus (f64 round = half away from zero, i64 saturation) */
uint64_t or_from_torus(double x) {
    double f = x - round(x);
    double v = round(f * 0x1p64);
    int64_t iv;
    if (v >= 0x1p63)
        iv = INT64_MAX;
    else
        iv = (int64_t)v;
    return (uint64_t)iv;
}

/* fft64::crypto::bootstrap pbs_modulus_switch with offset 0, lut_count_log 0 -> [0, 2N] */
uint64_t or_pbs_modulus_switch(uint64_t x, int N) {
    int logN = 0;
    while ((1 << logN) < N) logN++;
    uint64_t out = x >> (64 - logN - 2);
    out += out & 1;
    out >>= 1;
    return out;
}

/* polynomial_wrapping_monic_monomial_mul (degree may be any value, taken mod 2N) */
void or_monomial_mul(const uint64_t *in, uint64_t *out, int N, int64_t degree) {
    int64_t d = degree % (2 * N);
    if (d < 0) d += 2 * N;
    for (int j = 0; j < N; j++) {
        int64_t src = j - d; /* in (-2N, N) */
        int neg = 0;
        while (src < 0) {
            src += N;
            neg ^= 1;
        }
        out[j] = neg ? (0 - in[src]) : in[src];
    }
}

/* exact negacyclic product a (torus) * b (integer) mod (X^N + 1, 2^64) */
void or_negacyclic_mul_exact(const uint64_t *a, const int64_t *b, uint64_t *out, int N) {
    for (int i = 0; i < N; i++) out[i] = 0;
    for (int i = 0; i < N; i++) {
        if (!b[i]) continue;
        uint64_t bi = (uint64_t)b[i];
        for (int j = 0; j < N; j++) {
            uint64_t prod = a[j] * bi;
            int t = i + j;
            if (t < N)
                out[t] += prod;
            else
                out[t - N] -= prod;
        }
    }
}

/* shortint_woppbs_1bit.rs:125-132 */
uint64_t or_encode_bit(uint64_t bit) { return bit << 63; }
uint64_t or_decode_bit(uint64_t x) { return ((x + (1ull << 62)) & (1ull << 63)) >> 63; }

/* ======================================================================================
 * Negacyclic f64 FFT (tfhe-fft 0.7 math: fold p[j] + i*p[j+M], twist by e^{i*pi*j/N},
 * M = N/2 point complex DFT; torus inputs normalised by 2^-64; backward untwists with
 * conj(twist)/M and takes the fractional part).  The DFT itself is a fixed DIF radix-R
 * schedule (R=16 for M=256, R=8 for M=512, R=16x... see fft_plan) whose output lives in
 * digit-reversed order; the inverse is the mirrored DIT schedule.  Pointwise products are
 * order-agnostic, so the Fourier layout never needs un-permuting.
 * ====================================================================================== */
struct or_fft {
    int N, M, R, P;
    or_c64 *twist;   /* [M] (cos(pi j/N), sin(pi j/N)) */
    or_c64 *untwist; /* [M] (cos/M, -sin/M) */
    or_c64 *w;       /* [M] W_M^e = (cos(2 pi e/M), -sin(2 pi e/M)) */
};

/* cos/sin(2*pi*num/den) with exact quadrant/octant symmetry (shared spec with the product) */
static void sincos2pi(long num, long den, double *c, double *s) {
    num %= den;
    if (num < 0) num += den;
    long q = (4 * num) / den;
    long r = 4 * num - q * den; /* angle = q*pi/2 + (pi/2) * r/den, r in [0, den) */
    double c0, s0;
    if (2 * r <= den) {
        double a = (ORACLE_PI * (double)r) / (2.0 * (double)den);
        c0 = cos(a);
        s0 = sin(a);
    } else {
        double a = (ORACLE_PI * (double)(den - r)) / (2.0 * (double)den);
        c0 = sin(a);
        s0 = cos(a);
    }
    switch (q) {
    case 0: *c = c0; *s = s0; break;
    case 1: *c = -s0; *s = c0; break;
    case 2: *c = -c0; *s = -s0; break;
    default: *c = s0; *s = -c0; break;
    }
}

or_fft *or_fft_new(int N) {
    or_fft *f = (or_fft *)calloc(1, sizeof(or_fft));
    f->N = N;
    f->M = N / 2;
    if (f->M == 256) {
        f->R = 16; f->P = 2;
    } else if (f->M == 512) {
        f->R = 8; f->P = 3;
    } else if (f->M == 64) {
        f->R = 8; f->P = 2;
    } else if (f->M == 16) {
        f->R = 16; f->P = 1;
    } else if (f->M == 8) {
        f->R = 8; f->P = 1;
    } else {
        free(f);
        return NULL;
    }
    int M = f->M;
    f->twist = (or_c64 *)malloc(sizeof(or_c64) * M);
    f->untwist = (or_c64 *)malloc(sizeof(or_c64) * M);
    f->w = (or_c64 *)malloc(sizeof(or_c64) * M);
    for (int j = 0; j < M; j++) {
        double c, s;
        sincos2pi(j, 2L * N, &c, &s);
        f->twist[j].re = c;
        f->twist[j].im = s;
        f->untwist[j].re = c / (double)M;
        f->untwist[j].im = -s / (double)M;
        sincos2pi(j, M, &c, &s);
        f->w[j].re = c;
        f->w[j].im = -s;
    }
    return f;
}

void or_fft_free(or_fft *f) {
    if (!f) return;
    free(f->twist);
    free(f->untwist);
    free(f->w);
    free(f);
}

static inline or_c64 cmul(or_c64 a, or_c64 b) {
    or_c64 r;
    r.re = fma(a.re, b.re, -(a.im * b.im));
    r.im = fma(a.re, b.im, a.im * b.re);
    return r;
}
static inline or_c64 cconj(or_c64 a) {
    a.im = -a.im;
    return a;
}
static inline or_c64 cadd(or_c64 a, or_c64 b) { return (or_c64){a.re + b.re, a.im + b.im}; }
static inline or_c64 csub(or_c64 a, or_c64 b) { return (or_c64){a.re - b.re, a.im - b.im}; }

/* radix-4 DFT, natural in/out order; inv selects W4 = +i */
static inline void dft4(or_c64 *v, int s0, int st, int inv) {
    or_c64 a = v[s0], b = v[s0 + st], c = v[s0 + 2 * st], d = v[s0 + 3 * st];
    or_c64 t0 = cadd(a, c), t1 = csub(a, c), t2 = cadd(b, d), t3 = csub(b, d);
    v[s0] = cadd(t0, t2);
    v[s0 + 2 * st] = csub(t0, t2);
    if (!inv) {
        v[s0 + st] = (or_c64){t1.re + t3.im, t1.im - t3.re};
        v[s0 + 3 * st] = (or_c64){t1.re - t3.im, t1.im + t3.re};
    } else {
        v[s0 + st] = (or_c64){t1.re - t3.im, t1.im + t3.re};
        v[s0 + 3 * st] = (or_c64){t1.re + t3.im, t1.im - t3.re};
    }
}

/* multiply by W_R^e (table-driven; e == R/4 is the exact -i (fwd) / +i (inv)) */
static inline or_c64 tw_small(const or_fft *f, or_c64 x, int e, int R, int inv) {
    if (e == 0) return x;
    if (4 * e == R) return inv ? (or_c64){-x.im, x.re} : (or_c64){x.im, -x.re};
    or_c64 w = f->w[e * (f->M / R)];
    return cmul(x, inv ? cconj(w) : w);
}

/* DFT16 = 4x4: x[n1 + 4 n2] -> X[k1 + 4 k2]; DFT8 = 2x4: x[n1 + 2 n2] -> X[k1 + 4 k2] */
static void dftR(const or_fft *f, or_c64 *v, int R, int inv) {
    if (R == 16) {
        or_c64 y[16];
        for (int n1 = 0; n1 < 4; n1++) dft4(v, n1, 4, inv); /* over n2: v[n1 + 4 k1] */
        for (int n1 = 0; n1 < 4; n1++)
            for (int k1 = 0; k1 < 4; k1++) y[4 * k1 + n1] = tw_small(f, v[n1 + 4 * k1], n1 * k1, 16, inv);
        for (int k1 = 0; k1 < 4; k1++) dft4(y, 4 * k1, 1, inv); /* over n1: y[4 k1 + k2] */
        for (int k1 = 0; k1 < 4; k1++)
            for (int k2 = 0; k2 < 4; k2++) v[k1 + 4 * k2] = y[4 * k1 + k2];
    } else if (R == 8) {
        or_c64 y[8];
        for (int n1 = 0; n1 < 2; n1++) dft4(v, n1, 2, inv); /* v[n1 + 2 k1] */
        for (int n1 = 0; n1 < 2; n1++)
            for (int k1 = 0; k1 < 4; k1++) y[2 * k1 + n1] = tw_small(f, v[n1 + 2 * k1], n1 * k1, 8, inv);
        for (int k1 = 0; k1 < 4; k1++) {
            or_c64 a = y[2 * k1], b = y[2 * k1 + 1];
            v[k1] = cadd(a, b);
            v[k1 + 4] = csub(a, b);
        }
    } else {
        abort();
    }
}

void or_fft_raw_fwd(const or_fft *f, or_c64 *z) {
    int M = f->M, R = f->R;
    int L = M / R;
    or_c64 v[16];
    for (int s = 0; s < f->P; s++) {
        int groups = M / (R * L);
        for (int g = 0; g < groups; g++)
            for (int u = 0; u < L; u++) {
                int base = g * R * L + u;
                for (int m = 0; m < R; m++) v[m] = z[base + m * L];
                dftR(f, v, R, 0);
                for (int k = 0; k < R; k++) {
                    int e = u * k * (M / (R * L));
                    z[base + k * L] = e ? cmul(v[k], f->w[e]) : v[k];
                }
            }
        L /= R;
    }
}

void or_fft_raw_inv(const or_fft *f, or_c64 *z) {
    int M = f->M, R = f->R;
    int L = 1;
    or_c64 v[16];
    for (int s = f->P - 1; s >= 0; s--) {
        int groups = M / (R * L);
        for (int g = 0; g < groups; g++)
            for (int u = 0; u < L; u++) {
                int base = g * R * L + u;
                for (int k = 0; k < R; k++) {
                    int e = u * k * (M / (R * L));
                    v[k] = e ? cmul(z[base + k * L], cconj(f->w[e])) : z[base + k * L];
                }
                dftR(f, v, R, 1);
                for (int m = 0; m < R; m++) z[base + m * L] = v[m];
            }
        L *= R;
    }
}

/* FftView::forward_as_integer (digits as i64 -> f64) */
void or_fft_fwd_int(const or_fft *f, const int64_t *poly, or_c64 *out) {
    int M = f->M;
    for (int j = 0; j < M; j++) {
        double re = (double)poly[j], im = (double)poly[j + M];
        or_c64 t = f->twist[j];
        out[j].re = fma(re, t.re, -(im * t.im));
        out[j].im = fma(re, t.im, im * t.re);
    }
    or_fft_raw_fwd(f, out);
}

/* FftView::forward_as_torus (u64 -> i64 -> f64 * 2^-64) */
void or_fft_fwd_torus(const or_fft *f, const uint64_t *poly, or_c64 *out) {
    int M = f->M;
    for (int j = 0; j < M; j++) {
        double re = (double)(int64_t)poly[j] * 0x1p-64, im = (double)(int64_t)poly[j + M] * 0x1p-64;
        or_c64 t = f->twist[j];
        out[j].re = fma(re, t.re, -(im * t.im));
        out[j].im = fma(re, t.im, im * t.re);
    }
    or_fft_raw_fwd(f, out);
}

/* FftView::add_backward_as_torus */
void or_fft_add_bwd_torus(const or_fft *f, const or_c64 *in, uint64_t *out) {
    int M = f->M;
    or_c64 *z = (or_c64 *)malloc(sizeof(or_c64) * M);
    memcpy(z, in, sizeof(or_c64) * M);
    or_fft_raw_inv(f, z);
    for (int j = 0; j < M; j++) {
        or_c64 t = cmul(z[j], f->untwist[j]);
        out[j] += or_from_torus(t.re);
        out[j + M] += or_from_torus(t.im);
    }
    free(z);
}

/* ======================================================================================
 * The blind rotation's transform for N = 512 (params_sqrd_lvl_64: every CMux of the PBS; the
 * product's br512x4 / br512lat, DESIGN.md §5.1 "fused-twiddle transform").  The same negacyclic
 * DFT as or_fft_fwd_int / or_fft_add_bwd_torus (16 x 16 DIF, positions 16 kappa + lambda), with the
 * arithmetic rearranged so that no twiddle is a separate complex product:
 *  - a radix-4 stage whose 4 inputs carry unit factors w, w g, w g^2, w g^3 is evaluated relative to w
 *    with "fused" butterflies: x + g^2 y = x + c (y + i t y) for g^2 = c (1 + i t) (Linzer-Feig), i.e.
 *    24 fma per DFT4 instead of 3-4 complex products + 16 adds; the factor w travels to the next stage;
 *  - the twist of the forward transform splits into lane-uniform parts (psi^64 inside the first DFT4,
 *    whose e^{i pi/4} products act on the integer digits exactly) and factors that merge into the
 *    following stages' ratios; the forward output is the exact DFT (no leftover factor);
 *  - the inverse transform's input may carry any unit factor per position E2(pos) = psi^(kappa + (lambda
 *    mod 4)): it is divided out of the Fourier BSK once (lf_rescale_bsk), and it keeps every fused ratio
 *    off the imaginary axis (a ratio of exactly +-i has no cos-tan form).
 * Every per-lane constant is (cos, tan) of an angle 2 pi num / 1024 from sincos2pi.  The lane programs
 * below are the GPU's: lane (u, r) of pass A holds points j = u + 16 r + 64 i, lane (kappa, r) of pass B
 * positions 16 kappa + r + 4 i; the transposes between the two radix-4 stages of a pass move register
 * k of lane row r to register r of lane row k.  Bit-exact with tfhe-rs is not a goal of this transform
 * (its FFT is not pinned either); it is pinned to the exact negacyclic product numerically
 * (tests/test_oracle.py) and to the GPU bit for bit.
 * ====================================================================================== */
typedef struct {
    double c2, t2, c1, t1; /* (cos, tan) of g^2 and of g */
} lf4;
typedef struct {
    int N;        /* 512 (the plans share this tag: ext_product_add dispatches on it) */
    lf4 fa2[4];   /* forward pass A, stage 2, lane row k1: g = psi^16 W16^k1          (num 16 - 64 k1) */
    lf4 fb1[16];  /* forward pass B, stage 1, lane column kappa: g = psi^4 W_M^4kappa (num 4 - 16 kappa) */
    lf4 fb2[64];  /* forward pass B, stage 2, lane (kappa, l1): g = psi W_M^kappa W16^l1 */
    lf4 ib2[4];   /* inverse pass B, stage 2, lane row u1: g = psi W16^-u1            (num 1 + 64 u1) */
    lf4 ia1[16];  /* inverse pass A, stage 1, lane column u: g = psi^4 W_M^-4u        (num 4 + 16 u) */
    lf4 ia2[64];  /* inverse pass A, stage 2, lane (u, m1): g = psi W_M^-u W16^-m1   (num 1 + 4u + 64 m1) */
    double s2, c8, t8; /* 1/sqrt(2); cos, tan of pi/8 (psi^64) */
    or_c64 untw[256];  /* conj(twist[j]); the backward 2^-8 is exact and applied to the sum */
    or_c64 e2[256];    /* conj(E2(pos)): the Fourier BSK rescale */
} lf_plan;

static void lf_ct(long num, double *c, double *t) {
    double s;
    sincos2pi(num, 1024, c, &s);
    *t = s / *c;
}
static void lf_make(long num, lf4 *o) {
    lf_ct(2 * num, &o->c2, &o->t2);
    lf_ct(num, &o->c1, &o->t1);
}

static void or_lf_plan_build(lf_plan *P) {
    P->N = 512;
    for (int k = 0; k < 4; k++) {
        lf_make(16 - 64 * k, &P->fa2[k]);
        lf_make(1 + 64 * k, &P->ib2[k]);
    }
    for (int a = 0; a < 16; a++) {
        lf_make(4 - 16 * a, &P->fb1[a]);
        lf_make(4 + 16 * a, &P->ia1[a]);
        for (int l = 0; l < 4; l++) {
            lf_make(1 - 4 * a - 64 * l, &P->fb2[4 * a + l]);
            lf_make(1 + 4 * a + 64 * l, &P->ia2[4 * a + l]);
        }
    }
    double c, s;
    P->s2 = 1.0 / sqrt(2.0);
    lf_ct(64, &P->c8, &P->t8);
    for (int j = 0; j < 256; j++) {
        sincos2pi(j, 1024, &c, &s);
        P->untw[j].re = c;
        P->untw[j].im = -s;
        sincos2pi(-((j >> 4) + (j & 3)), 1024, &c, &s);
        P->e2[j].re = c;
        P->e2[j].im = s;
    }
}

/* x -> x (1 + i t) */
static inline or_c64 lf_rot(or_c64 x, double t) { return (or_c64){fma(-t, x.im, x.re), fma(t, x.re, x.im)}; }
static inline or_c64 lf_add(or_c64 a, double c, or_c64 t) { return (or_c64){fma(c, t.re, a.re), fma(c, t.im, a.im)}; }

/* DFT4 (W4 = -i forward, +i inverse) of x0, g x1, g^2 x2, g^3 x3, relative to x0's factor */
static void lf_dft4(const or_c64 *x, const lf4 *K, int inv, or_c64 *y) {
    or_c64 t = lf_rot(x[2], K->t2), s = lf_rot(x[3], K->t2);
    or_c64 u0 = lf_add(x[0], K->c2, t), u1 = lf_add(x[0], -K->c2, t);
    or_c64 v0 = lf_add(x[1], K->c2, s), v1 = lf_add(x[1], -K->c2, s);
    or_c64 p = lf_rot(v0, K->t1), q = lf_rot(v1, K->t1);
    y[0] = lf_add(u0, K->c1, p);
    y[2] = lf_add(u0, -K->c1, p);
    /* u1 -/+ i c1 q: (u1.re +/- c1 q.im, u1.im -/+ c1 q.re) */
    double c = inv ? -K->c1 : K->c1;
    y[1] = (or_c64){fma(c, q.im, u1.re), fma(-c, q.re, u1.im)};
    y[3] = (or_c64){fma(-c, q.im, u1.re), fma(c, q.re, u1.im)};
}

/* DFT4 over i of the integer pairs d_i = d[i][0] + i d[i][1] times (e^{i pi/8})^i: the e^{i pi/4} products of
 * the first stage act on the integers exactly ((re - im, re + im) / sqrt 2), the second stage is fused */
static void lf_int_dft4(const int64_t d[4][2], double s2, double c8, double t8, or_c64 *q) {
    double d0r = (double)d[0][0], d0i = (double)d[0][1], d1r = (double)d[1][0], d1i = (double)d[1][1];
    double p2r = (double)(d[2][0] - d[2][1]), p2i = (double)(d[2][0] + d[2][1]);
    double p3r = (double)(d[3][0] - d[3][1]), p3i = (double)(d[3][0] + d[3][1]);
    or_c64 Ep = {fma(s2, p2r, d0r), fma(s2, p2i, d0i)}, Em = {fma(-s2, p2r, d0r), fma(-s2, p2i, d0i)};
    or_c64 Op = {fma(s2, p3r, d1r), fma(s2, p3i, d1i)}, Om = {fma(-s2, p3r, d1r), fma(-s2, p3i, d1i)};
    or_c64 a = lf_rot(Op, t8), b = lf_rot(Om, t8);
    q[0] = lf_add(Ep, c8, a);
    q[2] = lf_add(Ep, -c8, a);
    q[1] = (or_c64){fma(c8, b.im, Em.re), fma(-c8, b.re, Em.im)};
    q[3] = (or_c64){fma(-c8, b.im, Em.re), fma(c8, b.re, Em.im)};
}

/* forward transform of one digit polynomial (N = 512 integers) into X[16 kappa + lambda] */
void or_lf_fwd(const void *plan, const int64_t *poly, or_c64 *X) {
    const lf_plan *P = (const lf_plan *)plan;
    or_c64 Q[16][4][4]; /* [u][r][k1] */
    or_c64 z[256];
    for (int u = 0; u < 16; u++)
        for (int r = 0; r < 4; r++) {
            int64_t d[4][2];
            for (int i = 0; i < 4; i++) {
                int j = u + 16 * r + 64 * i;
                d[i][0] = poly[j];
                d[i][1] = poly[j + 256];
            }
            lf_int_dft4(d, P->s2, P->c8, P->t8, Q[u][r]);
        }
    for (int u = 0; u < 16; u++)
        for (int k1 = 0; k1 < 4; k1++) {
            or_c64 x[4], y[4];
            for (int r = 0; r < 4; r++) x[r] = Q[u][r][k1];
            lf_dft4(x, &P->fa2[k1], 0, y);
            for (int k2 = 0; k2 < 4; k2++) z[u + 16 * (k1 + 4 * k2)] = y[k2];
        }
    or_c64 R[16][4][4]; /* [kappa][r][l1] */
    for (int a = 0; a < 16; a++)
        for (int r = 0; r < 4; r++) {
            or_c64 x[4];
            for (int i = 0; i < 4; i++) x[i] = z[(r + 4 * i) + 16 * a];
            lf_dft4(x, &P->fb1[a], 0, R[a][r]);
        }
    for (int a = 0; a < 16; a++)
        for (int l1 = 0; l1 < 4; l1++) {
            or_c64 x[4], y[4];
            for (int r = 0; r < 4; r++) x[r] = R[a][r][l1];
            lf_dft4(x, &P->fb2[4 * a + l1], 0, y);
            for (int l2 = 0; l2 < 4; l2++) X[16 * a + l1 + 4 * l2] = y[l2];
        }
}

/* backward transform of Y[16 kappa + lambda] (which carries the factor E2) added to the torus
 * polynomial out (N = 512): untwist conj(twist), 2^-8 exact, from_torus */
void or_lf_bwd_add(const void *plan, const or_c64 *Y, uint64_t *out) {
    const lf_plan *P = (const lf_plan *)plan;
    or_c64 R[16][4][4]; /* [kappa][r][u1] */
    or_c64 z[256];
    for (int a = 0; a < 16; a++)
        for (int r = 0; r < 4; r++) {
            or_c64 v[4];
            for (int i = 0; i < 4; i++) v[i] = Y[16 * a + r + 4 * i];
            dft4(v, 0, 1, 1);
            for (int k = 0; k < 4; k++) R[a][r][k] = v[k];
        }
    for (int a = 0; a < 16; a++)
        for (int u1 = 0; u1 < 4; u1++) {
            or_c64 x[4], y[4];
            for (int r = 0; r < 4; r++) x[r] = R[a][r][u1];
            lf_dft4(x, &P->ib2[u1], 1, y);
            for (int u2 = 0; u2 < 4; u2++) z[16 * a + u1 + 4 * u2] = y[u2];
        }
    or_c64 S[16][4][4]; /* [u][r][m1] */
    for (int u = 0; u < 16; u++)
        for (int r = 0; r < 4; r++) {
            or_c64 x[4];
            for (int i = 0; i < 4; i++) x[i] = z[u + 16 * (r + 4 * i)];
            lf_dft4(x, &P->ia1[u], 1, S[u][r]);
        }
    for (int u = 0; u < 16; u++)
        for (int m1 = 0; m1 < 4; m1++) {
            or_c64 x[4], y[4];
            for (int r = 0; r < 4; r++) x[r] = S[u][r][m1];
            lf_dft4(x, &P->ia2[4 * u + m1], 1, y);
            for (int m2 = 0; m2 < 4; m2++) {
                int j = u + 16 * (m1 + 4 * m2);
                or_c64 t = cmul(y[m2], P->untw[j]);
                out[j] += or_from_torus(t.re * 0x1p-8);
                out[j + 256] += or_from_torus(t.im * 0x1p-8);
            }
        }
}

void *or_lf_plan_new(void) {
    lf_plan *P = (lf_plan *)malloc(sizeof(lf_plan));
    or_lf_plan_build(P);
    return P;
}
void or_lf_plan_free(void *plan) { free(plan); }
void or_lf_e2(const void *plan, or_c64 *e2) { memcpy(e2, ((const lf_plan *)plan)->e2, sizeof(or_c64) * 256); }

/* ======================================================================================
 * The same for N = 1024 (the 8-bit model's PBS: k = 2, 6 levels of 2^7; the product's br1024 /
 * br1024lat PBS mode).  M = 512 in or_fft_raw_fwd's three radix-8 passes (pass 0 on
 * points t + 64 m, pass 1 on 64 gg + uu + 8 m for lane t = 8 gg + uu, pass 2 on 8 t + m; positions are
 * its output order), every DFT8 split 2 x 4 with the twiddles fused the same way:
 *  - DFT8 of x_m g^m relative to x_0's factor (lf_dft8): fused DFT4s of ratio g^2 over the even and the
 *    odd m, then four fused butterflies a +- rho b, rho = g W8^k1: 72 fma instead of a DFT8 (56 flops)
 *    plus 7 twiddle products (28);
 *  - pass 0's inputs carry the twist psi^(t + 64 m) = psi^t (psi^64)^m: its DFT4s are the N = 512
 *    transform's integer DFT4 (ratio psi^128 = e^{i pi/8}) and its butterflies lane-uniform; psi^t and
 *    the twiddles W^{t kk} become pass 1's ratios g = psi^8 W^{8 gg}, the rest pass 2's ratios
 *    g = psi W^{gg + 8 kk} (lane (gg, kk) = (t >> 3, t & 7)); the forward output is the exact DFT;
 *  - the inverse input carries E2(pos) = psi^((pos >> 6) + ((pos >> 3) & 7)) (the Fourier BSK holds
 *    G conj(E2)), constant over each pass-2 DFT8, which stays a plain inverse DFT8 (dftR); inverse passes
 *    1 and 0 are fused with ratios psi W^{-8 uu} and psi W^{-t}; every ratio is off the axes.
 * Angles 2 pi num / 2048: psi = e^{i pi / 1024} is num 1, W = W_512 num -4, W8 num -256.
 * ====================================================================================== */
typedef struct {
    int N;       /* 1024 */
    or_fft *f;   /* the plain inverse DFT8's W8 factors */
    double s2, c8, t8; /* 1/sqrt(2); cos, tan of pi/8 (psi^128) */
    double p0[8];      /* pass-0 butterflies: (cos, tan) of psi^64 W8^k1         (num 64 - 256 k1) */
    double f1[8][12];  /* forward pass 1, lane group gg: g = psi^8 W^(8 gg)      (num 8 - 32 gg) */
    double f2[64][12]; /* forward pass 2, lane t: g = psi W^((t >> 3) + 8 (t & 7)) (num 1 - 4 (t >> 3) - 32 (t & 7)) */
    double i1[8][12];  /* inverse pass 1, lane column uu: g = psi W^(-8 uu)     (num 1 + 32 uu) */
    double i0[64][12]; /* inverse pass 0, lane t: g = psi W^(-t)                (num 1 + 4 t) */
    or_c64 untw[512];  /* conj(twist[j]); the backward 2^-9 is exact and applied to the sum */
    or_c64 e2[512];    /* conj(E2(pos)) */
} lf1k_plan;

static void lf1k_ct(long num, double *c, double *t) {
    double s;
    sincos2pi(num, 2048, c, &s);
    *t = s / *c;
}
/* a fused DFT8 of ratio g = e^{2 pi i num / 2048}: (cos, tan) of g^4, g^2 (its DFT4s), then of g W8^-+k1 */
static void lf8_make(long num, int inv, double *e) {
    lf1k_ct(4 * num, &e[0], &e[1]);
    lf1k_ct(2 * num, &e[2], &e[3]);
    for (int k1 = 0; k1 < 4; k1++) lf1k_ct(num + (inv ? 256 : -256) * k1, &e[4 + 2 * k1], &e[5 + 2 * k1]);
}

static void or_lf1k_plan_build(lf1k_plan *P) {
    P->N = 1024;
    P->f = or_fft_new(1024);
    P->s2 = 1.0 / sqrt(2.0);
    lf1k_ct(128, &P->c8, &P->t8);
    for (int k1 = 0; k1 < 4; k1++) lf1k_ct(64 - 256 * k1, &P->p0[2 * k1], &P->p0[2 * k1 + 1]);
    for (int g = 0; g < 8; g++) {
        lf8_make(8 - 32 * g, 0, P->f1[g]);
        lf8_make(1 + 32 * g, 1, P->i1[g]);
    }
    for (int t = 0; t < 64; t++) {
        lf8_make(1 - 4 * (t >> 3) - 32 * (t & 7), 0, P->f2[t]);
        lf8_make(1 + 4 * t, 1, P->i0[t]);
    }
    for (int j = 0; j < 512; j++) {
        double c, s;
        sincos2pi(j, 2048, &c, &s);
        P->untw[j].re = c;
        P->untw[j].im = -s;
        sincos2pi(-((j >> 6) + ((j >> 3) & 7)), 2048, &c, &s);
        P->e2[j].re = c;
        P->e2[j].im = s;
    }
}

/* DFT8 (W8 forward / conj inverse) of x_m g^m relative to x_0's factor, natural order out */
static void lf_dft8(const or_c64 *x, const double *e, int inv, or_c64 *y) {
    const lf4 K = {e[0], e[1], e[2], e[3]};
    or_c64 a[4] = {x[0], x[2], x[4], x[6]}, b[4] = {x[1], x[3], x[5], x[7]}, A[4], B[4];
    lf_dft4(a, &K, inv, A);
    lf_dft4(b, &K, inv, B);
    for (int k1 = 0; k1 < 4; k1++) {
        or_c64 r = lf_rot(B[k1], e[5 + 2 * k1]);
        y[k1] = lf_add(A[k1], e[4 + 2 * k1], r);
        y[k1 + 4] = lf_add(A[k1], -e[4 + 2 * k1], r);
    }
}

/* forward transform of one digit polynomial (N = 1024 integers) into X[pos] */
void or_lf1k_fwd(const void *plan, const int64_t *poly, or_c64 *X) {
    const lf1k_plan *P = (const lf1k_plan *)plan;
    or_c64 z[512], z2[512];
    for (int t = 0; t < 64; t++) {
        or_c64 A[2][4];
        for (int n1 = 0; n1 < 2; n1++) {
            int64_t d[4][2];
            for (int i = 0; i < 4; i++) {
                int j = t + 64 * (n1 + 2 * i);
                d[i][0] = poly[j];
                d[i][1] = poly[j + 512];
            }
            lf_int_dft4(d, P->s2, P->c8, P->t8, A[n1]);
        }
        for (int k1 = 0; k1 < 4; k1++) {
            or_c64 r = lf_rot(A[1][k1], P->p0[2 * k1 + 1]);
            z[t + 64 * k1] = lf_add(A[0][k1], P->p0[2 * k1], r);
            z[t + 64 * (k1 + 4)] = lf_add(A[0][k1], -P->p0[2 * k1], r);
        }
    }
    for (int t = 0; t < 64; t++) {
        int gg = t >> 3, uu = t & 7;
        or_c64 x[8], y[8];
        for (int m = 0; m < 8; m++) x[m] = z[64 * gg + uu + 8 * m];
        lf_dft8(x, P->f1[gg], 0, y);
        for (int k = 0; k < 8; k++) z2[64 * gg + uu + 8 * k] = y[k];
    }
    for (int t = 0; t < 64; t++) {
        or_c64 x[8], y[8];
        for (int m = 0; m < 8; m++) x[m] = z2[8 * t + m];
        lf_dft8(x, P->f2[t], 0, y);
        for (int k = 0; k < 8; k++) X[8 * t + k] = y[k];
    }
}

/* backward transform of Y[pos] (which carries the factor E2) added to the torus polynomial out
 * (N = 1024): untwist conj(twist), 2^-9 exact, from_torus */
void or_lf1k_bwd_add(const void *plan, const or_c64 *Y, uint64_t *out) {
    const lf1k_plan *P = (const lf1k_plan *)plan;
    or_c64 z[512], z2[512];
    for (int t = 0; t < 64; t++) {
        or_c64 v[8];
        for (int k = 0; k < 8; k++) v[k] = Y[8 * t + k];
        dftR(P->f, v, 8, 1);
        for (int m = 0; m < 8; m++) z[8 * t + m] = v[m];
    }
    for (int t = 0; t < 64; t++) {
        int gg = t >> 3, uu = t & 7;
        or_c64 x[8], y[8];
        for (int k = 0; k < 8; k++) x[k] = z[64 * gg + uu + 8 * k];
        lf_dft8(x, P->i1[uu], 1, y);
        for (int m = 0; m < 8; m++) z2[64 * gg + uu + 8 * m] = y[m];
    }
    for (int t = 0; t < 64; t++) {
        or_c64 x[8], y[8];
        for (int k = 0; k < 8; k++) x[k] = z2[t + 64 * k];
        lf_dft8(x, P->i0[t], 1, y);
        for (int m = 0; m < 8; m++) {
            int j = t + 64 * m;
            or_c64 tt = cmul(y[m], P->untw[j]);
            out[j] += or_from_torus(tt.re * 0x1p-9);
            out[j + 512] += or_from_torus(tt.im * 0x1p-9);
        }
    }
}

void *or_lf1k_plan_new(void) {
    lf1k_plan *P = (lf1k_plan *)malloc(sizeof(lf1k_plan));
    or_lf1k_plan_build(P);
    return P;
}
void or_lf1k_e2(const void *plan, or_c64 *e2) { memcpy(e2, ((const lf1k_plan *)plan)->e2, sizeof(or_c64) * 512); }

/* the plans' constants in the product's table layouts (lf512.hpp / lf1k.hpp), for
 * tests/native/lf_tables_test.cpp, which compares them with the product's own tables bit for bit */
static void lf4_put(double *t, int off, int n, int idx, const lf4 *k) {
    t[off + 2 * idx] = k->c2;
    t[off + 2 * idx + 1] = k->t2;
    t[off + 2 * (n + idx)] = k->c1;
    t[off + 2 * (n + idx) + 1] = k->t1;
}
void or_lf_table(const void *plan, double *t /*[1700]*/) {
    const lf_plan *P = (const lf_plan *)plan;
    memset(t, 0, sizeof(double) * 1700);
    for (int k = 0; k < 4; k++) {
        lf4_put(t, 0, 4, k, &P->fa2[k]);
        lf4_put(t, 336, 4, k, &P->ib2[k]);
    }
    for (int a = 0; a < 16; a++) {
        lf4_put(t, 16, 16, a, &P->fb1[a]);
        lf4_put(t, 352, 16, a, &P->ia1[a]);
        for (int l = 0; l < 4; l++) {
            lf4_put(t, 80, 64, a + 16 * l, &P->fb2[4 * a + l]);
            lf4_put(t, 416, 64, a + 16 * l, &P->ia2[4 * a + l]);
        }
    }
    t[672] = P->s2;
    t[673] = P->c8;
    t[674] = P->t8;
    memcpy(t + 676, P->untw, sizeof(or_c64) * 256);
    memcpy(t + 1188, P->e2, sizeof(or_c64) * 256);
}
static void lf1k_put(double *t, int off, int n, int idx, const double *e) {
    for (int q = 0; q < 6; q++) {
        t[off + 2 * (q * n + idx)] = e[2 * q];
        t[off + 2 * (q * n + idx) + 1] = e[2 * q + 1];
    }
}
void or_lf1k_table(const void *plan, double *t /*[3788]*/) {
    const lf1k_plan *P = (const lf1k_plan *)plan;
    memset(t, 0, sizeof(double) * 3788);
    t[0] = P->s2;
    t[1] = P->c8;
    t[2] = P->t8;
    memcpy(t + 4, P->p0, sizeof(double) * 8);
    for (int g = 0; g < 8; g++) {
        lf1k_put(t, 12, 8, g, P->f1[g]);
        lf1k_put(t, 876, 8, g, P->i1[g]);
    }
    for (int l = 0; l < 64; l++) {
        lf1k_put(t, 108, 64, l, P->f2[l]);
        lf1k_put(t, 972, 64, l, P->i0[l]);
    }
    memcpy(t + 1740, P->untw, sizeof(or_c64) * 512);
    memcpy(t + 2764, P->e2, sizeof(or_c64) * 512);
}

/* either plan (the tag is its first member) */
static int lf_plan_n(const void *plan) { return *(const int *)plan; }
void or_lf_any_free(void *plan) {
    if (!plan) return;
    if (lf_plan_n(plan) == 1024) or_fft_free(((lf1k_plan *)plan)->f);
    free(plan);
}

/* the Fourier BSK the fused transform multiplies with: G * conj(E2(pos)) per position */
static void lf_rescale(const void *plan, or_c64 *G, size_t polys) {
    const int M = lf_plan_n(plan) / 2;
    const or_c64 *e2 = M == 256 ? ((const lf_plan *)plan)->e2 : ((const lf1k_plan *)plan)->e2;
    for (size_t i = 0; i < polys; i++)
        for (int f = 0; f < M; f++) G[i * M + f] = cmul(G[i * M + f], e2[f]);
}

/* ======================================================================================
 * GLWE / LWE encryption (tfhe-rs encrypt_lwe_ciphertext / encrypt_glwe_ciphertext), with
 * the keygen randomness spec of DESIGN.md: ciphertext #idx of purpose P draws its mask from
 * ChaCha20(seed, nonce = 2P | (idx >> 40) << 8, ctr = (idx mod 2^40) * 2^24) and its noise from
 * the same stream origin with nonce 2P+1 (injective over 64-bit indices).
 * ====================================================================================== */
static uint64_t ct_nonce(int purpose, int noise, uint64_t idx) {
    return (2ull * (uint64_t)purpose + (uint64_t)noise) | ((idx >> 40) << 8);
}
static uint64_t ct_counter(uint64_t idx) { return (idx & ((1ull << 40) - 1)) * CT_STRIDE; }
static void lwe_encrypt(const uint64_t *sk, int dim, uint64_t msg, double sigma, const uint8_t seed[32],
                        int purpose, uint64_t idx, uint64_t *out) {
    rng_t rm, rn;
    rng_init(&rm, seed, ct_nonce(purpose, 0, idx), ct_counter(idx));
    rng_init(&rn, seed, ct_nonce(purpose, 1, idx), ct_counter(idx));
    uint64_t b = 0;
    for (int i = 0; i < dim; i++) {
        out[i] = rng_u64(&rm);
        b += out[i] * sk[i];
    }
    b += msg + rng_gauss_torus(&rn, sigma);
    out[dim] = b;
}

/* GLWE encryption of plaintext polynomial `msg` [N] (NULL = zero) under glwe key (k polys) */
static void glwe_encrypt(const uint64_t *S, int k, int N, const uint64_t *msg, double sigma,
                         const uint8_t seed[32], int purpose, uint64_t idx, uint64_t *out) {
    rng_t rm, rn;
    rng_init(&rm, seed, ct_nonce(purpose, 0, idx), ct_counter(idx));
    rng_init(&rn, seed, ct_nonce(purpose, 1, idx), ct_counter(idx));
    uint64_t *B = out + (size_t)k * N;
    for (int p = 0; p < k; p++)
        for (int j = 0; j < N; j++) out[(size_t)p * N + j] = rng_u64(&rm);
    for (int j = 0; j < N; j++) B[j] = 0;
    for (int p = 0; p < k; p++) {
        const uint64_t *A = out + (size_t)p * N;
        const uint64_t *s = S + (size_t)p * N;
        /* B += A * S_p, S_p binary: sum of negacyclic rotations of A */
        for (int i = 0; i < N; i++) {
            if (!s[i]) continue;
            for (int j = 0; j < N; j++) {
                int t = i + j;
                if (t < N)
                    B[t] += A[j];
                else
                    B[t - N] -= A[j];
            }
        }
    }
    for (int j = 0; j < N; j++) B[j] += (msg ? msg[j] : 0) + rng_gauss_torus(&rn, sigma);
}

size_t or_ksk_len(const or_params *p) { return (size_t)p->k * p->N * p->ks_l * (p->n + 1); }
size_t or_bsk_len(const or_params *p) {
    return (size_t)p->n * p->pbs_l * (p->k + 1) * (p->k + 1) * p->N;
}
size_t or_pfpksk_len(const or_params *p) {
    if (p->model == 2) return (size_t)p->n * p->pfks_l * (p->k + 1) * p->N; /* packing keyswitch key */
    return (size_t)(p->k + 1) * (p->k * p->N + 1) * p->pfks_l * (p->k + 1) * p->N;
}

typedef struct {
    const or_params *p;
    const uint8_t *seed;
    const uint64_t *lwe_sk, *glwe_sk;
    uint64_t *ksk, *bsk, *pfpksk;
    int tid, nthreads;
} kg_job;

static void *kg_worker(void *arg) {
    kg_job *J = (kg_job *)arg;
    const or_params *p = J->p;
    int n = p->n, k = p->k, N = p->N, K = k * N;
    size_t glwe = (size_t)(k + 1) * N;
    uint64_t *msg = (uint64_t *)malloc(sizeof(uint64_t) * N);
    /* KSK: lwe_keyswitch_key_generation; block i, level l encrypts s_big[i] * 2^(64 - B l) */
    for (size_t c = J->tid; c < (size_t)K * p->ks_l; c += J->nthreads) {
        size_t i = c / p->ks_l;
        int l = (int)(c % p->ks_l) + 1;
        uint64_t m = J->glwe_sk[i] << (64 - p->ks_b * l);
        lwe_encrypt(J->lwe_sk, n, m, p->lwe_std, J->seed, P_KSK, c, J->ksk + c * (n + 1));
    }
    /* BSK: GGSW(s_i), level l, row r: r<k plaintext = -s_i*D_l*S_r, r=k plaintext = s_i*D_l */
    for (size_t c = J->tid; c < (size_t)n * p->pbs_l * (k + 1); c += J->nthreads) {
        size_t i = c / ((size_t)p->pbs_l * (k + 1));
        int l = (int)((c / (k + 1)) % p->pbs_l) + 1;
        int r = (int)(c % (k + 1));
        uint64_t factor = (0 - J->lwe_sk[i]) << (64 - p->pbs_b * l); /* encrypt_constant_ggsw */
        if (r < k)
            for (int j = 0; j < N; j++) msg[j] = J->glwe_sk[(size_t)r * N + j] * factor;
        else {
            memset(msg, 0, sizeof(uint64_t) * N);
            msg[0] = 0 - factor;
        }
        glwe_encrypt(J->glwe_sk, k, N, msg, p->glwe_std, J->seed, P_BSK, c, J->bsk + c * glwe);
    }
    if (p->model == 2) {
        /* shortint_1bit: lwe_packing_keyswitch_key_generation (shortint_1bit.rs:176-186): input key
         * element i, level l: GLWE encryption of the constant polynomial s_i * 2^(64 - B l) */
        for (size_t c = J->tid; c < (size_t)n * p->pfks_l; c += J->nthreads) {
            size_t i = c / p->pfks_l;
            int l = (int)(c % p->pfks_l) + 1;
            memset(msg, 0, sizeof(uint64_t) * N);
            msg[0] = J->lwe_sk[i] << (64 - p->pfks_b * l);
            glwe_encrypt(J->glwe_sk, k, N, msg, p->pfks_std, J->seed, P_PFPKSK, c, J->pfpksk + c * glwe);
        }
        free(msg);
        return NULL;
    }
    /* PFPKSK list (circuit_bootstrap_lwe_pfpksk_list): key q, input i (s_K = -1), level l:
     * plaintext = P_q * (-s_i) * 2^(64 - B l), P_q = S_q (q<k) or the constant -1 (q=k). */
    for (size_t c = J->tid; c < (size_t)(k + 1) * (K + 1) * p->pfks_l; c += J->nthreads) {
        size_t q = c / ((size_t)(K + 1) * p->pfks_l);
        size_t i = (c / p->pfks_l) % (K + 1);
        int l = (int)(c % p->pfks_l) + 1;
        uint64_t s = i < (size_t)K ? J->glwe_sk[i] : ~0ull;
        uint64_t f = (0 - s) << (64 - p->pfks_b * l);
        if (q < (size_t)k)
            for (int j = 0; j < N; j++) msg[j] = J->glwe_sk[q * N + j] * f;
        else {
            memset(msg, 0, sizeof(uint64_t) * N);
            msg[0] = (~0ull) * f;
        }
        glwe_encrypt(J->glwe_sk, k, N, msg, p->pfks_std, J->seed, P_PFPKSK, c, J->pfpksk + c * glwe);
    }
    free(msg);
    return NULL;
}

/* the parameter sets whose blind rotation runs the fused-twiddle transform: the product's br512x4 /
 * br512lat shape N = 512, k = 4 (params_sqrd_lvl_64, 3 levels of 2^12, and the shortint_1bit set, 7 levels
 * of 2^6; the engine's lf512_ tests the same two fields) */
static int lf_set(const or_params *p) { return p->N == 512 && p->k == 4; }
/* ... and the N = 1024 one (the product's br1024 / br1024lat PBS shape: k = 2, 6 levels of 2^7, the 8-bit
 * model's set) */
static int lf1k_set(const or_params *p) { return p->N == 1024 && p->k == 2 && p->pbs_l == 6 && p->pbs_b == 7; }

/* transform: OR_TRANSFORM_PRODUCT (the fused-twiddle transform for the sets above, as the product) or
 * OR_TRANSFORM_RADIX (the radix-16 / radix-8 schedule shaped like tfhe-fft for every set, no rescale) */
static void server_key_fourier(or_server_key *sk, int transform) {
    const or_params *p = &sk->p;
    int M = p->N / 2;
    size_t polys = (size_t)p->n * p->pbs_l * (p->k + 1) * (p->k + 1);
    sk->bsk_f = (or_c64 *)malloc(sizeof(or_c64) * polys * M);
    for (size_t i = 0; i < polys; i++)
        or_fft_fwd_torus(sk->fft, sk->bsk + i * p->N, sk->bsk_f + i * M);
    sk->lf = NULL;
    if (transform == OR_TRANSFORM_PRODUCT && lf_set(p)) sk->lf = or_lf_plan_new();
    if (transform == OR_TRANSFORM_PRODUCT && lf1k_set(p)) sk->lf = or_lf1k_plan_new();
    if (sk->lf) lf_rescale(sk->lf, sk->bsk_f, polys);
}

/* shortint_woppbs_1bit.rs:245-268 (gen_keys + new_wopbs_key_only_for_wopbs) */
int or_gen_keys(int param_id, const uint8_t seed[32], int threads, or_client_key **ckp,
                or_server_key **skp) {
    or_params p;
    if (or_params_get(param_id, &p)) return -1;
    int K = p.k * p.N;
    or_client_key *ck = (or_client_key *)calloc(1, sizeof(*ck));
    ck->p = p;
    ck->lwe_sk = (uint64_t *)malloc(sizeof(uint64_t) * p.n);
    ck->glwe_sk = (uint64_t *)malloc(sizeof(uint64_t) * K);
    uint8_t *buf = (uint8_t *)malloc(K > p.n ? K : p.n);
    or_chacha20_stream(seed, P_LWE_SK, 0, buf, p.n);
    for (int i = 0; i < p.n; i++) ck->lwe_sk[i] = buf[i] & 1;
    or_chacha20_stream(seed, P_GLWE_SK, 0, buf, K);
    for (int i = 0; i < K; i++) ck->glwe_sk[i] = buf[i] & 1;
    free(buf);

    or_server_key *sk = (or_server_key *)calloc(1, sizeof(*sk));
    sk->p = p;
    sk->fft = or_fft_new(p.N);
    sk->ksk = (uint64_t *)malloc(sizeof(uint64_t) * or_ksk_len(&p));
    sk->bsk = (uint64_t *)malloc(sizeof(uint64_t) * or_bsk_len(&p));
    sk->pfpksk = (uint64_t *)malloc(sizeof(uint64_t) * or_pfpksk_len(&p));
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    kg_job *jobs = (kg_job *)malloc(sizeof(kg_job) * threads);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (kg_job){&p, seed, ck->lwe_sk, ck->glwe_sk, sk->ksk, sk->bsk, sk->pfpksk, t, threads};
        pthread_create(&th[t], NULL, kg_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    server_key_fourier(sk, OR_TRANSFORM_PRODUCT);
    *ckp = ck;
    *skp = sk;
    return 0;
}

or_server_key *or_server_key_from_raw(int param_id, const uint64_t *ksk, const uint64_t *bsk,
                                      const uint64_t *pfpksk) {
    return or_server_key_from_raw_t(param_id, ksk, bsk, pfpksk, OR_TRANSFORM_PRODUCT);
}

or_server_key *or_server_key_from_raw_t(int param_id, const uint64_t *ksk, const uint64_t *bsk,
                                        const uint64_t *pfpksk, int transform) {
    or_params p;
    if (or_params_get(param_id, &p)) return NULL;
    or_server_key *sk = (or_server_key *)calloc(1, sizeof(*sk));
    sk->p = p;
    sk->fft = or_fft_new(p.N);
    sk->ksk = (uint64_t *)malloc(sizeof(uint64_t) * or_ksk_len(&p));
    sk->bsk = (uint64_t *)malloc(sizeof(uint64_t) * or_bsk_len(&p));
    sk->pfpksk = (uint64_t *)malloc(sizeof(uint64_t) * or_pfpksk_len(&p));
    memcpy(sk->ksk, ksk, sizeof(uint64_t) * or_ksk_len(&p));
    memcpy(sk->bsk, bsk, sizeof(uint64_t) * or_bsk_len(&p));
    memcpy(sk->pfpksk, pfpksk, sizeof(uint64_t) * or_pfpksk_len(&p));
    server_key_fourier(sk, transform);
    return sk;
}

void or_client_key_free(or_client_key *ck) {
    if (!ck) return;
    free(ck->lwe_sk);
    free(ck->glwe_sk);
    free(ck);
}
void or_server_key_free(or_server_key *sk) {
    if (!sk) return;
    free(sk->ksk);
    free(sk->bsk);
    free(sk->pfpksk);
    free(sk->bsk_f);
    or_fft_free(sk->fft);
    or_lf_any_free(sk->lf);
    free(sk);
}

/* ClientKey::encrypt (shortint_woppbs_1bit.rs:200-217): big key, lwe noise, encode_bit */
void or_encrypt_bit(const or_client_key *ck, const uint8_t seed[32], uint64_t index, uint64_t bit,
                    uint64_t *out) {
    lwe_encrypt(ck->glwe_sk, ck->p.k * ck->p.N, or_encode_bit(bit), ck->p.lwe_std, seed, P_ENCRYPT,
                index, out);
}
uint64_t or_decrypt_phase(const or_client_key *ck, const uint64_t *ct) {
    int K = ck->p.k * ck->p.N;
    uint64_t s = 0;
    for (int i = 0; i < K; i++) s += ct[i] * ck->glwe_sk[i];
    return ct[K] - s;
}
uint64_t or_decrypt_small_phase(const or_client_key *ck, const uint64_t *ct) {
    uint64_t s = 0;
    for (int i = 0; i < ck->p.n; i++) s += ct[i] * ck->lwe_sk[i];
    return ct[ck->p.n] - s;
}
/* ClientKey::decrypt (shortint_woppbs_1bit.rs:219-225) */
uint64_t or_decrypt_bit(const or_client_key *ck, const uint64_t *ct) {
    return or_decode_bit(or_decrypt_phase(ck, ct));
}
void or_glwe_decrypt(const or_client_key *ck, const uint64_t *glwe, uint64_t *plain) {
    int k = ck->p.k, N = ck->p.N;
    for (int j = 0; j < N; j++) plain[j] = glwe[(size_t)k * N + j];
    for (int p = 0; p < k; p++) {
        const uint64_t *A = glwe + (size_t)p * N;
        const uint64_t *s = ck->glwe_sk + (size_t)p * N;
        for (int i = 0; i < N; i++) {
            if (!s[i]) continue;
            for (int j = 0; j < N; j++) {
                int t = i + j;
                if (t < N)
                    plain[t] -= A[j];
                else
                    plain[t - N] += A[j];
            }
        }
    }
}

/* ======================================================================================
 * Hot-path primitives
 * ====================================================================================== */

/* tfhe-rs keyswitch_lwe_ciphertext: out = (0,..,0,b) - sum_i sum_l d_{i,l} * KSK[i][l] */
void or_keyswitch(const or_server_key *sk, const uint64_t *in, uint64_t *out) {
    const or_params *p = &sk->p;
    int n = p->n, K = p->k * p->N;
    int64_t d[64];
    for (int j = 0; j < n; j++) out[j] = 0;
    out[n] = in[K];
    for (int i = 0; i < K; i++) {
        or_decompose(in[i], p->ks_b, p->ks_l, d);
        for (int l = 0; l < p->ks_l; l++) {
            if (!d[l]) continue;
            const uint64_t *row = sk->ksk + ((size_t)i * p->ks_l + l) * (n + 1);
            uint64_t dv = (uint64_t)d[l];
            for (int j = 0; j <= n; j++) out[j] -= row[j] * dv;
        }
    }
}

/* fft64::crypto::ggsw::add_external_product_assign.  Fourier GGSW layout
 * [lev-1][row p][col c][M]; levels are consumed finest first (ggsw.into_levels().rev() zipped
 * with the decomposition iterator), rows in order; the f64 MAC is the fixed fma sequence below. */
static void ext_product_add(const or_server_key *sk, const void *lf, const or_c64 *ggsw, int levels, int base_log,
                            const uint64_t *in, uint64_t *out);
void or_external_product_add(const or_server_key *sk, const or_c64 *ggsw, int levels, int base_log,
                             const uint64_t *in, uint64_t *out) {
    ext_product_add(sk, NULL, ggsw, levels, base_log, in, out);
}

/* lf != NULL: the blind rotation's external product with the fused-twiddle transform (ggsw = a BSK
 * element of the rescaled Fourier BSK) */
static void ext_product_add(const or_server_key *sk, const void *lf, const or_c64 *ggsw, int levels, int base_log,
                            const uint64_t *in, uint64_t *out) {
    const or_params *p = &sk->p;
    int k = p->k, N = p->N, M = N / 2;
    size_t glwe = (size_t)(k + 1) * N;
    int64_t *dig = (int64_t *)malloc(sizeof(int64_t) * glwe * levels); /* [lev][p][N] */
    or_c64 *acc = (or_c64 *)calloc((size_t)(k + 1) * M, sizeof(or_c64));
    or_c64 *X = (or_c64 *)malloc(sizeof(or_c64) * M);
    int64_t *poly = (int64_t *)malloc(sizeof(int64_t) * N);
    int64_t d[64];
    for (size_t t = 0; t < glwe; t++) {
        or_decompose(in[t], base_log, levels, d);
        for (int l = 0; l < levels; l++) dig[(size_t)l * glwe + t] = d[l];
    }
    for (int lev = levels; lev >= 1; lev--) {
        for (int r = 0; r <= k; r++) {
            memcpy(poly, dig + (size_t)(lev - 1) * glwe + (size_t)r * N, sizeof(int64_t) * N);
            if (lf && lf_plan_n(lf) == 1024)
                or_lf1k_fwd(lf, poly, X);
            else if (lf)
                or_lf_fwd(lf, poly, X);
            else
                or_fft_fwd_int(sk->fft, poly, X);
            for (int c = 0; c <= k; c++) {
                const or_c64 *G = ggsw + (((size_t)(lev - 1) * (k + 1) + r) * (k + 1) + c) * M;
                or_c64 *A = acc + (size_t)c * M;
                for (int f = 0; f < M; f++) {
                    double re = A[f].re, im = A[f].im;
                    re = fma(X[f].re, G[f].re, re);
                    re = fma(-X[f].im, G[f].im, re);
                    im = fma(X[f].re, G[f].im, im);
                    im = fma(X[f].im, G[f].re, im);
                    A[f].re = re;
                    A[f].im = im;
                }
            }
        }
    }
    for (int c = 0; c <= k; c++) {
        if (lf && lf_plan_n(lf) == 1024)
            or_lf1k_bwd_add(lf, acc + (size_t)c * M, out + (size_t)c * N);
        else if (lf)
            or_lf_bwd_add(lf, acc + (size_t)c * M, out + (size_t)c * N);
        else
            or_fft_add_bwd_torus(sk->fft, acc + (size_t)c * M, out + (size_t)c * N);
    }
    free(dig);
    free(acc);
    free(X);
    free(poly);
}

/* fft64::crypto::ggsw::cmux */
void or_cmux(const or_server_key *sk, uint64_t *ct0, uint64_t *ct1, const or_c64 *ggsw, int levels,
             int base_log) {
    size_t glwe = (size_t)(sk->p.k + 1) * sk->p.N;
    for (size_t t = 0; t < glwe; t++) ct1[t] -= ct0[t];
    or_external_product_add(sk, ggsw, levels, base_log, ct1, ct0);
}

/* glwe_sample_extraction::extract_lwe_sample_from_glwe_ciphertext, nth = 0 */
static void sample_extract(const uint64_t *glwe, int k, int N, uint64_t *lwe) {
    for (int p = 0; p < k; p++) {
        const uint64_t *A = glwe + (size_t)p * N;
        lwe[(size_t)p * N] = A[0];
        for (int j = 1; j < N; j++) lwe[(size_t)p * N + j] = 0 - A[N - j];
    }
    lwe[(size_t)k * N] = glwe[(size_t)k * N];
}

/* fft64::crypto::bootstrap blind_rotate_assign (PBS flavour) + bootstrap: ACC = LUT * X^{-b~},
 * then for each mask element a_i != 0: cmux(ACC, ACC * X^{a~_i}, BSK_i); sample extract. */
void or_bootstrap(const or_server_key *sk, const uint64_t *lwe_in, const uint64_t *lut,
                  uint64_t *lwe_out) {
    const or_params *p = &sk->p;
    int n = p->n, k = p->k, N = p->N, M = N / 2;
    size_t glwe = (size_t)(k + 1) * N;
    uint64_t *acc = (uint64_t *)malloc(sizeof(uint64_t) * glwe);
    uint64_t *ct1 = (uint64_t *)malloc(sizeof(uint64_t) * glwe);
    int64_t bt = (int64_t)or_pbs_modulus_switch(lwe_in[n], N);
    for (int c = 0; c <= k; c++) or_monomial_mul(lut + (size_t)c * N, acc + (size_t)c * N, N, -bt);
    size_t ggsw_sz = (size_t)p->pbs_l * (k + 1) * (k + 1) * M;
    for (int i = 0; i < n; i++) {
        if (lwe_in[i] == 0) continue;
        int64_t at = (int64_t)or_pbs_modulus_switch(lwe_in[i], N);
        for (int c = 0; c <= k; c++) or_monomial_mul(acc + (size_t)c * N, ct1 + (size_t)c * N, N, at);
        for (size_t t = 0; t < glwe; t++) ct1[t] -= acc[t];  /* cmux: acc += ggsw [x] (ct1 - acc) */
        ext_product_add(sk, sk->lf, sk->bsk_f + (size_t)i * ggsw_sz, p->pbs_l, p->pbs_b, ct1, acc);
    }
    sample_extract(acc, k, N, lwe_out);
    free(acc);
    free(ct1);
}

/* fft64::crypto::wop_pbs::homomorphic_shift_boolean: body += 2^62; ACC body = -alpha;
 * PBS; body += alpha, alpha = 2^(63 - cbs_b * level) */
void or_homomorphic_shift_boolean(const or_server_key *sk, const uint64_t *lwe_in, int level,
                                  uint64_t *lwe_out) {
    const or_params *p = &sk->p;
    int n = p->n, k = p->k, N = p->N;
    size_t glwe = (size_t)(k + 1) * N;
    uint64_t *in = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
    memcpy(in, lwe_in, sizeof(uint64_t) * (n + 1));
    in[n] += 1ull << 62;
    uint64_t alpha = 1ull << (63 - p->cbs_b * level);
    uint64_t *lut = (uint64_t *)calloc(glwe, sizeof(uint64_t));
    for (int j = 0; j < N; j++) lut[(size_t)k * N + j] = 0 - alpha;
    or_bootstrap(sk, in, lut, lwe_out);
    lwe_out[(size_t)k * N] += alpha;
    free(in);
    free(lut);
}

/* private_functional_keyswitch_lwe_ciphertext_into_glwe_ciphertext with PFPKSK #q:
 * out = - sum_{i<=K} sum_l d_{i,l} * PFPKSK[q][i][l] */
void or_pfks(const or_server_key *sk, int q, const uint64_t *in, uint64_t *out) {
    const or_params *p = &sk->p;
    int K = p->k * p->N;
    size_t glwe = (size_t)(p->k + 1) * p->N;
    int64_t d[64];
    memset(out, 0, sizeof(uint64_t) * glwe);
    for (int i = 0; i <= K; i++) {
        or_decompose(in[i], p->pfks_b, p->pfks_l, d);
        for (int l = 0; l < p->pfks_l; l++) {
            if (!d[l]) continue;
            const uint64_t *key = sk->pfpksk + (((size_t)q * (K + 1) + i) * p->pfks_l + l) * glwe;
            uint64_t dv = (uint64_t)d[l];
            for (size_t t = 0; t < glwe; t++) out[t] -= key[t] * dv;
        }
    }
}

/* wop_pbs::circuit_bootstrap_boolean with delta_log = 63 (shift 0): per level, PBS then the k+1
 * PFKS into the GGSW level matrix rows. ggsw: [cbs_l][k+1][(k+1)N] */
void or_circuit_bootstrap_boolean(const or_server_key *sk, const uint64_t *lwe_in, uint64_t *ggsw) {
    const or_params *p = &sk->p;
    int K = p->k * p->N;
    size_t glwe = (size_t)(p->k + 1) * p->N;
    uint64_t *big = (uint64_t *)malloc(sizeof(uint64_t) * (K + 1));
    for (int lev = 1; lev <= p->cbs_l; lev++) {
        or_homomorphic_shift_boolean(sk, lwe_in, lev, big);
        for (int q = 0; q <= p->k; q++) or_pfks(sk, q, big, ggsw + ((size_t)(lev - 1) * (p->k + 1) + q) * glwe);
    }
    free(big);
}

/* FourierGgswCiphertext::fill_with_forward_fourier */
void or_ggsw_to_fourier(const or_server_key *sk, const uint64_t *ggsw, int levels, or_c64 *out) {
    int N = sk->p.N, M = N / 2;
    size_t polys = (size_t)levels * (sk->p.k + 1) * (sk->p.k + 1);
    for (size_t i = 0; i < polys; i++) or_fft_fwd_torus(sk->fft, ggsw + i * N, out + i * M);
}

/* wop_pbs::vertical_packing: cmux tree over the first `tree` GGSWs (MSB first), then
 * blind_rotate_assign (VP flavour) over the rest in reverse with X^{-2^t}, then extract coeff 0 */
void or_vertical_packing(const or_server_key *sk, const uint64_t *lut, int n_polys,
                         const or_c64 *ggsws, int n_in, uint64_t *lwe_out) {
    const or_params *p = &sk->p;
    int k = p->k, N = p->N, M = N / 2;
    size_t glwe = (size_t)(k + 1) * N;
    size_t ggsw_sz = (size_t)p->cbs_l * (k + 1) * (k + 1) * M;
    int tree = 0;
    while ((1 << tree) < n_polys) tree++;
    if (tree > n_in) tree = 0;
    /* cmux_tree_memory_optimized: leaves are trivial GLWEs of the LUT polys; level t combines
     * pairs with the GGSW of bit (tree-1-t) of the selector (MSB first order). */
    uint64_t *nodes = (uint64_t *)calloc(glwe * (size_t)n_polys, sizeof(uint64_t));
    for (int i = 0; i < n_polys; i++) memcpy(nodes + (size_t)i * glwe + (size_t)k * N, lut + (size_t)i * N, sizeof(uint64_t) * N);
    int cnt = n_polys;
    for (int t = tree - 1; t >= 0; t--) {
        for (int i = 0; i < cnt / 2; i++) {
            uint64_t *c0 = nodes + (size_t)(2 * i) * glwe, *c1 = nodes + (size_t)(2 * i + 1) * glwe;
            or_cmux(sk, c0, c1, ggsws + (size_t)t * ggsw_sz, p->cbs_l, p->cbs_b);
            if (i) memcpy(nodes + (size_t)i * glwe, c0, sizeof(uint64_t) * glwe);
        }
        cnt /= 2;
    }
    uint64_t *acc = nodes;
    uint64_t *ct1 = (uint64_t *)malloc(sizeof(uint64_t) * glwe);
    int64_t deg = 1;
    for (int g = n_in - 1; g >= tree; g--) {
        for (int c = 0; c <= k; c++) or_monomial_mul(acc + (size_t)c * N, ct1 + (size_t)c * N, N, -deg);
        deg <<= 1;
        or_cmux(sk, acc, ct1, ggsws + (size_t)g * ggsw_sz, p->cbs_l, p->cbs_b);
    }
    sample_extract(acc, k, N, lwe_out);
    free(nodes);
    free(ct1);
}

size_t or_lut_small_len(int N, int input_bits) {
    int logN = 0;
    while ((1 << logN) < N) logN++;
    int tree = input_bits > logN ? input_bits - logN : 0;
    return (size_t)N << tree;
}

/* generate_multivariate_luts (shortint_woppbs_1bit.rs:366-403): small LUT j holds, at
 * coefficient v, encode_bit(bit (output_bits-1-j) of f(v)) */
void or_generate_lut(int N, int input_bits, int output_bits, const uint64_t *f_table, uint64_t *out) {
    size_t small = or_lut_small_len(N, input_bits);
    memset(out, 0, sizeof(uint64_t) * small * output_bits);
    for (int j = 0; j < output_bits; j++)
        for (size_t v = 0; v < ((size_t)1 << input_bits); v++)
            out[(size_t)j * small + v] = or_encode_bit((f_table[v] >> (output_bits - 1 - j)) & 1);
}

/* FheContext::circuit_bootstrap (shortint_woppbs_1bit.rs:292-336) -> extract_dual_bit_from_bit
 * (:339-363, = keyswitch) per bit, then circuit_bootstrap_boolean_vertical_packing */
void or_circuit_bootstrap(const or_server_key *sk, const uint64_t *bits, int n_in,
                          const uint64_t *lut, int n_out, uint64_t *out) {
    const or_params *p = &sk->p;
    int n = p->n, k = p->k, N = p->N, M = N / 2, K = k * N;
    size_t glwe = (size_t)(k + 1) * N;
    size_t ggsw_std = (size_t)p->cbs_l * (k + 1) * glwe;
    size_t ggsw_f = (size_t)p->cbs_l * (k + 1) * (k + 1) * M;
    (void)M;
    (void)ggsw_std;
    (void)ggsw_f;
    uint64_t *small = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1) * n_in);
    for (int b = 0; b < n_in; b++) or_keyswitch(sk, bits + (size_t)b * (K + 1), small + (size_t)b * (n + 1));
    or_cbs_vp_small(sk, small, n_in, lut, n_out, out);
    free(small);
}

/* circuit_bootstrap_boolean_vertical_packing on small-key bits (tfhe-rs wop_pbs; the 8-bit model's
 * WopbsKey::circuit_bootstrapping_vertical_packing, shortint_woppbs_8bit.rs:299-335): bits
 * [n_in][n+1] (MSB first), lut [n_out][small_len], out [n_out][K+1] */
void or_cbs_vp_small(const or_server_key *sk, const uint64_t *bits, int n_in, const uint64_t *lut, int n_out,
                     uint64_t *out) {
    const or_params *p = &sk->p;
    int n = p->n, k = p->k, N = p->N, M = N / 2, K = k * N;
    size_t glwe = (size_t)(k + 1) * N;
    size_t ggsw_std = (size_t)p->cbs_l * (k + 1) * glwe;
    size_t ggsw_f = (size_t)p->cbs_l * (k + 1) * (k + 1) * M;
    uint64_t *g = (uint64_t *)malloc(sizeof(uint64_t) * ggsw_std);
    or_c64 *gf = (or_c64 *)malloc(sizeof(or_c64) * ggsw_f * n_in);
    for (int b = 0; b < n_in; b++) {
        or_circuit_bootstrap_boolean(sk, bits + (size_t)b * (n + 1), g);
        or_ggsw_to_fourier(sk, g, p->cbs_l, gf + (size_t)b * ggsw_f);
    }
    size_t small_len = or_lut_small_len(N, n_in);
    int n_polys = (int)(small_len / N);
    for (int j = 0; j < n_out; j++)
        or_vertical_packing(sk, lut + (size_t)j * small_len, n_polys, gf, n_in, out + (size_t)j * (K + 1));
    free(g);
    free(gf);
}

/* ======================================================================================
 * AES (src/aes_128.rs, src/aes_128/plain.rs, src/aes_128/fhe/fhe_sbox_gal_mul_pbs.rs)
 * ====================================================================================== */
const uint8_t or_sbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76,
    0xca, 0x82, 0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0,
    0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15,
    0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75,
    0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84,
    0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf,
    0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8,
    0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2,
    0xcd, 0x0c, 0x13, 0xec, 0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73,
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb,
    0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79,
    0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08,
    0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a,
    0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e,
    0xe1, 0xf8, 0x98, 0x11, 0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf,
    0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16,
};
static const uint8_t RC[11] = {0x00, 0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1B, 0x36};

/* aes_128.rs:42-56 -- including the reduction quirk (XOR 0x1b when the high bit is CLEAR) */
uint8_t or_gf_256_mul_quirk(uint8_t a, uint8_t b) {
    uint8_t res = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) res ^= a;
        uint8_t hi = a & 0x80;
        a = (uint8_t)(a << 1);
        if (hi != 0x80) a ^= 0x1b;
        b >>= 1;
    }
    return res;
}

/* plain.rs:106-132 */
void or_plain_key_schedule(const uint8_t key[16], uint8_t rk[176]) {
    memcpy(rk, key, 16);
    for (int i = 4; i < 44; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 4 == 0) {
            uint8_t r0 = t[0];
            t[0] = or_sbox[t[1]] ^ RC[i / 4];
            t[1] = or_sbox[t[2]];
            t[2] = or_sbox[t[3]];
            t[3] = or_sbox[r0];
        }
        for (int j = 0; j < 4; j++) rk[4 * i + j] = rk[4 * (i - 4) + j] ^ t[j];
    }
}

/* plain.rs:75-103 (state index 4*col + row == block byte order) */
void or_plain_encrypt_block(const uint8_t rk[176], const uint8_t in[16], int rounds, uint8_t out[16]) {
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
    for (int r = 1; r <= rounds; r++) {
        int last = (r == rounds);
        for (int i = 0; i < 16; i++) s[i] = or_sbox[s[i]];
        for (int c = 0; c < 4; c++)
            for (int row = 0; row < 4; row++) t[4 * c + row] = s[4 * ((c + row) % 4) + row];
        if (!last) {
            for (int c = 0; c < 4; c++) {
                uint8_t *col = t + 4 * c, o[4];
                for (int i = 0; i < 4; i++)
                    o[i] = or_gf_256_mul_quirk(col[i], 2) ^ col[(i + 3) % 4] ^ col[(i + 2) % 4] ^
                           or_gf_256_mul_quirk(col[(i + 1) % 4], 3);
                memcpy(col, o, 4);
            }
        }
        const uint8_t *k = last ? rk + 160 : rk + 16 * r;
        for (int i = 0; i < 16; i++) s[i] = t[i] ^ k[i];
    }
    memcpy(out, s, 16);
}

/* ---- FHE driver: fhe_sbox_gal_mul_pbs::encrypt_block_for_rounds (:84-132) ---- */
typedef struct {
    const or_server_key *sk;
    const uint64_t *in; /* [n_bytes][8][K+1] */
    uint64_t *out;      /* [n_bytes][n_out][K+1] */
    const uint64_t *lut;
    int n_out, n_bytes, tid, nthreads;
} sb_job;

static void *sb_worker(void *arg) {
    sb_job *J = (sb_job *)arg;
    int K = J->sk->p.k * J->sk->p.N;
    for (int b = J->tid; b < J->n_bytes; b += J->nthreads)
        or_circuit_bootstrap(J->sk, J->in + (size_t)b * 8 * (K + 1), 8, J->lut, J->n_out,
                             J->out + (size_t)b * J->n_out * (K + 1));
    return NULL;
}

static void sub_bytes_lut(const or_server_key *sk, const uint64_t *in, int n_bytes, const uint64_t *lut,
                          int n_out, int threads, uint64_t *out) {
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    sb_job *jobs = (sb_job *)malloc(sizeof(sb_job) * threads);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (sb_job){sk, in, out, lut, n_out, n_bytes, t, threads};
        pthread_create(&th[t], NULL, sb_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
}

/* fhe_impls/shortint_woppbs_1bit.rs:94-128 (8 -> 24 LUT: S, 2S', 3S' with the quirky gf) */
static void galmul_lut(int N, uint64_t *lut) {
    uint64_t f[256];
    for (int x = 0; x < 256; x++) {
        uint8_t s = or_sbox[x];
        f[x] = ((uint64_t)or_gf_256_mul_quirk(s, 1) << 16) | ((uint64_t)or_gf_256_mul_quirk(s, 2) << 8) |
               (uint64_t)or_gf_256_mul_quirk(s, 3);
    }
    or_generate_lut(N, 8, 24, f, lut);
}
static void sbox_lut(int N, uint64_t *lut) {
    uint64_t f[256];
    for (int x = 0; x < 256; x++) f[x] = or_sbox[x];
    or_generate_lut(N, 8, 8, f, lut);
}

void or_sub_bytes_gal_mul(const or_server_key *sk, const uint64_t *state_bytes, int n_bytes,
                          int threads, uint64_t *out) {
    int N = sk->p.N;
    uint64_t *lut = (uint64_t *)malloc(sizeof(uint64_t) * 24 * N);
    galmul_lut(N, lut);
    sub_bytes_lut(sk, state_bytes, n_bytes, lut, 24, threads, out);
    free(lut);
}

static void lwe_add(uint64_t *a, const uint64_t *b, int len) {
    for (int i = 0; i < len; i++) a[i] += b[i];
}

void or_aes_encrypt_block(const or_server_key *sk, const uint64_t *rk, const uint64_t *block,
                          int rounds, int threads, uint64_t *out) {
    int N = sk->p.N, K = sk->p.k * N, L = K + 1;
    size_t byte_sz = (size_t)8 * L;
    uint64_t *state = (uint64_t *)malloc(sizeof(uint64_t) * 16 * byte_sz);
    uint64_t *muls = (uint64_t *)malloc(sizeof(uint64_t) * 16 * 3 * byte_sz);
    uint64_t *lut24 = (uint64_t *)malloc(sizeof(uint64_t) * 24 * N);
    uint64_t *lut8 = (uint64_t *)malloc(sizeof(uint64_t) * 8 * N);
    galmul_lut(N, lut24);
    sbox_lut(N, lut8);
    /* ARK(rk[0..4]): byte index 4j + i (block order) ^= word j byte i */
    memcpy(state, block, sizeof(uint64_t) * 16 * byte_sz);
    for (int i = 0; i < 16 * 8; i++) lwe_add(state + (size_t)i * L, rk + (size_t)i * L, L);
    for (int r = 1; r < rounds; r++) {
        sub_bytes_lut(sk, state, 16, lut24, 24, threads, muls); /* muls[byte][24][L] */
        /* ShiftRows on the three states, MixColumns, ARK(rk[4r..4r+4]) */
        for (int c = 0; c < 4; c++)
            for (int row = 0; row < 4; row++)
                for (int bit = 0; bit < 8; bit++) {
                    uint64_t *o = state + ((size_t)(4 * c + row) * 8 + bit) * L;
                    /* after ShiftRows, state[r'][c] = sub[r'][(c + r') % 4] */
#define SRC(rr, m) (muls + (((size_t)(4 * ((c + (rr)) % 4) + (rr)) * 24) + 8 * (m) + bit) * L)
                    memcpy(o, SRC(row, 1), sizeof(uint64_t) * L);            /* x2 */
                    lwe_add(o, SRC((row + 3) % 4, 0), L);                   /* x1 */
                    lwe_add(o, SRC((row + 2) % 4, 0), L);                   /* x1 */
                    lwe_add(o, SRC((row + 1) % 4, 2), L);                   /* x3 */
#undef SRC
                    lwe_add(o, rk + ((size_t)(16 * r + 4 * c + row) * 8 + bit) * L, L);
                }
    }
    /* last round: sub_bytes (8->8 SBOX), shift_rows, ARK(rk[40..44]) */
    sub_bytes_lut(sk, state, 16, lut8, 8, threads, muls); /* muls[byte][8][L] */
    for (int c = 0; c < 4; c++)
        for (int row = 0; row < 4; row++)
            for (int bit = 0; bit < 8; bit++) {
                uint64_t *o = out + ((size_t)(4 * c + row) * 8 + bit) * L;
                memcpy(o, muls + (((size_t)(4 * ((c + row) % 4) + row) * 8) + bit) * L, sizeof(uint64_t) * L);
                lwe_add(o, rk + ((size_t)(160 + 4 * c + row) * 8 + bit) * L, L);
            }
    free(state);
    free(muls);
    free(lut24);
    free(lut8);
}

/* ======================================================================================
 * 8-bit model (src/tfhe/shortint_woppbs_8bit.rs, src/aes_128/fhe/fhe_impls/shortint_woppbs_8bit.rs,
 * src/aes_128/fhe/fhe_sbox_pbs.rs)
 * ====================================================================================== */
/* ClientKey::encrypt (shortint_woppbs_8bit.rs:199-214): LWE under the SMALL key, lwe noise */
void or_encrypt_small_bit(const or_client_key *ck, const uint8_t seed[32], uint64_t index, uint64_t bit,
                          uint64_t *out) {
    lwe_encrypt(ck->lwe_sk, ck->p.n, or_encode_bit(bit), ck->p.lwe_std, seed, P_ENCRYPT, index, out);
}
uint64_t or_decrypt_small_bit(const or_client_key *ck, const uint64_t *ct) {
    return or_decode_bit(or_decrypt_small_phase(ck, ct));
}
/* shortint ClientKey::encrypt_without_padding (EncryptionKeyChoice::Big: big key, glwe noise),
 * message modulus 256, carry 1: plaintext = m * 2^56 (test inputs for extract_bits) */
void or_encrypt_int(const or_client_key *ck, const uint8_t seed[32], uint64_t index, uint64_t value,
                    uint64_t *out) {
    lwe_encrypt(ck->glwe_sk, ck->p.k * ck->p.N, (value & 255) << 56, ck->p.glwe_std, seed, P_ENCRYPT_INT, index,
                out);
}
/* decrypt_without_padding: round(phase / 2^56) mod 256 */
uint64_t or_decrypt_int(const or_client_key *ck, const uint64_t *ct) {
    uint64_t ph = or_decrypt_phase(ck, ct);
    return ((ph + (1ull << 55)) >> 56) & 255;
}

/* WopbsKey::generate_lut_without_padding (tfhe-rs shortint/wopbs, called by
 * FheContext::generate_lookup_table, shortint_woppbs_8bit.rs:262-265) for message modulus 256,
 * carry 1: lut[i] = (f(i mod 256) mod 256) << 56 over max(256, N) entries */
void or_generate_lut_without_padding(int N, const uint64_t *f_table, uint64_t *out) {
    int size = N > 256 ? N : 256;
    for (int i = 0; i < size; i++) out[i] = (f_table[i & 255] & 255) << 56;
}

/* tfhe-rs fft64::crypto::wop_pbs::extract_bits (shortint_woppbs_8bit.rs:268-296 calls it through
 * WopbsKey::extract_bits with DeltaLog(56), ExtractedBitsCount(8)): big-key lwe_in [K+1] ->
 * out [nbits][n+1] small-key bit ciphertexts, MSB first.  Bit bit_idx (LSB first): shift it to the
 * MSB, keyswitch (the output), then unless it is the last: PBS of (ks + q/4) with the accumulator
 * -alpha, alpha = 2^(delta_log - 1 + bit_idx), + alpha, and subtract from the input. */
void or_extract_bits(const or_server_key *sk, const uint64_t *lwe_in, int delta_log, int nbits, uint64_t *out) {
    const or_params *p = &sk->p;
    int n = p->n, k = p->k, N = p->N, K = k * N;
    size_t glwe = (size_t)(k + 1) * N;
    uint64_t *buf = (uint64_t *)malloc(sizeof(uint64_t) * (K + 1));
    uint64_t *sh = (uint64_t *)malloc(sizeof(uint64_t) * (K + 1));
    uint64_t *pbs = (uint64_t *)malloc(sizeof(uint64_t) * (K + 1));
    uint64_t *ks = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
    uint64_t *acc = (uint64_t *)calloc(glwe, sizeof(uint64_t));
    memcpy(buf, lwe_in, sizeof(uint64_t) * (K + 1));
    for (int bit_idx = 0; bit_idx < nbits; bit_idx++) {
        int shift = 64 - delta_log - bit_idx - 1;
        for (int i = 0; i <= K; i++) sh[i] = buf[i] << shift;
        or_keyswitch(sk, sh, ks);
        memcpy(out + (size_t)(nbits - 1 - bit_idx) * (n + 1), ks, sizeof(uint64_t) * (n + 1));
        if (bit_idx == nbits - 1) break;
        ks[n] += 1ull << 62;
        uint64_t alpha = 1ull << (delta_log - 1 + bit_idx);
        for (int j = 0; j < N; j++) acc[(size_t)k * N + j] = 0 - alpha;
        or_bootstrap(sk, ks, acc, pbs);
        pbs[K] += alpha;
        for (int i = 0; i <= K; i++) buf[i] -= pbs[i];
    }
    free(buf);
    free(sh);
    free(pbs);
    free(ks);
    free(acc);
}

/* Byte::bootstrap_with_lut (fhe_impls/shortint_woppbs_8bit.rs:37-42): bootstrap_from_bits
 * (CBS-VP of the 8 small-key bits with a without-padding LUT -> one big-key int ciphertext), then
 * extract_bits_from_ciphertext.  bits/out [8][n+1], lut [N] */
void or_bootstrap_with_lut8(const or_server_key *sk, const uint64_t *bits, const uint64_t *lut, uint64_t *out) {
    int K = sk->p.k * sk->p.N;
    uint64_t *ict = (uint64_t *)malloc(sizeof(uint64_t) * (K + 1));
    or_cbs_vp_small(sk, bits, 8, lut, 1, ict);
    or_extract_bits(sk, ict, 56, 8, out);
    free(ict);
}

/* fhe_sbox_pbs::gf_256_mul (:33-53) on symbolic bytes: coef[o][i] = how many times input bit i
 * (MSB-first) is added into output bit o (XORs are LWE additions, so nothing cancels) */
void or_gf_256_mul_terms(uint8_t b, int coef[8][8]) {
    int a[8][8], res[8][8];
    memset(a, 0, sizeof(a));
    memset(res, 0, sizeof(res));
    for (int i = 0; i < 8; i++) a[i][i] = 1;
    for (int it = 0; it < 8; it++) {
        if (b & 1)
            for (int o = 0; o < 8; o++)
                for (int i = 0; i < 8; i++) res[o][i] += a[o][i];
        int red[8];
        memcpy(red, a[0], sizeof(red)); /* shl_assign_1: old a[0] out, rotate left, trivial 0 in */
        for (int o = 0; o < 7; o++) memcpy(a[o], a[o + 1], sizeof(red));
        memset(a[7], 0, sizeof(red));
        const int taps[4] = {3, 4, 6, 7};
        for (int t = 0; t < 4; t++)
            for (int i = 0; i < 8; i++) a[taps[t]][i] += red[i];
        b >>= 1;
    }
    memcpy(coef, res, sizeof(res));
}

/* MixColumns of fhe_sbox_pbs (:56-73) as a linear map on one column's 32 bits:
 * coef[32 out][32 in], byte-major, MSB-first bits */
void or_mix_column_terms(int coef[32][32]) {
    int g1[8][8], g2[8][8], g3[8][8];
    or_gf_256_mul_terms(1, g1);
    or_gf_256_mul_terms(2, g2);
    or_gf_256_mul_terms(3, g3);
    memset(coef, 0, sizeof(int) * 32 * 32);
    for (int i = 0; i < 4; i++)
        for (int o = 0; o < 8; o++)
            for (int x = 0; x < 8; x++) {
                coef[8 * i + o][8 * i + x] += g2[o][x];
                coef[8 * i + o][8 * ((i + 3) % 4) + x] += g1[o][x];
                coef[8 * i + o][8 * ((i + 2) % 4) + x] += g1[o][x];
                coef[8 * i + o][8 * ((i + 1) % 4) + x] += g3[o][x];
            }
}

typedef struct {
    const or_server_key *sk;
    const uint64_t *in, *lut;
    uint64_t *out;
    int n_bytes, tid, nthreads;
} sb8_job;

static void *sb8_worker(void *arg) {
    sb8_job *J = (sb8_job *)arg;
    size_t byte_sz = (size_t)8 * (J->sk->p.n + 1);
    for (int b = J->tid; b < J->n_bytes; b += J->nthreads)
        or_bootstrap_with_lut8(J->sk, J->in + b * byte_sz, J->lut, J->out + b * byte_sz);
    return NULL;
}

/* SubBytes of fhe_sbox_pbs (:23-31) with ByteT::sbox_substitute of the 8-bit model, threads over bytes */
void or_sub_bytes8(const or_server_key *sk, const uint64_t *state, int n_bytes, int threads, uint64_t *out) {
    int N = sk->p.N;
    uint64_t f[256];
    for (int x = 0; x < 256; x++) f[x] = or_sbox[x];
    uint64_t *lut = (uint64_t *)malloc(sizeof(uint64_t) * (N > 256 ? N : 256));
    or_generate_lut_without_padding(N, f, lut);
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    sb8_job *jobs = (sb8_job *)malloc(sizeof(sb8_job) * threads);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (sb8_job){sk, state, lut, out, n_bytes, t, threads};
        pthread_create(&th[t], NULL, sb8_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    free(lut);
}

/* fhe_sbox_pbs::encrypt_block_for_rounds (:75-121) on small-key bit arrays: rk [44*32][n+1],
 * block/out [128][n+1] (block byte order, MSB-first bits) */
void or_aes8_encrypt_block(const or_server_key *sk, const uint64_t *rk, const uint64_t *block, int rounds,
                           int threads, uint64_t *out) {
    int L = sk->p.n + 1;
    size_t byte_sz = (size_t)8 * L;
    uint64_t *state = (uint64_t *)malloc(sizeof(uint64_t) * 16 * byte_sz);
    uint64_t *sb = (uint64_t *)malloc(sizeof(uint64_t) * 16 * byte_sz);
    int coef[32][32];
    or_mix_column_terms(coef);
    memcpy(state, block, sizeof(uint64_t) * 16 * byte_sz);
    for (int i = 0; i < 128; i++) lwe_add(state + (size_t)i * L, rk + (size_t)i * L, L);
    for (int r = 1; r <= rounds; r++) {
        int last = r == rounds;
        or_sub_bytes8(sk, state, 16, threads, sb);
        /* shift_rows: state[row][c] = sb[row][(c + row) % 4]; byte index 4c + row */
        for (int c = 0; c < 4; c++)
            for (int row = 0; row < 4; row++)
                memcpy(state + (size_t)(4 * c + row) * byte_sz, sb + (size_t)(4 * ((c + row) % 4) + row) * byte_sz,
                       sizeof(uint64_t) * byte_sz);
        if (!last) {
            memcpy(sb, state, sizeof(uint64_t) * 16 * byte_sz);
            for (int c = 0; c < 4; c++)
                for (int o = 0; o < 32; o++) {
                    uint64_t *dst = state + ((size_t)32 * c + o) * L;
                    memset(dst, 0, sizeof(uint64_t) * L);
                    for (int i = 0; i < 32; i++)
                        for (int t = 0; t < coef[o][i]; t++) lwe_add(dst, sb + ((size_t)32 * c + i) * L, L);
                }
        }
        const uint64_t *k = rk + (size_t)(last ? 160 : 16 * r) * byte_sz;
        for (int i = 0; i < 128; i++) lwe_add(state + (size_t)i * L, k + (size_t)i * L, L);
    }
    memcpy(out, state, sizeof(uint64_t) * 16 * byte_sz);
    free(state);
    free(sb);
}

/* ======================================================================================
 * shortint_1bit model (src/tfhe/shortint_1bit.rs; AES driver src/aes_128/fhe/fhe_impls/shortint_1bit.rs)
 * Bits are shortint ciphertexts under the SMALL key (EncryptionKeyChoice::Small), message m * 2^62
 * (message modulus 2, carry 1: delta = 2^63 / 2).
 * ====================================================================================== */
/* shortint ClientKey::encrypt (shortint_1bit.rs:157-160 -> tfhe shortint encrypt, Small key, lwe noise) */
void or_s1_encrypt(const or_client_key *ck, const uint8_t seed[32], uint64_t index, uint64_t bit, uint64_t *out) {
    lwe_encrypt(ck->lwe_sk, ck->p.n, (bit & 1) << 62, ck->p.lwe_std, seed, P_ENCRYPT, index, out);
}
/* shortint decrypt_message_and_carry % message_modulus: (x + ((x & delta/2) << 1)) / delta mod 2 */
uint64_t or_s1_decrypt(const or_client_key *ck, const uint64_t *ct) {
    uint64_t x = or_decrypt_small_phase(ck, ct);
    uint64_t rounding = (x & (1ull << 61)) << 1;
    return ((x + rounding) >> 62) & 1;
}

/* test_vector_from_cleartext_fn (shortint_1bit.rs:365-390): body[0..N/2) = encode(f(0)),
 * body[N/2..N) = encode(f(1)), encode_bit = m << 62 (:339-343), then rotate_left(N/4) */
void or_s1_tv_from_fn(int k, int N, uint64_t f0, uint64_t f1, uint64_t *glwe) {
    memset(glwe, 0, sizeof(uint64_t) * (size_t)(k + 1) * N);
    uint64_t *body = glwe + (size_t)k * N;
    uint64_t *tmp = (uint64_t *)malloc(sizeof(uint64_t) * N);
    int box = N / 2, half = box / 2;
    for (int j = 0; j < N; j++) tmp[j] = (j < box ? (f0 & 1) : (f1 & 1)) << 62;
    for (int j = 0; j < N; j++) body[j] = tmp[(j + half) % N]; /* slice::rotate_left(half) */
    free(tmp);
}

/* tfhe-rs keyswitch_lwe_ciphertext_into_glwe_ciphertext: out = 0, body[0] = b, then
 * out -= sum_{i<n} sum_l d_{i,l} * PKSK[i][l] (decomposition of each mask element, levels 1..l) */
void or_s1_pks(const or_server_key *sk, const uint64_t *in, uint64_t *out) {
    const or_params *p = &sk->p;
    int n = p->n;
    size_t glwe = (size_t)(p->k + 1) * p->N;
    int64_t d[64];
    memset(out, 0, sizeof(uint64_t) * glwe);
    out[(size_t)p->k * p->N] = in[n];
    for (int i = 0; i < n; i++) {
        or_decompose(in[i], p->pfks_b, p->pfks_l, d);
        for (int l = 0; l < p->pfks_l; l++) {
            if (!d[l]) continue;
            const uint64_t *key = sk->pfpksk + ((size_t)i * p->pfks_l + l) * glwe;
            uint64_t dv = (uint64_t)d[l];
            for (size_t t = 0; t < glwe; t++) out[t] -= key[t] * dv;
        }
    }
}

static void glwe_monomial_mul(const or_params *p, uint64_t *g, int64_t degree) {
    uint64_t *tmp = (uint64_t *)malloc(sizeof(uint64_t) * p->N);
    for (int c = 0; c <= p->k; c++) {
        or_monomial_mul(g + (size_t)c * p->N, tmp, p->N, degree);
        memcpy(g + (size_t)c * p->N, tmp, sizeof(uint64_t) * p->N);
    }
    free(tmp);
}
static void glwe_add(const or_params *p, uint64_t *a, const uint64_t *b) {
    for (size_t t = 0; t < (size_t)(p->k + 1) * p->N; t++) a[t] += b[t];
}

/* keyswitch_lwe_ciphertext_list_and_pack_in_glwe_ciphertext: ciphertext #j keyswitched, times X^j, summed */
void or_s1_pack(const or_server_key *sk, const uint64_t *cts, int count, uint64_t *out) {
    const or_params *p = &sk->p;
    size_t glwe = (size_t)(p->k + 1) * p->N;
    uint64_t *buf = (uint64_t *)malloc(sizeof(uint64_t) * glwe);
    memset(out, 0, sizeof(uint64_t) * glwe);
    for (int j = 0; j < count; j++) {
        or_s1_pks(sk, cts + (size_t)j * (p->n + 1), buf);
        glwe_monomial_mul(p, buf, j);
        glwe_add(p, out, buf);
    }
    free(buf);
}

/* test_vector_from_ciphertexts (shortint_1bit.rs:392-492), step by step as the reference writes it:
 * ct0 fills coefficients [0, N/4) and [3N/4, N), ct1 fills [N/4, 3N/4) */
void or_s1_tv_from_cts(const or_server_key *sk, const uint64_t *ct0, const uint64_t *ct1, uint64_t *tv) {
    const or_params *p = &sk->p;
    int N = p->N, box = N / 2, half = box / 2;
    size_t glwe = (size_t)(p->k + 1) * N;
    uint64_t *buf = (uint64_t *)malloc(sizeof(uint64_t) * glwe);
    memset(tv, 0, sizeof(uint64_t) * glwe);
    or_s1_pks(sk, ct0, buf);
    for (int i = 0; i < half; i++) {
        glwe_add(p, tv, buf);
        glwe_monomial_mul(p, buf, 1);
    }
    glwe_monomial_mul(p, buf, N - half - half);
    for (int i = N - half; i < N; i++) {
        glwe_add(p, tv, buf);
        glwe_monomial_mul(p, buf, 1);
    }
    or_s1_pks(sk, ct1, buf);
    glwe_monomial_mul(p, buf, half);
    for (int i = half; i < N - half; i++) {
        glwe_add(p, tv, buf);
        glwe_monomial_mul(p, buf, 1);
    }
    free(buf);
}

/* FheContext::bootstrap_assign (shortint_1bit.rs:264-294): apply_programmable_bootstrap (blind
 * rotation of the test vector, sample extraction) then keyswitch_lwe_ciphertext to the small key */
void or_s1_bootstrap(const or_server_key *sk, const uint64_t *in, const uint64_t *tv, uint64_t *out) {
    const or_params *p = &sk->p;
    uint64_t *big = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)p->k * p->N + 1));
    or_bootstrap(sk, in, tv, big);
    or_keyswitch(sk, big, out);
    free(big);
}

/* generate_multivariate_test_vector (:519-536) + calculate_multivariate_function / apply_selectors_rec
 * (:538-576): the last bit selects inside each test vector, the results are packed pairwise into the
 * next level's test vectors (test_vector_from_ciphertexts), the next-to-last bit selects among those... */
void or_s1_multivariate(const or_server_key *sk, const uint64_t *bits, int nbits, const uint64_t *f_table,
                        uint64_t *out) {
    const or_params *p = &sk->p;
    size_t glwe = (size_t)(p->k + 1) * p->N, L = (size_t)p->n + 1;
    int ntv = 1 << (nbits - 1);
    uint64_t *tvs = (uint64_t *)malloc(sizeof(uint64_t) * glwe * ntv);
    uint64_t *res = (uint64_t *)malloc(sizeof(uint64_t) * L * ntv);
    for (int v = 0; v < ntv; v++) or_s1_tv_from_fn(p->k, p->N, f_table[2 * v], f_table[2 * v + 1], tvs + v * glwe);
    for (int sel = nbits - 1;; sel--) {
        const uint64_t *selector = bits + (size_t)sel * L;
        for (int v = 0; v < ntv; v++) or_s1_bootstrap(sk, selector, tvs + v * glwe, res + v * L);
        if (ntv == 1) break;
        ntv /= 2;
        for (int v = 0; v < ntv; v++) or_s1_tv_from_cts(sk, res + 2 * v * L, res + (2 * v + 1) * L, tvs + v * glwe);
    }
    memcpy(out, res, sizeof(uint64_t) * L);
    free(tvs);
    free(res);
}
