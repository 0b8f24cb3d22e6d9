// Client side: ChaCha20 randomness, key generation, bit encryption, LUT generation, FFT tables.
// See client.hpp for the reference mapping.
#include "client.hpp"

#include <algorithm>

#include <cmath>
#include <cstring>
#include <thread>

namespace tae {

namespace {
constexpr double kPi = 3.14159265358979323846;

inline uint32_t rotl(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }

inline void quarter(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
    a += b; d = rotl(d ^ a, 16);
    c += d; b = rotl(b ^ c, 12);
    a += b; d = rotl(d ^ a, 8);
    c += d; b = rotl(b ^ c, 7);
}
}  // namespace

void chacha20_block(const uint8_t key[32], uint64_t nonce, uint64_t counter, uint8_t out[64]) {
    uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
    for (int i = 0; i < 8; i++) std::memcpy(&st[4 + i], key + 4 * i, 4);  // little-endian host
    st[12] = (uint32_t)counter;
    st[13] = (uint32_t)(counter >> 32);
    st[14] = (uint32_t)nonce;
    st[15] = (uint32_t)(nonce >> 32);
    uint32_t x[16];
    std::memcpy(x, st, sizeof(st));
    for (int r = 0; r < 10; r++) {
        quarter(x[0], x[4], x[8], x[12]);
        quarter(x[1], x[5], x[9], x[13]);
        quarter(x[2], x[6], x[10], x[14]);
        quarter(x[3], x[7], x[11], x[15]);
        quarter(x[0], x[5], x[10], x[15]);
        quarter(x[1], x[6], x[11], x[12]);
        quarter(x[2], x[7], x[8], x[13]);
        quarter(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; i++) {
        uint32_t v = x[i] + st[i];
        std::memcpy(out + 4 * i, &v, 4);
    }
}

ChaChaStream::ChaChaStream(const uint8_t key[32], uint64_t nonce, uint64_t counter)
    : nonce_(nonce), ctr_(counter), pos_(64) {
    std::memcpy(key_, key, 32);
}

uint64_t ChaChaStream::next_u64() {
    if (pos_ == 64) {
        chacha20_block(key_, nonce_, ctr_++, buf_);
        pos_ = 0;
    }
    uint64_t v;
    std::memcpy(&v, buf_ + pos_, 8);
    pos_ += 8;
    return v;
}

uint64_t ChaChaStream::next_gaussian_torus(double sigma) {
    const uint64_t w1 = next_u64(), w2 = next_u64();
    const double u1 = (double)((w1 >> 11) + 1) * 0x1p-53;
    const double u2 = (double)(w2 >> 11) * 0x1p-53;
    const double radius = std::sqrt(-2.0 * std::log(u1));
    const double z = radius * std::cos(2.0 * kPi * u2);
    const double v = std::rint(z * (sigma * 0x1p64));
    return (uint64_t)(int64_t)v;
}

namespace {

// LWE encryption of `msg` under key `sk` (dimension dim), ciphertext #idx of `purpose`.
void lwe_encrypt(const uint8_t seed[32], Purpose purpose, uint64_t idx, const uint64_t *sk, int dim,
                 uint64_t msg, double sigma, uint64_t *out) {
    ChaChaStream mask(seed, ct_nonce(purpose, 0, idx), ct_counter(idx));
    ChaChaStream noise(seed, ct_nonce(purpose, 1, idx), ct_counter(idx));
    uint64_t body = 0;
    for (int i = 0; i < dim; i++) {
        out[i] = mask.next_u64();
        body += out[i] * sk[i];
    }
    out[dim] = body + msg + noise.next_gaussian_torus(sigma);
}

// GLWE encryption of plaintext polynomial `msg` (nullptr = 0) under the binary key S (k polys).
void glwe_encrypt(const uint8_t seed[32], Purpose purpose, uint64_t idx, const uint64_t *S, int k,
                  int N, const uint64_t *msg, double sigma, uint64_t *out) {
    ChaChaStream mask(seed, ct_nonce(purpose, 0, idx), ct_counter(idx));
    ChaChaStream noise(seed, ct_nonce(purpose, 1, idx), ct_counter(idx));
    const size_t kN = (size_t)k * N;
    for (size_t t = 0; t < kN; t++) out[t] = mask.next_u64();
    uint64_t *body = out + kN;
    std::memset(body, 0, sizeof(uint64_t) * N);
    // body += A_p * S_p: the key is binary, so accumulate negacyclic rotations of A_p
    for (int p = 0; p < k; p++) {
        const uint64_t *A = out + (size_t)p * N;
        const uint64_t *s = S + (size_t)p * N;
        for (int i = 0; i < N; i++) {
            if (!s[i]) continue;
            const int split = N - i;
            for (int j = 0; j < split; j++) body[i + j] += A[j];
            for (int j = split; j < N; j++) body[i + j - N] -= A[j];
        }
    }
    for (int j = 0; j < N; j++) body[j] += (msg ? msg[j] : 0) + noise.next_gaussian_torus(sigma);
}

template <class F>
void parallel_for(size_t count, int threads, F fn) {
    if (threads < 1) threads = 1;
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++)
        pool.emplace_back([=]() {
            for (size_t c = (size_t)t; c < count; c += (size_t)threads) fn(c);
        });
    for (auto &th : pool) th.join();
}

}  // namespace

void ClientKey::encrypt_bit_at(uint64_t bit, uint64_t index, uint64_t *out) const {
    lwe_encrypt(seed.data(), ENCRYPT, index, glwe_sk.data(), p.K(), encode_bit(bit), p.lwe_std, out);
}

void ClientKey::encrypt_small_bit_at(uint64_t bit, uint64_t index, uint64_t *out) const {
    lwe_encrypt(seed.data(), ENCRYPT, index, lwe_sk.data(), p.n, encode_bit(bit), p.lwe_std, out);
}

void ClientKey::encrypt_s1_bit_at(uint64_t bit, uint64_t index, uint64_t *out) const {
    lwe_encrypt(seed.data(), ENCRYPT, index, lwe_sk.data(), p.n, (bit & 1) << 62, p.lwe_std, out);
}

uint64_t ClientKey::phase_small(const uint64_t *ct) const {
    uint64_t s = 0;
    for (int i = 0; i < p.n; i++) s += ct[i] * lwe_sk[i];
    return ct[p.n] - s;
}

void ClientKey::encrypt_int_at(uint64_t value, uint64_t index, uint64_t *out) const {
    lwe_encrypt(seed.data(), ENCRYPT_INT, index, glwe_sk.data(), p.K(), (value & 255) << 56, p.glwe_std, out);
}

void s1_test_vector(const Params &p, uint64_t f0, uint64_t f1, uint64_t *glwe) {
    const int N = p.N, box = N / 2, half = box / 2;
    std::memset(glwe, 0, sizeof(uint64_t) * p.glwe_len());
    uint64_t *body = glwe + (size_t)p.k * N;
    for (int j = 0; j < N; j++) {
        const int src = (j + half) % N;  // slice::rotate_left(half)
        body[j] = (src < box ? (f0 & 1) : (f1 & 1)) << 62;
    }
}

void generate_lut_without_padding(int N, const uint64_t *f_table, uint64_t *out) {
    const int size = std::max(N, 256);
    for (int i = 0; i < size; i++) out[i] = (f_table[i & 255] & 255) << 56;
}

uint64_t ClientKey::phase(const uint64_t *ct) const {
    const int K = p.K();
    uint64_t s = 0;
    for (int i = 0; i < K; i++) s += ct[i] * glwe_sk[i];
    return ct[K] - s;
}

void generate_client_key(const Params &p, const uint8_t seed[32], ClientKey &ck) {
    const int n = p.n, K = p.K();
    ck.p = p;
    std::memcpy(ck.seed.data(), seed, 32);
    ck.lwe_sk.assign(n, 0);
    ck.glwe_sk.assign(K, 0);
    {
        ChaChaStream s1(seed, LWE_SK, 0), s2(seed, GLWE_SK, 0);
        // one keystream byte per key bit (bit = byte & 1)
        std::vector<uint8_t> bytes((size_t)std::max(n, K) + 64);
        for (size_t o = 0; o < (size_t)n; o += 8) {
            uint64_t w = s1.next_u64();
            std::memcpy(&bytes[o], &w, 8);
        }
        for (int i = 0; i < n; i++) ck.lwe_sk[i] = bytes[i] & 1;
        for (size_t o = 0; o < (size_t)K; o += 8) {
            uint64_t w = s2.next_u64();
            std::memcpy(&bytes[o], &w, 8);
        }
        for (int i = 0; i < K; i++) ck.glwe_sk[i] = bytes[i] & 1;
    }
}

void generate_keys(const Params &p, const uint8_t seed[32], int threads, ClientKey &ck,
                   ServerKeyRaw &sk) {
    const int n = p.n, k = p.k, N = p.N, K = p.K();
    generate_client_key(p, seed, ck);
    sk.p = p;
    sk.ksk.assign(p.ksk_len(), 0);
    sk.bsk.assign(p.bsk_len(), 0);
    sk.pfpksk.assign(p.pfpksk_len(), 0);
    const size_t glwe = p.glwe_len();
    const uint64_t *S = ck.glwe_sk.data();

    // KSK (lwe_keyswitch_key_generation): row (i, l) = LWE_small(s_big[i] * 2^(64 - ks_b*l))
    parallel_for((size_t)K * p.ks_l, threads, [&](size_t c) {
        const size_t i = c / p.ks_l;
        const int l = (int)(c % p.ks_l) + 1;
        lwe_encrypt(seed, KSK, c, ck.lwe_sk.data(), n, S[i] << (64 - p.ks_b * l), p.lwe_std,
                    sk.ksk.data() + c * p.small_len());
    });
    // BSK (encrypt_constant_ggsw_ciphertext of s_i): row r<k plaintext = -s_i*D_l*S_r,
    // row k plaintext = s_i*D_l (constant), D_l = 2^(64 - pbs_b*l)
    parallel_for((size_t)n * p.pbs_l * (k + 1), threads, [&](size_t c) {
        std::vector<uint64_t> msg(N, 0);
        const size_t i = c / ((size_t)p.pbs_l * (k + 1));
        const int l = (int)((c / (k + 1)) % p.pbs_l) + 1;
        const int r = (int)(c % (k + 1));
        const uint64_t factor = (0 - ck.lwe_sk[i]) << (64 - p.pbs_b * l);
        if (r < k)
            for (int j = 0; j < N; j++) msg[j] = S[(size_t)r * N + j] * factor;
        else
            msg[0] = 0 - factor;
        glwe_encrypt(seed, BSK, c, S, k, N, msg.data(), p.glwe_std, sk.bsk.data() + c * glwe);
    });
    if (p.model == 2) {
        // shortint_1bit: lwe_packing_keyswitch_key_generation (shortint_1bit.rs:176-186): input key
        // element i, level l: GLWE encryption of the constant polynomial s_i * 2^(64 - pfks_b*l)
        parallel_for((size_t)n * p.pfks_l, threads, [&](size_t c) {
            std::vector<uint64_t> msg(N, 0);
            const size_t i = c / p.pfks_l;
            const int l = (int)(c % p.pfks_l) + 1;
            msg[0] = ck.lwe_sk[i] << (64 - p.pfks_b * l);
            glwe_encrypt(seed, PFPKSK, c, S, k, N, msg.data(), p.pfks_std, sk.pfpksk.data() + c * glwe);
        });
        return;
    }
    // PFPKSK list (circuit_bootstrap_lwe_pfpksk_list, f(x) = -x): key q, input i (s_K = -1),
    // level l: plaintext P_q * (-s_i) * 2^(64 - pfks_b*l), P_q = S_q (q<k) or the constant -1.
    parallel_for((size_t)(k + 1) * (K + 1) * p.pfks_l, threads, [&](size_t c) {
        std::vector<uint64_t> msg(N, 0);
        const size_t q = c / ((size_t)(K + 1) * p.pfks_l);
        const size_t i = (c / p.pfks_l) % (K + 1);
        const int l = (int)(c % p.pfks_l) + 1;
        const uint64_t s = i < (size_t)K ? S[i] : ~0ull;
        const uint64_t f = (0 - s) << (64 - p.pfks_b * l);
        if (q < (size_t)k)
            for (int j = 0; j < N; j++) msg[j] = S[q * N + j] * f;
        else
            msg[0] = 0 - f;
        glwe_encrypt(seed, PFPKSK, c, S, k, N, msg.data(), p.pfks_std, sk.pfpksk.data() + c * glwe);
    });
}

size_t lut_small_len(int N, int input_bits) {
    int logN = 0;
    while ((1 << logN) < N) logN++;
    const int tree = input_bits > logN ? input_bits - logN : 0;
    return (size_t)N << tree;
}

void generate_lut(int N, int input_bits, int output_bits, const uint64_t *f_table, uint64_t *out) {
    const size_t small = lut_small_len(N, input_bits);
    std::memset(out, 0, sizeof(uint64_t) * small * output_bits);
    for (int j = 0; j < output_bits; j++)
        for (size_t v = 0; v < ((size_t)1 << input_bits); v++)
            out[(size_t)j * small + v] = encode_bit((f_table[v] >> (output_bits - 1 - j)) & 1);
}

namespace {
// cos/sin(2*pi*num/den) with exact quadrant symmetry (FFT table spec)
void sincos_2pi(long num, long den, double &c, double &s) {
    num %= den;
    if (num < 0) num += den;
    const long q = (4 * num) / den;
    const long r = 4 * num - q * den;
    double c0, s0;
    if (2 * r <= den) {
        const double a = (kPi * (double)r) / (2.0 * (double)den);
        c0 = std::cos(a);
        s0 = std::sin(a);
    } else {
        const double a = (kPi * (double)(den - r)) / (2.0 * (double)den);
        c0 = std::sin(a);
        s0 = std::cos(a);
    }
    switch (q) {
    case 0: c = c0; s = s0; break;
    case 1: c = -s0; s = c0; break;
    case 2: c = -c0; s = -s0; break;
    default: c = s0; s = -c0; break;
    }
}
}  // namespace

// The blind rotation's fused-twiddle transform constants (lf512.hpp layout; the oracle's or_lf_plan_build
// computes the same values with the same sincos): per fused stage (cos, tan) of g^2 and of g, g = e^{2 pi i
// num / 1024}
std::vector<double> make_lf512_table() {
    std::vector<double> t(1700, 0.0);
    auto ct = [&](long num, double *o) {
        double c, s;
        sincos_2pi(num, 1024, c, s);
        o[0] = c;
        o[1] = s / c;
    };
    auto k4 = [&](int off, int n, int idx, long num) {  // chunk-major [2][n][2]
        ct(2 * num, &t[off + 2 * idx]);
        ct(num, &t[off + 2 * (n + idx)]);
    };
    for (int k = 0; k < 4; k++) {
        k4(0, 4, k, 16 - 64 * k);    // FA2
        k4(336, 4, k, 1 + 64 * k);   // IB2
    }
    for (int a = 0; a < 16; a++) {
        k4(16, 16, a, 4 - 16 * a);    // FB1
        k4(352, 16, a, 4 + 16 * a);   // IA1
        for (int l = 0; l < 4; l++) {
            k4(80, 64, a + 16 * l, 1 - 4 * a - 64 * l);   // FB2, entry = lane (kappa, l1)
            k4(416, 64, a + 16 * l, 1 + 4 * a + 64 * l);  // IA2, entry = lane (u, m1)
        }
    }
    t[672] = 1.0 / std::sqrt(2.0);
    ct(64, &t[673]);
    for (int j = 0; j < 256; j++) {
        double c, s;
        sincos_2pi(j, 1024, c, s);
        t[676 + 2 * j] = c;
        t[676 + 2 * j + 1] = -s;
        sincos_2pi(-((j >> 4) + (j & 3)), 1024, c, s);
        t[1188 + 2 * j] = c;
        t[1188 + 2 * j + 1] = s;
    }
    return t;
}

// ... for N = 1024 (lf1k.hpp layout; the oracle's or_lf1k_plan_build): angles 2 pi num / 2048, a fused DFT8
// of ratio g = (cos, tan) of g^4, g^2, g W8^-+k1 as 6 chunks of 2 doubles, chunk-major per table
std::vector<double> make_lf1k_table() {
    std::vector<double> t(3788, 0.0);
    auto ct = [&](long num, double *o) {
        double c, s;
        sincos_2pi(num, 2048, c, s);
        o[0] = c;
        o[1] = s / c;
    };
    auto k8 = [&](int off, int n, int idx, long num, bool inv) {
        double e[12];
        ct(4 * num, &e[0]);
        ct(2 * num, &e[2]);
        for (int k1 = 0; k1 < 4; k1++) ct(num + (inv ? 256 : -256) * k1, &e[4 + 2 * k1]);
        for (int q = 0; q < 6; q++) {
            t[off + 2 * (q * n + idx)] = e[2 * q];
            t[off + 2 * (q * n + idx) + 1] = e[2 * q + 1];
        }
    };
    t[0] = 1.0 / std::sqrt(2.0);
    ct(128, &t[1]);
    for (int k1 = 0; k1 < 4; k1++) ct(64 - 256 * k1, &t[4 + 2 * k1]);
    for (int g = 0; g < 8; g++) {
        k8(12, 8, g, 8 - 32 * g, false);   // F1
        k8(876, 8, g, 1 + 32 * g, true);   // I1
    }
    for (int l = 0; l < 64; l++) {
        k8(108, 64, l, 1 - 4 * (l >> 3) - 32 * (l & 7), false);  // F2
        k8(972, 64, l, 1 + 4 * l, true);                          // I0
    }
    for (int j = 0; j < 512; j++) {
        double c, s;
        sincos_2pi(j, 2048, c, s);
        t[1740 + 2 * j] = c;
        t[1740 + 2 * j + 1] = -s;
        sincos_2pi(-((j >> 6) + ((j >> 3) & 7)), 2048, c, s);
        t[2764 + 2 * j] = c;
        t[2764 + 2 * j + 1] = s;
    }
    return t;
}

FftTables make_fft_tables(int N) {
    FftTables t;
    t.N = N;
    t.M = N / 2;
    t.twist.resize(2 * t.M);
    t.untwist.resize(2 * t.M);
    t.w.resize(2 * t.M);
    for (int j = 0; j < t.M; j++) {
        double c, s;
        sincos_2pi(j, 2L * N, c, s);
        t.twist[2 * j] = c;
        t.twist[2 * j + 1] = s;
        t.untwist[2 * j] = c / (double)t.M;
        t.untwist[2 * j + 1] = -s / (double)t.M;
        sincos_2pi(j, t.M, c, s);
        t.w[2 * j] = c;
        t.w[2 * j + 1] = -s;
    }
    return t;
}

}  // namespace tae
