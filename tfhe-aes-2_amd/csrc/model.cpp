// Host-side model mirror: noise bookkeeping, circuit_bootstrap, AES round driver, key schedule.
// See model.hpp for the reference mapping.
#include "model.hpp"

#include <algorithm>
#include <array>
#include <cstring>

#include "aes.hpp"
#include "cplx.hpp"
#include "../../include/tfhe_aes_gpu.h"

namespace tae {

// ---------------------------------------------------------------------------------------------
// AES constants (src/aes_128.rs)
// ---------------------------------------------------------------------------------------------
const uint8_t kSbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76, 0xca, 0x82,
    0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0, 0xb7, 0xfd, 0x93, 0x26,
    0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15, 0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96,
    0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75, 0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0,
    0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84, 0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb,
    0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf, 0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f,
    0x50, 0x3c, 0x9f, 0xa8, 0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff,
    0xf3, 0xd2, 0xcd, 0x0c, 0x13, 0xec, 0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73,
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb, 0xe0, 0x32,
    0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79, 0xe7, 0xc8, 0x37, 0x6d,
    0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08, 0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6,
    0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a, 0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e,
    0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e, 0xe1, 0xf8, 0x98, 0x11, 0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e,
    0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf, 0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f,
    0xb0, 0x54, 0xbb, 0x16};
const uint8_t kRcon[11] = {0x00, 0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1B, 0x36};

void gf_256_mul_bit_terms(uint8_t b, int terms[8][8]) {
    int a[8][8] = {}, res[8][8] = {};
    for (int i = 0; i < 8; i++) a[i][i] = 1;
    for (int it = 0; it < 8; it++) {
        if (b & 1)
            for (int o = 0; o < 8; o++)
                for (int i = 0; i < 8; i++) res[o][i] += a[o][i];
        // Byte::shl_assign_1 (data_model.rs:45-49): bit 0 leaves, the rest rotate left, a trivial
        // zero enters at bit 7; the leaving bit is XORed into bits 3, 4, 6, 7
        int red[8];
        for (int i = 0; i < 8; i++) red[i] = a[0][i];
        for (int o = 0; o < 7; o++)
            for (int i = 0; i < 8; i++) a[o][i] = a[o + 1][i];
        for (int i = 0; i < 8; i++) a[7][i] = 0;
        for (int tap : {3, 4, 6, 7})
            for (int i = 0; i < 8; i++) a[tap][i] += red[i];
        b >>= 1;
    }
    for (int o = 0; o < 8; o++)
        for (int i = 0; i < 8; i++) terms[o][i] = res[o][i];
}

void mix_column_terms(int terms[32][32]) {
    int g[4][8][8];
    for (int m = 1; m <= 3; m++) gf_256_mul_bit_terms((uint8_t)m, g[m]);
    for (int o = 0; o < 32; o++)
        for (int i = 0; i < 32; i++) terms[o][i] = 0;
    for (int r = 0; r < 4; r++)
        for (int o = 0; o < 8; o++)
            for (int x = 0; x < 8; x++) {
                terms[8 * r + o][8 * r + x] += g[2][o][x];
                terms[8 * r + o][8 * ((r + 3) % 4) + x] += g[1][o][x];
                terms[8 * r + o][8 * ((r + 2) % 4) + x] += g[1][o][x];
                terms[8 * r + o][8 * ((r + 1) % 4) + x] += g[3][o][x];
            }
}

uint8_t gf_256_mul(uint8_t a, uint8_t b) {
    uint8_t res = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) res ^= a;
        const uint8_t high_bit = a & 0x80;
        a = (uint8_t)(a << 1);
        if (high_bit != 0x80) a ^= 0x1b;  // sic: aes_128.rs:50
        b >>= 1;
    }
    return res;
}

void plain_key_schedule(const uint8_t key[16], uint8_t rk[176]) {
    std::memcpy(rk, key, 16);
    for (int i = 4; i < 44; i++) {
        uint8_t t[4];
        std::memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 4 == 0) {
            const uint8_t first = t[0];
            t[0] = (uint8_t)(kSbox[t[1]] ^ kRcon[i / 4]);
            t[1] = kSbox[t[2]];
            t[2] = kSbox[t[3]];
            t[3] = kSbox[first];
        }
        for (int j = 0; j < 4; j++) rk[4 * i + j] = rk[4 * (i - 4) + j] ^ t[j];
    }
}

// ---------------------------------------------------------------------------------------------
// Noise bookkeeping
// ---------------------------------------------------------------------------------------------
static std::atomic<uint64_t> g_ct_counter{0};
uint64_t next_ct_id() { return g_ct_counter.fetch_add(1); }

void NoiseLevel::add_assign(const NoiseLevel &rhs, uint64_t max_noise_sq) {
    // assert!(components ∩ rhs.components == ∅, "noise components not independent")
    auto a = components.cbegin();
    auto b = rhs.components.cbegin();
    while (a != components.cend() && b != rhs.components.cend()) {
        if (*a == *b) throw ModelError{TAE_E_INDEP, "noise components not independent"};
        if (*a < *b)
            ++a;
        else
            ++b;
    }
    std::vector<uint64_t> merged;
    merged.reserve(components.size() + rhs.components.size());
    std::merge(components.begin(), components.end(), rhs.components.begin(), rhs.components.end(),
               std::back_inserter(merged));
    components.swap(merged);
    noise_level_squared += rhs.noise_level_squared;
    if (noise_level_squared > max_noise_sq)  // MaxNoiseLevel::validate(..).unwrap()
        throw ModelError{TAE_E_NOISE, "NoiseTooBig { noise_level: " + std::to_string(noise_level_squared) +
                                          ", max_noise_level: " + std::to_string(max_noise_sq) + " }"};
}

void BitCt::xor_assign(const BitCt &rhs) {
    if (rhs.ct.size() != ct.size()) throw ModelError{TAE_E_ARG, "ciphertext size mismatch"};
    for (size_t i = 0; i < ct.size(); i++) ct[i] += rhs.ct[i];  // lwe_ciphertext_add_assign
    noise.add_assign(rhs.noise, max_noise_sq);
}

BitCt Context::trivial(uint64_t bit) const {
    if (bit > 1) throw ModelError{TAE_E_ARG, "cleartext out of bounds: " + std::to_string(bit)};
    BitCt b;
    b.ct.assign(bit_len(), 0);
    b.ct.back() = params().model == 2 ? bit << 62 : encode_bit(bit);  // shortint create_trivial: m * delta
    b.noise = NoiseLevel::trivial();
    b.max_noise_sq = params().max_noise_sq;
    return b;
}

BitCt Context::wrap(std::vector<uint64_t> ct, uint64_t noise_level_squared) const {
    BitCt b;
    b.ct = std::move(ct);
    // 8-bit model: shortint NoiseLevel (additive, no component ids; shortint_woppbs_8bit.rs:94-163);
    // shortint_1bit: XOR is unchecked_add (shortint_1bit.rs:103-116), nothing is tracked
    b.noise = params().model == 8   ? NoiseLevel{noise_level_squared, {}}
              : params().model == 2 ? NoiseLevel{}
                                    : NoiseLevel::with_noise_level(noise_level_squared, next_ct_id());
    b.max_noise_sq = params().max_noise_sq;
    return b;
}

Lut Context::generate_lookup_table(int input_bits, int output_bits, const uint64_t *f_values) const {
    if (!(input_bits > 0 && input_bits <= 16)) throw ModelError{TAE_E_PARAM, "input_bits must be in 1..=16"};
    if (!(output_bits > 0 && output_bits <= 64)) throw ModelError{TAE_E_PARAM, "output_bits must be in 1..=64"};
    Lut l;
    l.input_bits = input_bits;
    l.output_bits = output_bits;
    if (params().model == 8) {
        // 8-bit model: FheContext::generate_lookup_table (shortint_woppbs_8bit.rs:262-265) is a byte ->
        // byte map through WopbsKey::generate_lut_without_padding (one polynomial, 2^56 scale)
        if (input_bits != 8 || output_bits != 8)
            throw ModelError{TAE_E_PARAM, "the 8-bit model's lookup tables map 8 bits to 8 bits"};
        l.small_len = (size_t)std::max(params().N, 256);
        l.data.assign(l.small_len, 0);
        generate_lut_without_padding(params().N, f_values, l.data.data());
        return l;
    }
    l.small_len = lut_small_len(params().N, input_bits);
    l.data.assign(l.small_len * output_bits, 0);
    generate_lut(params().N, input_bits, output_bits, f_values, l.data.data());
    return l;
}

namespace {
struct DevBuf {
    void *p = nullptr;
    explicit DevBuf(size_t bytes) { hip_check(hipMalloc(&p, std::max<size_t>(bytes, 16)), "hipMalloc"); }
    ~DevBuf() {
        if (p) hipFree(p);
    }
    template <class T>
    T *as() const {
        return static_cast<T *>(p);
    }
};
}  // namespace

// Run fn(d_in, d_out, d_lut) on the engine stream with host staging unless device_mem.
template <class F>
void Context::run8(const uint64_t *in, size_t in_len, uint64_t *out, size_t out_len, bool device_mem, F fn,
                   const Lut *lut) {
    std::lock_guard<std::mutex> g(mu_);
    hip_check(hipSetDevice(engine_->device()), "hipSetDevice");
    std::unique_ptr<DevBuf> d_lut;
    if (lut) {
        d_lut = std::make_unique<DevBuf>(lut->data.size() * 8);
        hip_check(hipMemcpyAsync(d_lut->p, lut->data.data(), lut->data.size() * 8, hipMemcpyHostToDevice,
                                 engine_->stream()),
                  "lut upload");
    }
    const uint64_t *dl = d_lut ? d_lut->as<uint64_t>() : nullptr;
    if (device_mem) {
        engine_->order_after_caller();
        fn(in, out, dl);
        engine_->synchronize();
        return;
    }
    DevBuf d_in(in_len * 8), d_out(out_len * 8);
    hip_check(hipMemcpyAsync(d_in.p, in, in_len * 8, hipMemcpyHostToDevice, engine_->stream()), "upload");
    fn(d_in.as<uint64_t>(), d_out.as<uint64_t>(), dl);
    hip_check(hipMemcpyAsync(out, d_out.p, out_len * 8, hipMemcpyDeviceToHost, engine_->stream()), "download");
    engine_->synchronize();
}

void Context::bootstrap_from_bits_raw(const uint64_t *bits, size_t groups, const Lut &lut, uint64_t *out,
                                      bool device_mem) {
    if (params().model != 8) throw ModelError{TAE_E_PARAM, "bootstrap_from_bits belongs to the 8-bit model"};
    if (lut.input_bits != 8) throw ModelError{TAE_E_ARG, "bootstrap_from_bits needs an 8-bit LUT"};
    run8(bits, groups * 8 * bit_len(), out, groups * params().big_len(), device_mem,
         [&](const uint64_t *in, uint64_t *o, const uint64_t *d_lut) { engine_->cbs_vp(in, groups, 8, d_lut, 1, o); },
         &lut);
}

void Context::extract_bits_raw(const uint64_t *ints, size_t groups, uint64_t *out, bool device_mem) {
    if (params().model != 8) throw ModelError{TAE_E_PARAM, "extract_bits_from_ciphertext belongs to the 8-bit model"};
    run8(ints, groups * params().big_len(), out, groups * 8 * bit_len(), device_mem,
         [&](const uint64_t *in, uint64_t *o, const uint64_t *) { engine_->extract_bits(in, groups, 56, 8, o); },
         nullptr);
}

void Context::circuit_bootstrap_raw(const uint64_t *bits, size_t groups, int n_in, const Lut &lut, uint64_t *out,
                                    bool device_mem) {
    if (n_in != lut.input_bits) throw ModelError{TAE_E_ARG, "number of input bits does not match the LUT"};
    if (params().model == 8) {
        // Byte::bootstrap_with_lut (fhe_impls/shortint_woppbs_8bit.rs:37-42): bits [G][8][n+1] -> [G][8][n+1]
        run8(bits, groups * 8 * bit_len(), out, groups * 8 * bit_len(), device_mem,
             [&](const uint64_t *in, uint64_t *o, const uint64_t *d_lut) { engine_->bootstrap_bytes8(in, groups, d_lut, o); },
             &lut);
        return;
    }
    std::lock_guard<std::mutex> g(mu_);
    const size_t L = params().big_len();
    hip_check(hipSetDevice(engine_->device()), "hipSetDevice");
    DevBuf d_lut(lut.data.size() * 8);
    hip_check(hipMemcpyAsync(d_lut.p, lut.data.data(), lut.data.size() * 8, hipMemcpyHostToDevice,
                             engine_->stream()),
              "lut upload");
    if (device_mem) {
        engine_->order_after_caller();
        engine_->circuit_bootstrap(bits, groups, n_in, d_lut.as<uint64_t>(), lut.output_bits, out);
        engine_->synchronize();
        return;
    }
    DevBuf d_in(groups * n_in * L * 8), d_out(groups * lut.output_bits * L * 8);
    hip_check(hipMemcpyAsync(d_in.p, bits, groups * n_in * L * 8, hipMemcpyHostToDevice, engine_->stream()), "upload");
    engine_->circuit_bootstrap(d_in.as<uint64_t>(), groups, n_in, d_lut.as<uint64_t>(), lut.output_bits,
                               d_out.as<uint64_t>());
    hip_check(hipMemcpyAsync(out, d_out.p, groups * lut.output_bits * L * 8, hipMemcpyDeviceToHost, engine_->stream()),
              "download");
    engine_->synchronize();
}

// FheContext::circuit_bootstrap (shortint_woppbs_1bit.rs:292-336)
std::vector<BitCt> Context::circuit_bootstrap(const std::vector<const BitCt *> &bits, const Lut &lut) {
    const size_t L = bit_len();
    for (const BitCt *b : bits)
        if (b->ct.size() != L) throw ModelError{TAE_E_ARG, "ciphertext size mismatch"};
    if (params().model == 8) {
        // Byte::bootstrap_with_lut: extract_bits outputs are BitCt::new (NOMINAL noise)
        if (bits.size() != 8) throw ModelError{TAE_E_ARG, "the 8-bit model bootstraps whole bytes"};
        std::vector<uint64_t> in8(8 * L), out8(8 * L);
        for (size_t b = 0; b < 8; b++) std::memcpy(&in8[b * L], bits[b]->ct.data(), L * 8);
        circuit_bootstrap_raw(in8.data(), 1, 8, lut, out8.data(), false);
        std::vector<BitCt> res;
        for (int j = 0; j < 8; j++)
            res.push_back(wrap(std::vector<uint64_t>(out8.begin() + j * L, out8.begin() + (j + 1) * L), 1));
        return res;
    }
    std::vector<uint64_t> in(bits.size() * L), out((size_t)lut.output_bits * L);
    for (size_t b = 0; b < bits.size(); b++) std::memcpy(&in[b * L], bits[b]->ct.data(), L * 8);
    circuit_bootstrap_raw(in.data(), 1, (int)bits.size(), lut, out.data(), false);
    // Lemma 3.2 of eprint 2017/430: output noise^2 = NOMINAL * input_bit_count (:322-325)
    std::vector<BitCt> res;
    for (int j = 0; j < lut.output_bits; j++)
        res.push_back(wrap(std::vector<uint64_t>(out.begin() + j * L, out.begin() + (j + 1) * L), bits.size()));
    return res;
}

// ---------------------------------------------------------------------------------------------
// AES (fhe_sbox_gal_mul_pbs.rs)
// ---------------------------------------------------------------------------------------------
// Metadata-only replay of encrypt_block_for_rounds for ONE block: rk [44*32], block [128].
std::vector<NoiseLevel> aes_noise_schedule(const std::vector<NoiseLevel> &rk, const std::vector<NoiseLevel> &block,
                                           int rounds, uint64_t max) {
    auto key_bit = [&](int word, int byte, int bit) -> const NoiseLevel & { return rk[(word * 4 + byte) * 8 + bit]; };
    std::vector<NoiseLevel> st = block;  // index (4*col + row)*8 + bit
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++)
            for (int b = 0; b < 8; b++) st[(4 * c + r) * 8 + b].add_assign(key_bit(c, r, b), max);
    auto cbs_outputs = [&](int n_out) {
        std::vector<NoiseLevel> o((size_t)16 * n_out);
        for (auto &x : o) x = NoiseLevel::with_noise_level(8, next_ct_id());
        return o;
    };
    for (int round = 1; round < rounds; round++) {
        std::vector<NoiseLevel> muls = cbs_outputs(24);  // [byte][24]
        auto src = [&](int rr, int c, int m, int b) -> const NoiseLevel & {
            return muls[(4 * ((c + rr) % 4) + rr) * 24 + 8 * m + b];
        };
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++)
                for (int b = 0; b < 8; b++) {
                    NoiseLevel v = src(r, c, 1, b);
                    v.add_assign(src((r + 3) % 4, c, 0, b), max);
                    v.add_assign(src((r + 2) % 4, c, 0, b), max);
                    v.add_assign(src((r + 1) % 4, c, 2, b), max);
                    v.add_assign(key_bit(4 * round + c, r, b), max);
                    st[(4 * c + r) * 8 + b] = std::move(v);
                }
    }
    std::vector<NoiseLevel> sb = cbs_outputs(8);
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++)
            for (int b = 0; b < 8; b++) {
                NoiseLevel v = sb[(4 * ((c + r) % 4) + r) * 8 + b];
                v.add_assign(key_bit(40 + c, r, b), max);
                st[(4 * c + r) * 8 + b] = std::move(v);
            }
    return st;
}

// fhe_sbox_pbs::encrypt_block_for_rounds (:75-121) on metadata: SubBytes = bootstrap_with_lut
// (outputs NOMINAL), MixColumns adds the network's terms, ARK the key bit.
std::vector<NoiseLevel> aes8_noise_schedule(const std::vector<NoiseLevel> &rk, const std::vector<NoiseLevel> &block,
                                            int rounds, uint64_t max) {
    int terms[32][32];
    mix_column_terms(terms);
    auto key_bit = [&](int word, int byte, int bit) -> const NoiseLevel & { return rk[(word * 4 + byte) * 8 + bit]; };
    std::vector<NoiseLevel> st = block;
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++)
            for (int b = 0; b < 8; b++) st[(4 * c + r) * 8 + b].add_assign(key_bit(c, r, b), max);
    const NoiseLevel nominal{1, {}};
    for (int round = 1; round <= rounds; round++) {
        const bool last = round == rounds;
        for (int c = 0; c < 4; c++)
            for (int o = 0; o < 32; o++) {
                NoiseLevel v{0, {}};
                if (last) {
                    v = nominal;
                } else {
                    for (int i = 0; i < 32; i++)
                        for (int t = 0; t < terms[o][i]; t++) v.add_assign(nominal, max);
                }
                v.add_assign(key_bit(last ? 40 + c : 4 * round + c, o / 8, o % 8), max);
                st[(4 * c + o / 8) * 8 + o % 8] = std::move(v);
            }
    }
    return st;
}

// fhe_sbox_pbs::gf_256_mul (:33-53) on the 1-bit model's noise metadata, XOR by XOR (MSB-first bits,
// Byte::shl_assign_1 = data_model.rs:45-49).  The loop keeps shifting and reducing the multiplicand
// after the last multiplier bit: from the fifth iteration on, the leaving bit already carries the
// component of the original bit 0 that the reduction XORs into bits 3, 4, 6, 7 again, so every call
// raises "noise components not independent" on non-trivial inputs.
static std::array<NoiseLevel, 8> gf_256_mul_noise(const std::array<NoiseLevel, 8> &x, uint8_t b, uint64_t max) {
    std::array<NoiseLevel, 8> a = x, res;  // res = Byte::trivial(ctx, 0)
    for (int it = 0; it < 8; it++) {
        if (b & 1)
            for (int i = 0; i < 8; i++) res[i].add_assign(a[i], max);
        const NoiseLevel reduce_x8 = a[0];
        for (int i = 0; i < 7; i++) a[i] = a[i + 1];
        a[7] = NoiseLevel::trivial();
        for (int tap : {3, 4, 6, 7}) a[tap].add_assign(reduce_x8, max);
        b >>= 1;
    }
    return res;
}

// fhe_sbox_pbs::encrypt_block_for_rounds (:75-121) over the 1-bit model (ShortintWoppbs1BitSboxPbsAesEncrypt,
// fhe_impls/shortint_woppbs_1bit.rs:47-81) on metadata: SubBytes = Byte::sbox_substitute (one 8 -> 8
// circuit bootstrap, outputs noise^2 = 8 with fresh ids), ShiftRows, MixColumns = the gf_256_mul network
// (:56-73), AddRoundKey.  MixColumns always raises TAE_E_INDEP (gf_256_mul_noise), which is why the
// reference #[ignore]s test_light / test_full of this combination (:160-176): only a 1-round run passes.
std::vector<NoiseLevel> sbox_pbs_noise_schedule(const std::vector<NoiseLevel> &rk, const std::vector<NoiseLevel> &block,
                                                int rounds, uint64_t max) {
    auto key_bit = [&](int word, int byte, int bit) -> const NoiseLevel & { return rk[(word * 4 + byte) * 8 + bit]; };
    std::vector<NoiseLevel> st = block;  // index (4*col + row)*8 + bit (State::from_array)
    auto xor_state = [&](int w0) {
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++)
                for (int b = 0; b < 8; b++) st[(4 * c + r) * 8 + b].add_assign(key_bit(w0 + c, r, b), max);
    };
    auto sub_bytes_shift_rows = [&] {
        std::vector<NoiseLevel> sb(128);
        for (auto &x : sb) x = NoiseLevel::with_noise_level(8, next_ct_id());
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++)
                for (int b = 0; b < 8; b++) st[(4 * c + r) * 8 + b] = sb[(4 * ((c + r) % 4) + r) * 8 + b];
    };
    xor_state(0);
    for (int round = 1; round < rounds; round++) {
        sub_bytes_shift_rows();
        std::vector<NoiseLevel> mixed(128);
        for (int c = 0; c < 4; c++) {
            std::array<NoiseLevel, 8> col[4];
            for (int r = 0; r < 4; r++)
                for (int b = 0; b < 8; b++) col[r][b] = st[(4 * c + r) * 8 + b];
            for (int i = 0; i < 4; i++) {
                std::array<NoiseLevel, 8> v = gf_256_mul_noise(col[i], 2, max);
                for (const auto &[src, m] : {std::pair<int, uint8_t>{(i + 3) % 4, 1}, {(i + 2) % 4, 1}, {(i + 1) % 4, 3}}) {
                    const std::array<NoiseLevel, 8> t = gf_256_mul_noise(col[src], m, max);
                    for (int b = 0; b < 8; b++) v[b].add_assign(t[b], max);
                }
                for (int b = 0; b < 8; b++) mixed[(4 * c + i) * 8 + b] = v[b];
            }
        }
        st.swap(mixed);
        xor_state(4 * round);
    }
    sub_bytes_shift_rows();
    xor_state(40);
    return st;
}

std::vector<NoiseLevel> Context::block_noise_schedule(AesDriver driver, const std::vector<NoiseLevel> &rk,
                                                      const std::vector<NoiseLevel> &block, int rounds) const {
    const uint64_t max = params().max_noise_sq;
    // shortint_1bit: XOR is shortint unchecked_add (shortint_1bit.rs:103-116) and SubBytes a fresh
    // bootstrap: nothing is validated, so the round function cannot fail on noise bookkeeping (its
    // decryption failures are the reference's #[ignore]d "too big noise accumulation")
    if (params().model == 2) return std::vector<NoiseLevel>(128);
    if (params().model == 8) return aes8_noise_schedule(rk, block, rounds, max);
    return driver == AesDriver::SboxPbs ? sbox_pbs_noise_schedule(rk, block, rounds, max)
                                        : aes_noise_schedule(rk, block, rounds, max);
}

// The device round functions.  1-bit model: Engine::aes_encrypt_blocks (fhe_sbox_gal_mul_pbs rounds, its
// last round = SubBytes 8 -> 8, ShiftRows, AddRoundKey).  The 1-bit fhe_sbox_pbs driver only gets here
// with rounds == 1 (its schedule raises at the first MixColumns), where it is exactly that last round.
void Context::run_aes_blocks(AesDriver driver, const uint64_t *d_rk, const uint64_t *d_in, size_t n_blocks, int rounds,
                             uint64_t *d_out) {
    if (params().model == 8) {
        engine_->aes8_encrypt_blocks(d_rk, d_in, n_blocks, rounds, d_out);
        return;
    }
    if (params().model == 2) {
        engine_->s1_aes_encrypt_blocks(d_rk, d_in, n_blocks, rounds, d_out);
        return;
    }
    if (driver == AesDriver::SboxPbs && rounds != 1)
        throw ModelError{TAE_E_INDEP, "noise components not independent"};
    engine_->aes_encrypt_blocks(d_rk, d_in, n_blocks, rounds, d_out);
}

void Context::aes_encrypt_blocks_raw(const uint64_t *rk, const uint64_t *blocks, size_t n_blocks, int rounds,
                                     uint64_t *out, bool device_mem, AesDriver driver) {
    if (rounds < 1 || rounds > kAesRounds) throw ModelError{TAE_E_PARAM, "rounds must be in 1..=10"};
    {
        // static validation of the fixed noise schedule for fresh inputs (noise^2 = 1, own ids)
        std::vector<NoiseLevel> krk(44 * 32), kbl(128);
        for (auto &x : krk) x = params().model != 1 ? NoiseLevel{1, {}} : NoiseLevel::with_noise_level(1, next_ct_id());
        for (auto &x : kbl) x = params().model != 1 ? NoiseLevel{1, {}} : NoiseLevel::with_noise_level(1, next_ct_id());
        block_noise_schedule(driver, krk, kbl, rounds);
    }
    const size_t S = bit_len();
    std::lock_guard<std::mutex> g(mu_);
    hip_check(hipSetDevice(engine_->device()), "hipSetDevice");
    if (device_mem) {
        engine_->order_after_caller();
        run_aes_blocks(driver, rk, blocks, n_blocks, rounds, out);
        engine_->synchronize();
        return;
    }
    DevBuf d_rk(44 * 32 * S * 8), d_in(n_blocks * 128 * S * 8), d_out(n_blocks * 128 * S * 8);
    hip_check(hipMemcpyAsync(d_rk.p, rk, 44 * 32 * S * 8, hipMemcpyHostToDevice, engine_->stream()), "upload rk");
    hip_check(hipMemcpyAsync(d_in.p, blocks, n_blocks * 128 * S * 8, hipMemcpyHostToDevice, engine_->stream()),
              "upload blocks");
    run_aes_blocks(driver, d_rk.as<uint64_t>(), d_in.as<uint64_t>(), n_blocks, rounds, d_out.as<uint64_t>());
    hip_check(hipMemcpyAsync(out, d_out.p, n_blocks * 128 * S * 8, hipMemcpyDeviceToHost, engine_->stream()),
              "download");
    engine_->synchronize();
}

std::vector<BitCt> Context::aes_encrypt_blocks(const std::vector<const BitCt *> &expanded_key,
                                               const std::vector<const BitCt *> &blocks, size_t n_blocks,
                                               int rounds, AesDriver driver) {
    if (expanded_key.size() != 44 * 32) throw ModelError{TAE_E_ARG, "expanded key must be 44 words (1408 bits)"};
    if (blocks.size() != n_blocks * 128) throw ModelError{TAE_E_ARG, "blocks must be 128 bits each"};
    if (rounds < 1 || rounds > kAesRounds) throw ModelError{TAE_E_PARAM, "rounds must be in 1..=10"};
    const size_t L = bit_len();
    for (const BitCt *b : expanded_key)
        if (b->ct.size() != L) throw ModelError{TAE_E_ARG, "ciphertext size mismatch"};
    for (const BitCt *b : blocks)
        if (b->ct.size() != L) throw ModelError{TAE_E_ARG, "ciphertext size mismatch"};
    std::vector<NoiseLevel> krk(44 * 32);
    for (size_t i = 0; i < krk.size(); i++) krk[i] = expanded_key[i]->noise;
    std::vector<std::vector<NoiseLevel>> out_noise(n_blocks);
    for (size_t blk = 0; blk < n_blocks; blk++) {
        std::vector<NoiseLevel> kb(128);
        for (int i = 0; i < 128; i++) kb[i] = blocks[blk * 128 + i]->noise;
        out_noise[blk] = block_noise_schedule(driver, krk, kb, rounds);
    }
    std::vector<uint64_t> rk(44 * 32 * L), in(n_blocks * 128 * L), out(n_blocks * 128 * L);
    for (size_t i = 0; i < 44 * 32; i++) std::memcpy(&rk[i * L], expanded_key[i]->ct.data(), L * 8);
    for (size_t i = 0; i < n_blocks * 128; i++) std::memcpy(&in[i * L], blocks[i]->ct.data(), L * 8);
    {
        std::lock_guard<std::mutex> g(mu_);
        hip_check(hipSetDevice(engine_->device()), "hipSetDevice");
        DevBuf d_rk(rk.size() * 8), d_in(in.size() * 8), d_out(out.size() * 8);
        hip_check(hipMemcpyAsync(d_rk.p, rk.data(), rk.size() * 8, hipMemcpyHostToDevice, engine_->stream()), "up");
        hip_check(hipMemcpyAsync(d_in.p, in.data(), in.size() * 8, hipMemcpyHostToDevice, engine_->stream()), "up");
        run_aes_blocks(driver, d_rk.as<uint64_t>(), d_in.as<uint64_t>(), n_blocks, rounds, d_out.as<uint64_t>());
        hip_check(hipMemcpyAsync(out.data(), d_out.p, out.size() * 8, hipMemcpyDeviceToHost, engine_->stream()), "dn");
        engine_->synchronize();
    }
    std::vector<BitCt> res(n_blocks * 128);
    for (size_t i = 0; i < n_blocks * 128; i++) {
        res[i].ct.assign(out.begin() + i * L, out.begin() + (i + 1) * L);
        res[i].noise = out_noise[i / 128][i % 128];
        res[i].max_noise_sq = params().max_noise_sq;
    }
    return res;
}

// fhe_sbox_gal_mul_pbs::key_schedule (:134-164) with ByteT::{sbox_substitute, bootstrap_assign}
// (fhe_impls/shortint_woppbs_1bit.rs:18-45): words 0..3 = key; word i>=4 from words i-4, i-1
// (SubWord(RotWord) + Rcon when i%4 == 0), then every bit of word i is bootstrapped (identity LUT).
std::vector<BitCt> Context::aes_key_schedule(const std::vector<const BitCt *> &key, AesDriver driver) {
    if (key.size() != 128) throw ModelError{TAE_E_ARG, "key must be 16 bytes (128 bits)"};
    if (params().model != 1 || driver == AesDriver::SboxPbs) return sbox_pbs_key_schedule(key);
    const size_t L = params().big_len();
    std::vector<BitCt> ek(44 * 32);
    for (int i = 0; i < 128; i++) ek[i] = *key[i];
    uint64_t ftab_sbox[256], ftab_id[2] = {0, 1};
    for (int x = 0; x < 256; x++) ftab_sbox[x] = kSbox[x];
    const Lut sbox = generate_lookup_table(8, 8, ftab_sbox);
    const Lut ident = generate_lookup_table(1, 1, ftab_id);
    auto bit_at = [&](int word, int byte, int bit) -> BitCt & { return ek[(word * 4 + byte) * 8 + bit]; };
    std::vector<uint64_t> in, out;
    for (int i = 4; i < 44; i++) {
        std::vector<BitCt> w(32);
        if (i % 4 == 0) {
            // sub_word(rotate_left(ek[i-1], 1)): 4 SBOX circuit bootstraps (one batched call)
            in.assign(4 * 8 * L, 0);
            out.assign(4 * 8 * L, 0);
            for (int byte = 0; byte < 4; byte++)
                for (int b = 0; b < 8; b++)
                    std::memcpy(&in[(byte * 8 + b) * L], bit_at(i - 1, (byte + 1) % 4, b).ct.data(), L * 8);
            circuit_bootstrap_raw(in.data(), 4, 8, sbox, out.data(), false);
            for (int t = 0; t < 32; t++) {
                BitCt s = wrap(std::vector<uint64_t>(out.begin() + t * L, out.begin() + (t + 1) * L), 8);
                BitCt v = ek[(i - 4) * 32 + t];
                v.xor_assign(s);
                w[t] = std::move(v);
            }
            for (int b = 0; b < 8; b++) w[b].xor_assign(trivial((kRcon[i / 4] >> (7 - b)) & 1));
        } else {
            for (int t = 0; t < 32; t++) {
                BitCt v = ek[(i - 4) * 32 + t];
                v.xor_assign(ek[(i - 1) * 32 + t]);
                w[t] = std::move(v);
            }
        }
        // boot_word: identity circuit bootstrap of every bit (32 one-bit groups, one call)
        in.assign(32 * L, 0);
        out.assign(32 * L, 0);
        for (int t = 0; t < 32; t++) std::memcpy(&in[t * L], w[t].ct.data(), L * 8);
        circuit_bootstrap_raw(in.data(), 32, 1, ident, out.data(), false);
        for (int t = 0; t < 32; t++)
            ek[i * 32 + t] = wrap(std::vector<uint64_t>(out.begin() + t * L, out.begin() + (t + 1) * L), 1);
    }
    return ek;
}

// fhe_sbox_pbs::key_schedule (:123-171): sub_word = sbox_substitute of each byte of RotWord(ek[i-1]);
// after every 4th word the four words i-3..i are boot_word-ed.  ByteT per model:
//   8-bit (fhe_impls/shortint_woppbs_8bit.rs:17-42): both are Byte::bootstrap_with_lut (SBOX / identity
//     8 -> 8, outputs NOMINAL);
//   1-bit (fhe_impls/shortint_woppbs_1bit.rs:17-50): sbox_substitute is one 8 -> 8 circuit bootstrap
//     (outputs noise^2 = 8), bootstrap_assign one 1 -> 1 identity circuit bootstrap per bit (noise^2 = 1).
// Every bootstrap of a step goes to the device as one batched call.
std::vector<BitCt> Context::sbox_pbs_key_schedule(const std::vector<const BitCt *> &key) {
    const size_t L = bit_len();
    const bool m8 = params().model == 8;
    for (const BitCt *b : key)
        if (b->ct.size() != L) throw ModelError{TAE_E_ARG, "ciphertext size mismatch"};
    std::vector<BitCt> ek(44 * 32);
    for (int i = 0; i < 128; i++) ek[i] = *key[i];
    uint64_t ftab_sbox[256], ftab_id[256];
    for (int x = 0; x < 256; x++) {
        ftab_sbox[x] = kSbox[x];
        ftab_id[x] = (uint64_t)x;
    }
    const Lut sbox = generate_lookup_table(8, 8, ftab_sbox);
    const Lut ident = m8 ? generate_lookup_table(8, 8, ftab_id) : generate_lookup_table(1, 1, ftab_id);
    if (params().model == 2) {
        // shortint_1bit ByteT (fhe_impls/shortint_1bit.rs:17-50): sbox_substitute = 8 multivariate functions
        // of the byte's bits, bootstrap_assign = one PBS per bit with the identity test vector; outputs
        // are fresh shortint ciphertexts (no bookkeeping: unchecked adds)
        const Engine &e = *engine_;
        auto boot = [&](std::vector<BitCt *> bits, bool sbox) {
            const size_t nbits = bits.size();
            std::vector<uint64_t> in(nbits * L), out(nbits * L);
            for (size_t t = 0; t < nbits; t++) std::memcpy(&in[t * L], bits[t]->ct.data(), L * 8);
            std::lock_guard<std::mutex> g(mu_);
            hip_check(hipSetDevice(engine_->device()), "hipSetDevice");
            DevBuf d_in(in.size() * 8), d_out(out.size() * 8);
            hip_check(hipMemcpyAsync(d_in.p, in.data(), in.size() * 8, hipMemcpyHostToDevice, engine_->stream()), "up");
            if (sbox)
                engine_->s1_multivariate(d_in.as<uint64_t>(), nbits / 8, 8, e.s1_sbox_tvs(), 8, d_out.as<uint64_t>());
            else
                engine_->s1_bootstrap(d_in.as<uint64_t>(), e.s1_identity_tv(), 1, d_out.as<uint64_t>(), nbits);
            hip_check(hipMemcpyAsync(out.data(), d_out.p, out.size() * 8, hipMemcpyDeviceToHost, engine_->stream()), "dn");
            engine_->synchronize();
            for (size_t t = 0; t < nbits; t++) *bits[t] = wrap(std::vector<uint64_t>(out.begin() + t * L, out.begin() + (t + 1) * L), 0);
        };
        auto bit_at = [&](int word, int byte, int bit) -> BitCt & { return ek[(word * 4 + byte) * 8 + bit]; };
        for (int i = 4; i < 44; i++) {
            if (i % 4 == 0) {
                std::vector<BitCt> rot(32);
                std::vector<BitCt *> rp(32);
                for (int byte = 0; byte < 4; byte++)
                    for (int b = 0; b < 8; b++) rot[byte * 8 + b] = bit_at(i - 1, (byte + 1) % 4, b);
                for (int t = 0; t < 32; t++) rp[t] = &rot[t];
                boot(rp, true);
                for (int t = 0; t < 32; t++) {
                    BitCt v = ek[(i - 4) * 32 + t];
                    v.xor_assign(rot[t]);
                    ek[i * 32 + t] = std::move(v);
                }
                for (int b = 0; b < 8; b++) ek[i * 32 + b].xor_assign(trivial((kRcon[i / 4] >> (7 - b)) & 1));
            } else {
                for (int t = 0; t < 32; t++) {
                    BitCt v = ek[(i - 4) * 32 + t];
                    v.xor_assign(ek[(i - 1) * 32 + t]);
                    ek[i * 32 + t] = std::move(v);
                }
            }
            if (i % 4 == 3) {
                std::vector<BitCt *> ws(128);
                for (int t = 0; t < 128; t++) ws[t] = &ek[(i - 3) * 32 + t];
                boot(ws, false);
            }
        }
        return ek;
    }
    auto boot = [&](std::vector<BitCt *> bits, const Lut &lut) {  // groups of lut.input_bits, in place
        const int n_in = lut.input_bits;
        const size_t groups = bits.size() / n_in;
        std::vector<uint64_t> in(bits.size() * L), out(bits.size() * L);
        for (size_t t = 0; t < bits.size(); t++) std::memcpy(&in[t * L], bits[t]->ct.data(), L * 8);
        circuit_bootstrap_raw(in.data(), groups, n_in, lut, out.data(), false);
        // noise: shortint NOMINAL (8-bit); NOMINAL * input_bit_count (1-bit, shortint_woppbs_1bit.rs:322-325)
        for (size_t t = 0; t < bits.size(); t++)
            *bits[t] = wrap(std::vector<uint64_t>(out.begin() + t * L, out.begin() + (t + 1) * L), m8 ? 1 : n_in);
    };
    auto bit_at = [&](int word, int byte, int bit) -> BitCt & { return ek[(word * 4 + byte) * 8 + bit]; };
    for (int i = 4; i < 44; i++) {
        if (i % 4 == 0) {
            std::vector<BitCt> rot(32);
            std::vector<BitCt *> rp(32);
            for (int byte = 0; byte < 4; byte++)
                for (int b = 0; b < 8; b++) rot[byte * 8 + b] = bit_at(i - 1, (byte + 1) % 4, b);
            for (int t = 0; t < 32; t++) rp[t] = &rot[t];
            boot(rp, sbox);
            for (int t = 0; t < 32; t++) {
                BitCt v = ek[(i - 4) * 32 + t];
                v.xor_assign(rot[t]);
                ek[i * 32 + t] = std::move(v);
            }
            for (int b = 0; b < 8; b++) ek[i * 32 + b].xor_assign(trivial((kRcon[i / 4] >> (7 - b)) & 1));
        } else {
            for (int t = 0; t < 32; t++) {
                BitCt v = ek[(i - 4) * 32 + t];
                v.xor_assign(ek[(i - 1) * 32 + t]);
                ek[i * 32 + t] = std::move(v);
            }
        }
        if (i % 4 == 3) {
            std::vector<BitCt *> ws(128);
            for (int t = 0; t < 128; t++) ws[t] = &ek[(i - 3) * 32 + t];
            boot(ws, ident);
        }
    }
    return ek;
}

void Context::aes_key_schedule_raw(const uint64_t *key, uint64_t *expanded, bool device_mem, AesDriver driver) {
    const size_t L = bit_len();
    std::vector<uint64_t> hk(128 * L);
    if (device_mem) {
        std::lock_guard<std::mutex> g(mu_);  // the engine (and its device) is shared: same lock as every entry
        engine_->order_after_caller();
        // on the engine stream, which waits for the caller's stream (a plain hipMemcpy runs on the null
        // stream, which does not wait for a non-blocking caller stream)
        hip_check(hipMemcpyAsync(hk.data(), key, hk.size() * 8, hipMemcpyDeviceToHost, engine_->stream()),
                  "download key");
        engine_->synchronize();
    } else {
        std::memcpy(hk.data(), key, hk.size() * 8);
    }
    std::vector<BitCt> kb(128);
    std::vector<const BitCt *> kp(128);
    for (int i = 0; i < 128; i++) {
        kb[i] = wrap(std::vector<uint64_t>(hk.begin() + i * L, hk.begin() + (i + 1) * L), 1);  // fresh
        kp[i] = &kb[i];
    }
    const std::vector<BitCt> ek = aes_key_schedule(kp, driver);
    std::vector<uint64_t> he(44 * 32 * L);
    for (size_t i = 0; i < ek.size(); i++) std::memcpy(&he[i * L], ek[i].ct.data(), L * 8);
    if (device_mem) {
        std::lock_guard<std::mutex> g(mu_);
        hip_check(hipMemcpyAsync(expanded, he.data(), he.size() * 8, hipMemcpyHostToDevice, engine_->stream()),
                  "upload expanded key");
        engine_->synchronize();
    } else
        std::memcpy(expanded, he.data(), he.size() * 8);
}



// ---------------------------------------------------------------------------------------------
// shortint_1bit model (src/tfhe/shortint_1bit.rs)
// ---------------------------------------------------------------------------------------------
void Context::require_s1() const {
    if (params().model != 2) throw ModelError{TAE_E_PARAM, "this call belongs to the shortint_1bit parameter set"};
}

void Context::s1_bootstrap_raw(const uint64_t *in, size_t B, const uint64_t *tvs, size_t n_tv, uint64_t *out,
                               bool device_mem) {
    require_s1();
    if (n_tv < 1) throw ModelError{TAE_E_ARG, "at least one test vector"};
    const size_t L = bit_len(), G = params().glwe_len();
    // the test vectors are host arrays, always (like the LUTs of the other models)
    std::lock_guard<std::mutex> g(mu_);
    hip_check(hipSetDevice(engine_->device()), "hipSetDevice");
    DevBuf d_tv(n_tv * G * 8);
    hip_check(hipMemcpyAsync(d_tv.p, tvs, n_tv * G * 8, hipMemcpyHostToDevice, engine_->stream()), "tv upload");
    if (device_mem) {
        engine_->order_after_caller();
        engine_->s1_bootstrap(in, d_tv.as<uint64_t>(), n_tv, out, B);
        engine_->synchronize();
        return;
    }
    DevBuf d_in(B * L * 8), d_out(B * L * 8);
    hip_check(hipMemcpyAsync(d_in.p, in, B * L * 8, hipMemcpyHostToDevice, engine_->stream()), "upload");
    engine_->s1_bootstrap(d_in.as<uint64_t>(), d_tv.as<uint64_t>(), n_tv, d_out.as<uint64_t>(), B);
    hip_check(hipMemcpyAsync(out, d_out.p, B * L * 8, hipMemcpyDeviceToHost, engine_->stream()), "download");
    engine_->synchronize();
}

void Context::s1_packing_keyswitch_raw(const uint64_t *cts, size_t count, uint64_t *glwe, bool device_mem) {
    require_s1();
    if (count < 1 || count > (size_t)params().N) throw ModelError{TAE_E_ARG, "packing keyswitch takes 1..N ciphertexts"};
    run8(cts, count * bit_len(), glwe, params().glwe_len(), device_mem,
         [&](const uint64_t *i, uint64_t *o, const uint64_t *) { engine_->s1_pack(i, (int)count, o); }, nullptr);
}

void Context::s1_test_vectors_from_ciphertexts_raw(const uint64_t *ct0, const uint64_t *ct1, size_t B, uint64_t *tvs,
                                                   bool device_mem) {
    require_s1();
    const size_t L = bit_len(), G = params().glwe_len();
    std::lock_guard<std::mutex> g(mu_);
    hip_check(hipSetDevice(engine_->device()), "hipSetDevice");
    // interleave the pairs (2b, 2b+1) = (ct0[b], ct1[b]) on the device, as the tree levels hold them
    DevBuf d_pairs(2 * B * L * 8), d_pks(2 * B * G * 8);
    const auto kind = device_mem ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (device_mem) engine_->order_after_caller();
    hip_check(hipMemcpy2DAsync(d_pairs.p, 2 * L * 8, ct0, L * 8, L * 8, B, kind, engine_->stream()), "pairs");
    hip_check(hipMemcpy2DAsync(d_pairs.as<uint64_t>() + L, 2 * L * 8, ct1, L * 8, L * 8, B, kind, engine_->stream()),
              "pairs");
    engine_->s1_pks(d_pairs.as<uint64_t>(), 2 * B, d_pks.as<uint64_t>());
    if (device_mem) {
        engine_->s1_tv_from_pks(d_pks.as<uint64_t>(), B, tvs);
    } else {
        DevBuf d_tv(B * G * 8);
        engine_->s1_tv_from_pks(d_pks.as<uint64_t>(), B, d_tv.as<uint64_t>());
        hip_check(hipMemcpyAsync(tvs, d_tv.p, B * G * 8, hipMemcpyDeviceToHost, engine_->stream()), "download");
        engine_->synchronize();
        return;
    }
    engine_->synchronize();
}

void Context::s1_multivariate_raw(const uint64_t *bits, size_t G, int nbits, const uint64_t *f_tables, int n_fn,
                                  uint64_t *out, bool device_mem) {
    require_s1();
    if (nbits < 1 || nbits > 8) throw ModelError{TAE_E_ARG, "multivariate functions take 1..=8 bits (shortint_1bit.rs:526)"};
    if (n_fn < 1) throw ModelError{TAE_E_ARG, "at least one function"};
    const size_t L = bit_len(), GL = params().glwe_len(), V = (size_t)1 << (nbits - 1);
    // generate_multivariate_test_vector (:519-536): test vector v of function f selects f(2v + bit)
    std::vector<uint64_t> tvs((size_t)n_fn * V * GL);
    for (int f = 0; f < n_fn; f++)
        for (size_t v = 0; v < V; v++) {
            const uint64_t *tab = f_tables + (size_t)f * 2 * V;
            if (tab[2 * v] > 1 || tab[2 * v + 1] > 1) throw ModelError{TAE_E_ARG, "function values must be 0 or 1"};
            s1_test_vector(params(), tab[2 * v], tab[2 * v + 1], &tvs[((size_t)f * V + v) * GL]);
        }
    std::lock_guard<std::mutex> g(mu_);
    hip_check(hipSetDevice(engine_->device()), "hipSetDevice");
    DevBuf d_tv(tvs.size() * 8);
    hip_check(hipMemcpyAsync(d_tv.p, tvs.data(), tvs.size() * 8, hipMemcpyHostToDevice, engine_->stream()), "tv upload");
    if (device_mem) {
        engine_->order_after_caller();
        engine_->s1_multivariate(bits, G, nbits, d_tv.as<uint64_t>(), n_fn, out);
        engine_->synchronize();
        return;
    }
    DevBuf d_in(G * nbits * L * 8), d_out(G * n_fn * L * 8);
    hip_check(hipMemcpyAsync(d_in.p, bits, G * nbits * L * 8, hipMemcpyHostToDevice, engine_->stream()), "upload");
    engine_->s1_multivariate(d_in.as<uint64_t>(), G, nbits, d_tv.as<uint64_t>(), n_fn, d_out.as<uint64_t>());
    hip_check(hipMemcpyAsync(out, d_out.p, G * n_fn * L * 8, hipMemcpyDeviceToHost, engine_->stream()), "download");
    engine_->synchronize();
}

}  // namespace tae
