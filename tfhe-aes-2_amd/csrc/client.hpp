// Client side of the 1-bit WoP-PBS model: key generation, bit encryption/decryption, LUTs.
//
// Reference: src/tfhe/shortint_woppbs_1bit.rs
//   ClientKey::{encrypt, decrypt}            :197-226
//   FheContext::generate_keys_with_params    :245-268 (tfhe::shortint::gen_keys +
//                                             WopbsKey::new_wopbs_key_only_for_wopbs)
//   encode_bit / decode_bit                  :125-132
//   generate_multivariate_luts               :366-403
// The reference seeds its CSPRNG from the OS (src/tfhe/engine.rs:164-168); this build draws all
// randomness from ChaCha20(seed) streams laid out as in DESIGN.md ("keygen spec") so that a run is
// reproducible and the CPU oracle can regenerate identical keys.
#pragma once
#include <array>
#include <atomic>
#include <cstdint>
#include <vector>

#include "params.hpp"

namespace tae {

// ---- ChaCha20 (DJB: 64-bit block counter, 64-bit nonce) ----
void chacha20_block(const uint8_t key[32], uint64_t nonce, uint64_t counter, uint8_t out[64]);

class ChaChaStream {
  public:
    ChaChaStream(const uint8_t key[32], uint64_t nonce, uint64_t counter);
    uint64_t next_u64();
    uint64_t next_gaussian_torus(double sigma);  // Box-Muller, rint(z * sigma * 2^64)
  private:
    uint8_t key_[32];
    uint64_t nonce_, ctr_;
    uint8_t buf_[64];
    int pos_;
};

// Keygen stream purposes (DESIGN.md keygen spec).
enum Purpose : uint64_t { LWE_SK = 1, GLWE_SK = 2, KSK = 3, BSK = 4, PFPKSK = 5, ENCRYPT = 6, ENCRYPT_INT = 7 };
constexpr uint64_t kCtStride = 1ull << 24;
// Ciphertext #idx of purpose P starts its mask stream at ChaCha20(nonce = 2P | (idx >> 40) << 8,
// counter = (idx mod 2^40) * 2^24) and its noise stream at nonce 2P + 1 (same high bits, same counter):
// injective over all 64-bit indices (the counter alone would wrap at idx = 2^40 and alias idx - 2^40).
inline uint64_t ct_nonce(Purpose purpose, int noise, uint64_t idx) {
    return (2 * (uint64_t)purpose + (uint64_t)noise) | ((idx >> 40) << 8);
}
inline uint64_t ct_counter(uint64_t idx) { return (idx & ((1ull << 40) - 1)) * kCtStride; }
// Encryption index space of the client key: explicit raw indices live below kAutoIndexBase; the
// indices tae_encrypt (and raw calls with TAE_INDEX_AUTO) reserve from next_index live above it,
// so the two can never collide.
constexpr uint64_t kAutoIndexBase = 1ull << 63;

inline uint64_t encode_bit(uint64_t bit) { return bit << 63; }
inline uint64_t decode_bit(uint64_t x) { return ((x + (1ull << 62)) & (1ull << 63)) >> 63; }

// Standard-domain server keys (what tfhe's WopbsKey holds before the Fourier conversion).
struct ServerKeyRaw {
    Params p;
    std::vector<uint64_t> ksk;     // [K][ks_l][n+1]
    std::vector<uint64_t> bsk;     // [n][pbs_l][k+1][(k+1)N]
    std::vector<uint64_t> pfpksk;  // [k+1][K+1][pfks_l][(k+1)N]
};

struct ClientKey {
    Params p;
    std::array<uint8_t, 32> seed;
    std::vector<uint64_t> lwe_sk;   // [n]
    std::vector<uint64_t> glwe_sk;  // [K] (GLWE key as LWE key of dimension K)
    std::atomic<uint64_t> next_index{0};

    // ClientKey::encrypt: LWE under the big key, lwe noise, encode_bit (encryption index explicit)
    void encrypt_bit_at(uint64_t bit, uint64_t index, uint64_t *out) const;
    uint64_t phase(const uint64_t *ct) const;
    uint64_t decrypt_bit(const uint64_t *ct) const { return decode_bit(phase(ct)); }

    // 8-bit model (shortint_woppbs_8bit.rs:196-225): bits are LWEs under the SMALL key [n+1]
    void encrypt_small_bit_at(uint64_t bit, uint64_t index, uint64_t *out) const;
    uint64_t phase_small(const uint64_t *ct) const;
    uint64_t decrypt_small_bit(const uint64_t *ct) const { return decode_bit(phase_small(ct)); }
    // shortint encrypt_without_padding / decrypt_without_padding (message modulus 256, carry 1):
    // big-key LWE of m * 2^56 with glwe noise (the FullWidthCiphertext of the 8-bit model)
    void encrypt_int_at(uint64_t value, uint64_t index, uint64_t *out) const;
    uint64_t decrypt_int(const uint64_t *ct) const { return ((phase(ct) + (1ull << 55)) >> 56) & 255; }
    // shortint_1bit model (shortint_1bit.rs:149-161): shortint encrypt / decrypt with message modulus 2,
    // carry 1 under the SMALL key: plaintext m * 2^62, decrypt_message_and_carry % 2
    void encrypt_s1_bit_at(uint64_t bit, uint64_t index, uint64_t *out) const;
    uint64_t decrypt_s1_bit(const uint64_t *ct) const { return decode_s1(phase_small(ct)); }
    static uint64_t decode_s1(uint64_t x) { return ((x + ((x & (1ull << 61)) << 1)) >> 62) & 1; }
    // bits of any model: big key (model 1) or small key (models 8 and 2)
    size_t bit_len() const { return p.bit_len(); }
    void encrypt_model_bit_at(uint64_t bit, uint64_t index, uint64_t *out) const {
        if (p.model == 8)
            encrypt_small_bit_at(bit, index, out);
        else if (p.model == 2)
            encrypt_s1_bit_at(bit, index, out);
        else
            encrypt_bit_at(bit, index, out);
    }
    uint64_t decrypt_model_bit(const uint64_t *ct) const {
        return p.model == 8 ? decrypt_small_bit(ct) : p.model == 2 ? decrypt_s1_bit(ct) : decrypt_bit(ct);
    }
};

// generate_keys_with_params; threads = worker threads for the key material.
void generate_keys(const Params &p, const uint8_t seed[32], int threads, ClientKey &ck,
                   ServerKeyRaw &sk);

// secret keys only (same streams as generate_keys)
void generate_client_key(const Params &p, const uint8_t seed[32], ClientKey &ck);

// generate_multivariate_luts: out [output_bits][N << tree_bits]
size_t lut_small_len(int N, int input_bits);
void generate_lut(int N, int input_bits, int output_bits, const uint64_t *f_table, uint64_t *out);

// WopbsKey::generate_lut_without_padding for message modulus 256 (8-bit model,
// shortint_woppbs_8bit.rs:262-265): out[i] = (f(i mod 256) mod 256) << 56, i < max(N, 256)
void generate_lut_without_padding(int N, const uint64_t *f_table /*[256]*/, uint64_t *out);

// shortint_1bit test_vector_from_cleartext_fn (shortint_1bit.rs:365-390) for f(0) = f0, f(1) = f1:
// trivial GLWE [(k+1)N], body boxes encode(f0) | encode(f1) (encode_bit = m << 62) rotated left by N/4
void s1_test_vector(const Params &p, uint64_t f0, uint64_t f1, uint64_t *glwe);

// Negacyclic FFT tables (twist, untwist, W_M) -- the spec shared with the kernels.
struct FftTables {
    int N, M;
    std::vector<double> twist, untwist, w;  // interleaved (re, im), M entries each
};
FftTables make_fft_tables(int N);
std::vector<double> make_lf512_table();  // lf512.hpp layout
std::vector<double> make_lf1k_table();   // lf1k.hpp layout

}  // namespace tae
