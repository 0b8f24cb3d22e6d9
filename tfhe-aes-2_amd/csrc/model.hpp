// Host-side mirror of the reference's model and AES traits, driving the device Engine.
//
// Reference (allanbrondum/tfhe-aes-2):
//   src/tfhe.rs:11-24                       ClientKeyT / ContextT
//   src/tfhe/shortint_woppbs_1bit.rs:26-151  BitCt, NoiseLevelWithComponents, BitXorAssign
//   src/tfhe/shortint_woppbs_1bit.rs:165-336 FheContext (ct ids, generate_lookup_table,
//                                            circuit_bootstrap)
//   src/aes_128/fhe/fhe_impls/shortint_woppbs_1bit.rs:17-151
//                                            ByteT impls + ShortintWoppbs1BitSboxGalMulPbsAesEncrypt
//   src/aes_128/fhe/fhe_sbox_gal_mul_pbs.rs:27-191 encrypt_block_for_rounds, key_schedule
//   src/aes_128/fhe/fhe_sbox_pbs.rs:22-171   the same for the fhe_sbox_pbs driver
// The ciphertext arithmetic runs in the Engine (HIP); this layer keeps the reference's noise
// bookkeeping (noise^2 level + independent component ids) on the host, per ciphertext.
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "client.hpp"
#include "engine.hpp"

namespace tae {

// Reference panics become status codes.
struct ModelError {
    int code;  // TAE_E_NOISE / TAE_E_INDEP / TAE_E_PARAM / TAE_E_ARG
    std::string msg;
};

// NoiseLevelWithComponents (shortint_woppbs_1bit.rs:34-78)
struct NoiseLevel {
    uint64_t noise_level_squared = 0;
    std::vector<uint64_t> components;  // sorted CiphertextIds

    static NoiseLevel with_noise_level(uint64_t nl, uint64_t id) { return {nl, {id}}; }
    static NoiseLevel trivial() { return {}; }
    // add_assign: asserts disjoint components, unions them, adds noise^2 and validates <= max
    void add_assign(const NoiseLevel &rhs, uint64_t max_noise_sq);
};

uint64_t next_ct_id();  // FheContext::next_ct_id (process-wide counter)

struct BitCt {
    std::vector<uint64_t> ct;  // [K+1]
    NoiseLevel noise;
    uint64_t max_noise_sq = 0;

    void xor_assign(const BitCt &rhs);  // BitXorAssign
};

enum class AesDriver { GalMul, SboxPbs };

struct Lut {  // WopbsLUTBase
    int input_bits = 0, output_bits = 0;
    size_t small_len = 0;
    std::vector<uint64_t> data;  // [output_bits][small_len]
};

class Context {  // FheContext
  public:
    Context(std::unique_ptr<Engine> engine) : engine_(std::move(engine)) {}
    const Params &params() const { return engine_->params(); }
    Engine &engine() { return *engine_; }
    std::mutex &mutex() { return mu_; }

    BitCt trivial(uint64_t bit) const;
    BitCt wrap(std::vector<uint64_t> ct, uint64_t noise_level_squared) const;  // BitCt::with_noise_level
    Lut generate_lookup_table(int input_bits, int output_bits, const uint64_t *f_values) const;
    std::vector<BitCt> circuit_bootstrap(const std::vector<const BitCt *> &bits, const Lut &lut);
    // batched raw circuit bootstrap (device or host arrays)
    void circuit_bootstrap_raw(const uint64_t *bits, size_t groups, int n_in, const Lut &lut, uint64_t *out,
                               bool device_mem);

    // Aes128Encrypt::encrypt_block_for_rounds over many blocks (noise bookkeeping per bit).  Driver
    // GalMul = fhe_sbox_gal_mul_pbs (ShortintWoppbs1BitSboxGalMulPbsAesEncrypt); SboxPbs = fhe_sbox_pbs
    // (ShortintWoppbs1BitSboxPbsAesEncrypt on the 1-bit model).  The 8-bit model has fhe_sbox_pbs only
    // (ShortintWoppbs8BitSboxPbsAesEncrypt) and ignores the flag.
    std::vector<BitCt> aes_encrypt_blocks(const std::vector<const BitCt *> &expanded_key,
                                          const std::vector<const BitCt *> &blocks, size_t n_blocks, int rounds,
                                          AesDriver driver = AesDriver::GalMul);
    // key_schedule: fhe_sbox_gal_mul_pbs (:134-164) or fhe_sbox_pbs (:123-171)
    std::vector<BitCt> aes_key_schedule(const std::vector<const BitCt *> &key, AesDriver driver = AesDriver::GalMul);
    // raw arrays, fresh inputs; static noise-schedule validation
    void aes_encrypt_blocks_raw(const uint64_t *rk, const uint64_t *blocks, size_t n_blocks, int rounds,
                                uint64_t *out, bool device_mem, AesDriver driver = AesDriver::GalMul);
    // raw key schedule: key [128][bit_len] fresh bits -> [44*32][bit_len]
    void aes_key_schedule_raw(const uint64_t *key, uint64_t *expanded, bool device_mem,
                              AesDriver driver = AesDriver::GalMul);

    // ---- 8-bit model (src/tfhe/shortint_woppbs_8bit.rs, fhe_impls/shortint_woppbs_8bit.rs) ----
    size_t bit_len() const { return params().bit_len(); }
    // FheContext::bootstrap_from_bits over G bytes: bits [G][8][n+1] -> int ciphertexts [G][K+1]
    void bootstrap_from_bits_raw(const uint64_t *bits, size_t groups, const Lut &lut, uint64_t *out, bool device_mem);
    // FheContext::extract_bits_from_ciphertext over G ints: [G][K+1] -> [G][8][n+1]
    void extract_bits_raw(const uint64_t *ints, size_t groups, uint64_t *out, bool device_mem);

    // ---- shortint_1bit model (src/tfhe/shortint_1bit.rs; param set SHORTINT_1BIT), raw arrays ----
    // FheContext::bootstrap over B bits [B][n+1] with test vectors tvs [n_tv][(k+1)N] (bit b takes b % n_tv)
    void s1_bootstrap_raw(const uint64_t *in, size_t B, const uint64_t *tvs, size_t n_tv, uint64_t *out, bool device_mem);
    // FheContext::packing_keyswitch: count bits -> one GLWE [(k+1)N]
    void s1_packing_keyswitch_raw(const uint64_t *cts, size_t count, uint64_t *glwe, bool device_mem);
    // test_vector_from_ciphertexts over B pairs (ct0[b], ct1[b]) -> [B][(k+1)N]
    void s1_test_vectors_from_ciphertexts_raw(const uint64_t *ct0, const uint64_t *ct1, size_t B, uint64_t *tvs,
                                              bool device_mem);
    // calculate_multivariate_function for n_fn functions (f_tables [n_fn][2^nbits], host, 0/1 values) of
    // G groups of nbits bits [G][nbits][n+1] -> [G][n_fn][n+1]
    void s1_multivariate_raw(const uint64_t *bits, size_t G, int nbits, const uint64_t *f_tables, int n_fn,
                             uint64_t *out, bool device_mem);

  private:
    void require_s1() const;
    template <class F>
    void run8(const uint64_t *in, size_t in_len, uint64_t *out, size_t out_len, bool device_mem, F fn, const Lut *lut);
    std::vector<BitCt> sbox_pbs_key_schedule(const std::vector<const BitCt *> &key);
    std::vector<NoiseLevel> block_noise_schedule(AesDriver driver, const std::vector<NoiseLevel> &rk,
                                                 const std::vector<NoiseLevel> &block, int rounds) const;
    void run_aes_blocks(AesDriver driver, const uint64_t *d_rk, const uint64_t *d_in, size_t n_blocks, int rounds,
                        uint64_t *d_out);
    std::unique_ptr<Engine> engine_;
    std::mutex mu_;
};

// Noise bookkeeping of the AES round function on metadata only: returns output noise levels
// (per bit) or throws ModelError exactly where the reference would panic.
std::vector<NoiseLevel> aes_noise_schedule(const std::vector<NoiseLevel> &rk, const std::vector<NoiseLevel> &block,
                                           int rounds, uint64_t max_noise_sq);
// fhe_sbox_pbs over the 1-bit model: raises TAE_E_INDEP at the first MixColumns (rounds >= 2).
std::vector<NoiseLevel> sbox_pbs_noise_schedule(const std::vector<NoiseLevel> &rk, const std::vector<NoiseLevel> &block,
                                                int rounds, uint64_t max_noise_sq);
// The same for fhe_sbox_pbs with the 8-bit model (additive shortint NoiseLevel, max 11; SubBytes
// outputs are NOMINAL = 1).
std::vector<NoiseLevel> aes8_noise_schedule(const std::vector<NoiseLevel> &rk, const std::vector<NoiseLevel> &block,
                                            int rounds, uint64_t max_noise_level);

}  // namespace tae
