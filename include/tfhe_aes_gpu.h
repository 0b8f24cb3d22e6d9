/*
 * tfhe_aes_gpu.h -- C-ABI of the MI355X-native FHE AES-128 evaluator (drop-in boundary).
 *
 * Plain C types only (opaque handles, pointers, sizes, int status codes); no torch/HIP types.
 * Every entry point names the reference interface it replaces (allanbrondum/tfhe-aes-2 @
 * 2025-03-07, paths relative to the reference root).  The reference is in-process Rust; these
 * are the symbols a Rust `extern "C"` shim implementing its traits would bind.
 *
 * Conventions
 *   - LWE ciphertexts are u64 arrays in the tfhe layout [a_0 .. a_{K-1}, b] (K = k*N, big key);
 *     a byte is 8 ciphertexts MSB-first (src/util.rs:33-42); a block is 16 bytes in block order;
 *     an expanded key is 44 words x 4 bytes (fhe.rs:16-38, [Word; 44]).
 *   - Errors are status codes instead of the reference's panics; tae_last_error() gives the
 *     message of the calling thread's last failure.
 *   - A context is bound to one GPU and internally serialised: safe to share across host
 *     threads (the reference's FheContext is Send + Sync).
 *   - There is no CPU fallback: without a usable GPU, context creation fails with TAE_E_NODEV.
 */
#ifndef TFHE_AES_GPU_H
#define TFHE_AES_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (the reference panics: "NoiseTooBig", "noise components not independent") */
#define TAE_OK 0
#define TAE_E_NOISE 1     /* MaxNoiseLevel::validate -> NoiseTooBig (shortint_woppbs_1bit.rs:74-76) */
#define TAE_E_INDEP 2     /* "noise components not independent" (shortint_woppbs_1bit.rs:64-70) */
#define TAE_E_PARAM 3     /* invalid parameter / unsupported shape */
#define TAE_E_HIP 4       /* HIP runtime failure */
#define TAE_E_ARG 5       /* invalid argument (null pointer, size mismatch) */
#define TAE_E_NODEV 6     /* no GPU available: the product path has no CPU fallback */

/* parameter sets: src/tfhe/shortint_woppbs_1bit/parameters.rs */
#define TAE_PARAMS_SQRD_LVL_1 0   /* :29-61  */
#define TAE_PARAMS_SQRD_LVL_4 1   /* :77-109 */
#define TAE_PARAMS_SQRD_LVL_64 2  /* :125-157, default (bin/main.rs:82-83) */
#define TAE_PARAMS_SQRD_LVL_256 3 /* :173-205 */
/* the 8-bit model's set: src/tfhe/shortint_woppbs_8bit.rs:39-86 (ShortintWoppbs8BitSboxPbsAesEncrypt,
 * fhe_impls/shortint_woppbs_8bit.rs:44-64).  Bits are LWEs under the SMALL key ([n+1] u64); a byte
 * is bootstrapped through one 8-bit integer ciphertext (big key, [K+1], plaintext m * 2^56). */
#define TAE_PARAMS_WOPPBS_8BIT 4
/* the shortint_1bit model's set: src/tfhe/shortint_1bit.rs:62-83 (ClassicPBSParameters, message modulus 2,
 * carry 1, EncryptionKeyChoice::Small; Shortint1BitSboxPbsAesEncrypt, fhe_impls/shortint_1bit.rs:52-72).
 * Bits are shortint ciphertexts under the SMALL key ([n+1] u64, plaintext m * 2^62); the third server key
 * array ("pfpksk") holds the packing keyswitch key [n][ks_l][(k+1)N] (shortint_1bit.rs:176-186). */
#define TAE_PARAMS_SHORTINT_1BIT 5

/* memory kinds for the raw-array entry points.  TAE_MEM_DEVICE: pointers into the context's device
 * memory.  By default the library orders itself after all work already queued on that device (it
 * synchronizes the device before its first read of caller buffers, e.g. after an RCCL broadcast or torch
 * copies on other streams); after tae_set_caller_stream it waits only for the work queued on that one
 * stream (an event, no host sync).  Device outputs are complete when the call returns. */
#define TAE_MEM_HOST 0
#define TAE_MEM_DEVICE 1

typedef struct tae_client_key tae_client_key; /* shortint_woppbs_1bit::ClientKey (:189-195) */
typedef struct tae_context tae_context;       /* shortint_woppbs_1bit::FheContext (:165-172) */
typedef struct tae_bit tae_bit;               /* shortint_woppbs_1bit::BitCt (:26-32) */
typedef struct tae_lut tae_lut;               /* tfhe::shortint::wopbs::WopbsLUTBase */

typedef struct {
    int n, k, N, pbs_l, pbs_b, ks_l, ks_b, cbs_l, cbs_b, pfks_l, pfks_b;
    double lwe_std, glwe_std, pfks_std;
    uint64_t max_noise_sq; /* 1-bit model: max noise^2; 8-bit model: shortint MaxNoiseLevel (11) */
    int model;             /* 1 = shortint_woppbs_1bit, 8 = shortint_woppbs_8bit */
} tae_params;

const char *tae_last_error(void);
const char *tae_version(void);
int tae_device_count(int *count);
int tae_get_params(int param_set, tae_params *out); /* parameters::params_sqrd_lvl_* */
/* u64 length of one bit ciphertext: K+1 (1-bit model, big key) or n+1 (8-bit model, small key) */
int tae_bit_len(int param_set, size_t *len);

/* ---- keys (FheContext::generate_keys_with_params, shortint_woppbs_1bit.rs:245-268) ----------
 * Client key generation on the host from a 32-byte seed (ChaCha20 streams, DESIGN.md keygen
 * spec), server keys uploaded to `device` and the bootstrapping key converted to the Fourier
 * domain there.  generate_keys_sqrd_lvl_* (:229-243) = this with the matching param_set. */
int tae_generate_keys(int param_set, const uint8_t seed[32], int device, int threads,
                      tae_client_key **client_key, tae_context **context);
/* Client key only + standard-domain server keys exported to caller buffers (sizes from
 * tae_server_key_sizes) -- used to broadcast keys across ranks before tae_context_create_raw. */
int tae_server_key_sizes(int param_set, size_t *ksk_len, size_t *bsk_len, size_t *pfpksk_len);
int tae_generate_keys_raw(int param_set, const uint8_t seed[32], int threads,
                          tae_client_key **client_key, uint64_t *ksk, uint64_t *bsk,
                          uint64_t *pfpksk);
/* Client key only (secret keys from the seed's LWE_SK / GLWE_SK streams; no server keys) -- every rank
 * of a multi-GPU run derives the same client key this way while server keys are broadcast. */
int tae_client_key_from_seed(int param_set, const uint8_t seed[32], tae_client_key **client_key);
/* Server context from raw keys: mem = TAE_MEM_HOST (copied to the device) or TAE_MEM_DEVICE
 * (device pointers on `device`, e.g. after an RCCL broadcast; they must outlive the context). */
int tae_context_create_raw(int param_set, int device, const uint64_t *ksk, const uint64_t *bsk,
                           const uint64_t *pfpksk, int mem, tae_context **context);
void tae_context_free(tae_context *ctx);

/* ---- On-disk keys (no reference counterpart: the reference keeps keys in memory) --
 * One little-endian file "TAEKEY02" holding a client key (its 32-byte seed + encryption counter)
 * and/or the standard-domain server keys (ksk, bsk, pfpksk as sized by tae_server_key_sizes), with
 * a trailing checksum (format: tfhe-aes-2_amd/csrc/keyio.cpp).  Rejected files -> TAE_E_ARG. */
#define TAE_KEYS_CLIENT 1
#define TAE_KEYS_SERVER 2
/* client_key may be NULL; ksk/bsk/pfpksk all NULL (client only) or all set */
int tae_keys_save(const char *path, int param_set, const tae_client_key *client_key, const uint64_t *ksk,
                  const uint64_t *bsk, const uint64_t *pfpksk);
/* parameter set and TAE_KEYS_* flags from the header (payload not verified) */
int tae_keys_file_info(const char *path, int *param_set, int *flags);
/* client_key (NULL: not wanted) and/or the three server arrays (all NULL: not wanted); the checksum
 * is verified before anything is returned (server arrays are filled in place: discard them on error) */
int tae_keys_load(const char *path, tae_client_key **client_key, uint64_t *ksk, uint64_t *bsk, uint64_t *pfpksk);
void tae_client_key_free(tae_client_key *ck);
int tae_client_key_secrets(const tae_client_key *ck, uint64_t *lwe_sk /*[n]*/,
                           uint64_t *glwe_sk /*[k*N]*/);
int tae_context_params(const tae_context *ctx, tae_params *out);

/* ---- ClientKeyT / ContextT (src/tfhe.rs:11-24) -------------------------------------------- */
int tae_encrypt(const tae_client_key *ck, uint64_t bit, tae_bit **out);       /* ClientKey::encrypt */
int tae_decrypt(const tae_client_key *ck, const tae_bit *bit, uint64_t *out); /* ClientKey::decrypt */
int tae_trivial(const tae_context *ctx, uint64_t bit, tae_bit **out);         /* ContextT::trivial */
/* raw: encrypt `count` bits ([count][K+1]) with encryption indices start..start+count-1.  Each index
 * selects the ciphertext's mask and noise streams (DESIGN.md keygen spec), so an index must never be
 * reused for a different plaintext under one key: explicit ranges must lie below 2^63 (TAE_E_ARG
 * otherwise); start_index = TAE_INDEX_AUTO reserves `count` fresh indices from the key's counter,
 * the region tae_encrypt draws from (disjoint from every explicit range). */
#define TAE_INDEX_AUTO UINT64_MAX
int tae_encrypt_bits_raw(const tae_client_key *ck, const uint8_t *bits, size_t count,
                         uint64_t start_index, uint64_t *out);
int tae_decrypt_bits_raw(const tae_client_key *ck, const uint64_t *cts, size_t count, uint8_t *bits);
/* 8-bit model integers (FullWidthCiphertext, shortint_woppbs_8bit.rs:167-178): shortint
 * encrypt_without_padding / decrypt_without_padding, message modulus 256 ([count][K+1]) */
int tae_encrypt_ints_raw(const tae_client_key *ck, const uint8_t *values, size_t count, uint64_t start_index,
                         uint64_t *out);
int tae_decrypt_ints_raw(const tae_client_key *ck, const uint64_t *cts, size_t count, uint8_t *values);

/* ---- BitCt (shortint_woppbs_1bit.rs:26-151) ----------------------------------------------- */
int tae_bit_clone(const tae_bit *bit, tae_bit **out);
void tae_bit_free(tae_bit *bit);
int tae_bit_xor_assign(tae_bit *lhs, const tae_bit *rhs); /* BitXorAssign (:134-142) */
int tae_bit_noise_level(const tae_bit *bit, uint64_t *noise_level_squared);
int tae_bit_data(const tae_bit *bit, uint64_t *out, size_t len); /* LWE coefficients [K+1] */
int tae_bit_from_data(const tae_context *ctx, const uint64_t *data, size_t len,
                      uint64_t noise_level_squared, tae_bit **out); /* BitCt::with_noise_level */
/* BitXorAssign over whole arrays of bits (xor_state, src/aes_128/fhe/data_model.rs:270-274):
 * lhs[i] += rhs[i] (wrapping u64 LWE addition = XOR of the encoded bits) for `count` bit ciphertexts
 * of tae_bit_len words each, on the context's GPU.  With both noise arrays (squared noise levels per
 * bit) the reference's NoiseTooBig rule is enforced before anything is written and out_noise_sq
 * (may be NULL) receives the sums; the component-independence check needs BitCt handles
 * (tae_bit_xor_assign) and is the caller's duty here.  The three noise arrays are always HOST
 * pointers, whatever `mem` says (mem applies to lhs / rhs only). */
int tae_xor_batch(const tae_context *ctx, uint64_t *lhs, const uint64_t *rhs, size_t count,
                  const uint64_t *lhs_noise_sq, const uint64_t *rhs_noise_sq, uint64_t *out_noise_sq, int mem);

/* ---- LUT + circuit bootstrap (shortint_woppbs_1bit.rs:274-336) ----------------------------- */
/* generate_lookup_table: f_values[1 << input_bits] */
int tae_generate_lookup_table(const tae_context *ctx, int input_bits, int output_bits,
                              const uint64_t *f_values, tae_lut **out);
void tae_lut_free(tae_lut *lut);
/* generate_multivariate_luts (shortint_woppbs_1bit.rs:366-403) without a context, for any power-of-two
 * polynomial size: out [output_bits][poly_size << max(0, input_bits - log2 poly_size)], small LUT j
 * holding encode_bit(bit output_bits-1-j of f(v)) at coefficient v (the layout pinned by the
 * reference's tests :665-697); out_len must equal that size.  input_bits is 1..16 as in the reference
 * (its assert 0 < input_bits <= 16 and u16 argument of f, :372); anything else is TAE_E_ARG. */
int tae_generate_multivariate_luts(int poly_size, int input_bits, int output_bits, const uint64_t *f_values,
                                   uint64_t *out, size_t out_len);
int tae_lut_data(const tae_lut *lut, uint64_t *out, size_t len, size_t *needed);
/* FheContext::circuit_bootstrap(&[&BitCt], &WopbsLUTBase) -> Vec<BitCt> */
int tae_circuit_bootstrap(const tae_context *ctx, const tae_bit *const *bits, size_t n_bits,
                          const tae_lut *lut, tae_bit **out /*[output_bits]*/);
/* batched: groups x n_in bits [groups][n_in][K+1] -> [groups][n_out][K+1] */
int tae_circuit_bootstrap_raw(const tae_context *ctx, const uint64_t *bits, size_t groups,
                              int n_in, const tae_lut *lut, uint64_t *out, int mem);

/* ---- 8-bit model FheContext (shortint_woppbs_8bit.rs:262-336) ------------------------------
 * generate_lookup_table: tae_generate_lookup_table(ctx, 8, 8, f[256]) (without-padding LUT);
 * tae_circuit_bootstrap[_raw] with n_in = 8 runs Byte::bootstrap_with_lut (8 bits -> 8 bits).
 * bootstrap_from_bits: bits [groups][8][n+1] -> ints [groups][K+1] */
int tae_bootstrap_from_bits_raw(const tae_context *ctx, const uint64_t *bits, size_t groups, const tae_lut *lut,
                                uint64_t *out, int mem);
/* extract_bits_from_ciphertext: ints [groups][K+1] -> bits [groups][8][n+1], MSB first */
int tae_extract_bits_raw(const tae_context *ctx, const uint64_t *ints, size_t groups, uint64_t *out, int mem);

/* ---- shortint_1bit model (context of TAE_PARAMS_SHORTINT_1BIT; src/tfhe/shortint_1bit.rs) -------------- */
/* Test vectors are GLWE ciphertexts [(k+1)N] u64 and always host arrays; bits are [n+1] (mem applies). */
/* FheContext::test_vector_from_cleartext_fn (:208-223, :365-390) for f(0) = f0, f(1) = f1 */
int tae_s1_test_vector_from_fn(int param_set, uint64_t f0, uint64_t f1, uint64_t *tv);
/* FheContext::bootstrap (:257-294, :296-350) over count bits: bit b is bootstrapped with tvs[b % n_tv] */
int tae_s1_bootstrap(const tae_context *ctx, const uint64_t *in, size_t count, const uint64_t *tvs, size_t n_tv,
                     uint64_t *out, int mem);
/* FheContext::packing_keyswitch (:240-255, :494-518): count (1..N) bits -> one GLWE, bit j at coefficient j */
int tae_s1_packing_keyswitch(const tae_context *ctx, const uint64_t *cts, size_t count, uint64_t *glwe, int mem);
/* FheContext::test_vector_from_ciphertexts (:225-238, :392-492) for count pairs: tvs [count][(k+1)N] (mem) */
int tae_s1_test_vectors_from_ciphertexts(const tae_context *ctx, const uint64_t *ct0, const uint64_t *ct1, size_t count,
                                         uint64_t *tvs, int mem);
/* calculate_multivariate_function (:539-583) with generate_multivariate_test_vector (:520-537) for n_fn
 * functions f_tables [n_fn][2^nbits] (host, 0/1, index = bits MSB first) of each of `groups` groups of
 * nbits (1..8) bits [groups][nbits][n+1] -> out [groups][n_fn][n+1] (ByteT::sbox_substitute is 8
 * functions of a byte, fhe_impls/shortint_1bit.rs:32-50) */
int tae_s1_multivariate(const tae_context *ctx, const uint64_t *bits, size_t groups, int nbits,
                        const uint64_t *f_tables, int n_fn, uint64_t *out, int mem);

/* ---- Aes128Encrypt for ShortintWoppbs1BitSboxGalMulPbsAesEncrypt -------------------------
 *      (src/aes_128/fhe.rs:16-38, fhe_impls/shortint_woppbs_1bit.rs:131-151,
 *       fhe_sbox_gal_mul_pbs.rs:84-191) */
/* encrypt_block_for_rounds: expanded_key[44*32] bits, block[128] bits, out[128] */
int tae_aes_encrypt_block_for_rounds(const tae_context *ctx, const tae_bit *const *expanded_key,
                                     const tae_bit *const *block, int rounds, tae_bit **out);
/* batched extension of encrypt_block (main.rs:141-159 runs blocks in parallel) */
int tae_aes_encrypt_blocks(const tae_context *ctx, const tae_bit *const *expanded_key,
                           const tae_bit *const *blocks, size_t n_blocks, int rounds, tae_bit **out);
/* key_schedule (fhe_sbox_gal_mul_pbs.rs:134-164): key[128] bits -> expanded[44*32] bits */
int tae_aes_key_schedule(const tae_context *ctx, const tae_bit *const *key, tae_bit **expanded);
/* raw arrays: rk [44*32][L], blocks [n][128][L], out [n][128][L] with L = tae_bit_len (K+1, or
 * n+1 for the 8-bit model's ShortintWoppbs8BitSboxPbsAesEncrypt / fhe_sbox_pbs.rs:75-121); inputs
 * fresh (noise level 1) -- the noise schedule of the round function is validated statically. */
int tae_aes_encrypt_blocks_raw(const tae_context *ctx, const uint64_t *rk, const uint64_t *blocks,
                               size_t n_blocks, int rounds, uint64_t *out, int mem);
/* key_schedule on raw fresh key bits [128][L] -> [44*32][L] (either model) */
int tae_aes_key_schedule_raw(const tae_context *ctx, const uint64_t *key, uint64_t *expanded, int mem);

/* ---- Aes128Encrypt for the fhe_sbox_pbs driver (src/aes_128/fhe/fhe_sbox_pbs.rs:22-171) ------------
 * ShortintWoppbs1BitSboxPbsAesEncrypt on the 1-bit model (fhe_impls/shortint_woppbs_1bit.rs:47-81:
 * SubBytes = one 8 -> 8 circuit bootstrap per byte, MixColumns = gf_256_mul by BitCt XORs) and
 * ShortintWoppbs8BitSboxPbsAesEncrypt on the 8-bit model (same as tae_aes_* there).  On the 1-bit model
 * every MixColumns breaks the BitCt noise rules, so rounds >= 2 return TAE_E_INDEP before any device work,
 * where the reference panics "noise components not independent" (its test_light / test_full of this
 * combination are #[ignore]d, :160-176); rounds == 1 and the key schedule run batched on the device. */
int tae_aes_sbox_pbs_encrypt_blocks(const tae_context *ctx, const tae_bit *const *expanded_key,
                                    const tae_bit *const *blocks, size_t n_blocks, int rounds, tae_bit **out);
/* fhe_sbox_pbs::key_schedule (:123-171): key[128] bits -> expanded[44*32] bits */
int tae_aes_sbox_pbs_key_schedule(const tae_context *ctx, const tae_bit *const *key, tae_bit **expanded);
int tae_aes_sbox_pbs_encrypt_blocks_raw(const tae_context *ctx, const uint64_t *rk, const uint64_t *blocks,
                                        size_t n_blocks, int rounds, uint64_t *out, int mem);
int tae_aes_sbox_pbs_key_schedule_raw(const tae_context *ctx, const uint64_t *key, uint64_t *expanded, int mem);

/* Static check of a driver's round-function noise schedule for fresh inputs (no context, no device):
 * TAE_OK, or the status the reference's panic maps to (TAE_E_INDEP / TAE_E_NOISE). */
#define TAE_DRIVER_GAL_MUL 0  /* fhe_sbox_gal_mul_pbs */
#define TAE_DRIVER_SBOX_PBS 1 /* fhe_sbox_pbs */
int tae_aes_noise_schedule_check(int param_set, int driver, int rounds);

/* ---- stage entry points (raw arrays; parity tests and profiling) ---------------------------- */
int tae_stage_keyswitch(const tae_context *ctx, const uint64_t *in, size_t count, uint64_t *out, int mem);
int tae_stage_pbs_shift_boolean(const tae_context *ctx, const uint64_t *small, size_t count, int level,
                                uint64_t *big, int mem);
int tae_stage_bootstrap(const tae_context *ctx, const uint64_t *small, size_t count,
                        const uint64_t *lut_glwe, uint64_t *big, int mem);
int tae_stage_pfks_ggsw(const tae_context *ctx, const uint64_t *big, size_t count, int level,
                        uint64_t *ggsw, int mem);
int tae_stage_ggsw_fourier(const tae_context *ctx, const uint64_t *ggsw, size_t count,
                           double *ggsw_f /*complex interleaved*/, int mem);
int tae_stage_vertical_packing(const tae_context *ctx, const double *ggsw_f, size_t groups, int n_in,
                               const uint64_t *lut, int n_out, uint64_t *out, int mem);

/* ---- device utilities -------------------------------------------------------------------- */
int tae_synchronize(const tae_context *ctx);
/* TAE_MEM_DEVICE inputs are produced on `stream` (a hipStream_t of the context's device, e.g. torch's
 * current stream); NULL restores the device-wide synchronize.  Not thread-safe against calls in flight. */
int tae_set_caller_stream(tae_context *ctx, void *stream);
/* 0 off; 1 per-stage HIP-event times of each batched call; 2 the same plus in-kernel clock stamps of the
 * throughput blind-rotation launches (a diagnostic mode: every stamped launch is read back synchronously) */
int tae_set_timing(const tae_context *ctx, int on);
/* per-stage ms of the last batched call: [keyswitch, pbs, pfks, ggsw_fft, vp] */
int tae_last_stage_times(const tae_context *ctx, float *ms5);
/* [keyswitch, pbs, pfks, ggsw_fft, vp, extract_bits, linear] ms + the CBS-level PBS launch count */
int tae_last_stage_times_v2(const tae_context *ctx, float *ms8);
/* v2's eight values, then the ms and the ciphertext count of the throughput blind-rotation kernel's
 * own launches (br512x4, without the small-batch remainder) -- the roofline's launch duration */
int tae_last_stage_times_v3(const tae_context *ctx, double *v10);
/* v3's ten values, then (timing mode 2) the effective shader clock in GHz of the throughput blind-rotation
 * launches (median over each launch's workgroups of shader cycles / 100 MHz reference ticks, averaged over
 * the launches; MI355X_MICROARCH.md "DVFS give-back") and the number of launches it averages (0: none) */
int tae_last_stage_times_v4(const tae_context *ctx, double *v12);

#ifdef __cplusplus
}
#endif
#endif
