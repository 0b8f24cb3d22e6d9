/*
 * tfhe_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference hot path (allanbrondum/tfhe-aes-2 @ 2025-03-07 on top of
 * tfhe-rs 0.11.2) used as the parity checker for the MI355X product.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.  The product
 * (tfhe-aes-2_amd/) never links, includes or calls anything under oracle/.
 *
 * What is restated (each function cites the reference file:line or the tfhe-rs 0.11.2 routine
 * it follows; tfhe-rs is an un-vendored third-party crate, pinned in Cargo.lock:721-724):
 *   - torus signed gadget decomposition          tfhe-rs SignedDecomposer / decompose_one_level
 *   - negacyclic f64 FFT (twisted, folded)        tfhe-fft 0.7.0 (Cargo.lock:773) via tfhe-rs fft64
 *   - external product / cmux                     tfhe-rs fft64::crypto::ggsw
 *   - blind rotation / PBS                        tfhe-rs fft64::crypto::bootstrap
 *   - keyswitch                                   tfhe-rs algorithms::lwe_keyswitch
 *   - private functional packing keyswitch        tfhe-rs algorithms::lwe_private_functional_packing_keyswitch
 *   - homomorphic_shift_boolean / circuit_bootstrap_boolean / vertical_packing
 *                                                 tfhe-rs fft64::crypto::wop_pbs
 *   - FheContext::circuit_bootstrap               src/tfhe/shortint_woppbs_1bit.rs:292-363
 *   - generate_multivariate_luts                  src/tfhe/shortint_woppbs_1bit.rs:366-403
 *   - encode_bit / decode_bit                     src/tfhe/shortint_woppbs_1bit.rs:125-132
 *   - AES driver (SBOX+GF PBS)                    src/aes_128/fhe/fhe_sbox_gal_mul_pbs.rs:27-191
 *
 * Pinning: the reference is Rust + tfhe-rs and cannot be built here (no cargo/rustc, crates not
 * vendored, no network).  Ciphertext-level values are therefore "parity unpinned" against
 * tfhe-rs; the oracle is pinned at the decrypted level by the reference's own golden vectors
 * (FIPS-197 C.1, the ChaCha20([0;32]) test_light / test_full blocks, the README counter-mode
 * blocks) and its exact-LUT tests (shortint_woppbs_1bit.rs:665-697).  The FFT's butterfly
 * schedule is fixed (see or_fft_*) so that the GPU product can be compared bit-exactly.
 */
#ifndef TFHE_ORACLE_H
#define TFHE_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    double re, im;
} or_c64;

/* WopbsParameters of src/tfhe/shortint_woppbs_1bit/parameters.rs */
typedef struct {
    int n;      /* lwe_dimension */
    int k;      /* glwe_dimension */
    int N;      /* polynomial_size */
    int pbs_l, pbs_b;
    int ks_l, ks_b;
    int cbs_l, cbs_b;
    int pfks_l, pfks_b;
    double lwe_std, glwe_std, pfks_std;
    uint64_t max_noise_sq;
    int model; /* 0: WoP-PBS models (ids 0-4); 2: shortint_1bit (id 5): pfpksk holds the packing
                * keyswitch key [n][pfks_l][(k+1)N], (pfks_l, pfks_b) = (ks_l, ks_b) */
} or_params;

/* 0 = params_sqrd_lvl_1 (:29), 1 = _4 (:77), 2 = _64 (:125), 3 = _256 (:173),
 * 4 = shortint_woppbs_8bit params() (shortint_woppbs_8bit.rs:39-86),
 * 5 = shortint_1bit PARAMS (src/tfhe/shortint_1bit.rs:62-83) */
int or_params_get(int id, or_params *out);

/* ---------------- randomness (keygen spec shared with the product) ---------- */
void or_chacha20_block(const uint8_t key[32], uint64_t nonce, uint64_t counter, uint8_t out[64]);
void or_chacha20_stream(const uint8_t key[32], uint64_t nonce, uint64_t counter, uint8_t *out,
                        size_t len);

/* ---------------- torus helpers ---------------- */
uint64_t or_closest_representable(uint64_t x, int base_log, int levels);
/* digits[lev-1] = digit of level lev (lev = 1 is the most significant). */
void or_decompose(uint64_t x, int base_log, int levels, int64_t *digits);
uint64_t or_from_torus(double x);
uint64_t or_pbs_modulus_switch(uint64_t x, int N);
void or_monomial_mul(const uint64_t *in, uint64_t *out, int N, int64_t degree); /* out = in * X^degree */
void or_negacyclic_mul_exact(const uint64_t *a, const int64_t *b, uint64_t *out, int N);
uint64_t or_encode_bit(uint64_t bit);
uint64_t or_decode_bit(uint64_t x);

/* ---------------- FFT ---------------- */
typedef struct or_fft or_fft;
or_fft *or_fft_new(int N);
void or_fft_free(or_fft *f);
void or_fft_fwd_int(const or_fft *f, const int64_t *poly, or_c64 *out);
void or_fft_fwd_torus(const or_fft *f, const uint64_t *poly, or_c64 *out);
void or_fft_add_bwd_torus(const or_fft *f, const or_c64 *in, uint64_t *out);
/* plain forward/inverse DFT of M = N/2 points in the product's digit-reversed order (tests) */
/* the blind rotation's fused-twiddle transform for N = 512 (tfhe_oracle.c) */
void *or_lf_plan_new(void);
void or_lf_plan_free(void *plan);
void or_lf_fwd(const void *plan, const int64_t *poly, or_c64 *X);
void or_lf_bwd_add(const void *plan, const or_c64 *Y, uint64_t *out);
void or_lf_e2(const void *plan, or_c64 *e2 /*[256]*/);
/* ... and for N = 1024 (the 8-bit model's PBS); or_lf_any_free frees either plan */
void *or_lf1k_plan_new(void);
void or_lf1k_fwd(const void *plan, const int64_t *poly, or_c64 *X);
void or_lf1k_bwd_add(const void *plan, const or_c64 *Y, uint64_t *out);
void or_lf1k_e2(const void *plan, or_c64 *e2 /*[512]*/);
void or_lf_any_free(void *plan);
/* the constants in the product's table layouts (tests/native/lf_tables_test.cpp) */
void or_lf_table(const void *plan, double *t /*[1700]*/);
void or_lf1k_table(const void *plan, double *t /*[3788]*/);
void or_fft_raw_fwd(const or_fft *f, or_c64 *z);
void or_fft_raw_inv(const or_fft *f, or_c64 *z);

/* ---------------- keys ---------------- */
typedef struct {
    or_params p;
    uint64_t *lwe_sk;  /* [n] bits */
    uint64_t *glwe_sk; /* [k*N] bits; as LWE key of dimension K = k*N */
} or_client_key;

typedef struct {
    or_params p;
    uint64_t *ksk;    /* [K][ks_l][n+1] */
    uint64_t *bsk;    /* [n][pbs_l][k+1][(k+1)*N] standard domain */
    uint64_t *pfpksk; /* [k+1][K+1][pfks_l][(k+1)*N] */
    or_c64 *bsk_f;    /* [n][pbs_l][k+1][k+1][N/2] Fourier domain */
    or_fft *fft;
    void *lf;         /* params_sqrd_lvl_64 and the 8-bit model's set: the blind rotation's fused-twiddle
                         transform (lf_plan / lf1k_plan), and bsk_f holds the BSK spectrum times conj(E2);
                         NULL otherwise */
} or_server_key;

int or_gen_keys(int param_id, const uint8_t seed[32], int threads, or_client_key **ck,
                or_server_key **sk);
/* Build a server key from raw standard-domain arrays (copied). */
or_server_key *or_server_key_from_raw(int param_id, const uint64_t *ksk, const uint64_t *bsk,
                                      const uint64_t *pfpksk);
/* The same with an explicit blind-rotation transform: OR_TRANSFORM_PRODUCT = what the product runs (the
 * fused-twiddle transforms for params_sqrd_lvl_64 and the 8-bit set, the radix schedule otherwise);
 * OR_TRANSFORM_RADIX = the radix-16 / radix-8 schedule shaped like tfhe-fft for every set (no conj(E2)
 * rescale of the Fourier BSK): the PBS-level tie of the fused transforms back to tfhe-fft's
 * (tests/test_oracle_transforms.py). */
#define OR_TRANSFORM_PRODUCT 0
#define OR_TRANSFORM_RADIX 1
or_server_key *or_server_key_from_raw_t(int param_id, const uint64_t *ksk, const uint64_t *bsk,
                                        const uint64_t *pfpksk, int transform);
void or_client_key_free(or_client_key *ck);
void or_server_key_free(or_server_key *sk);
size_t or_ksk_len(const or_params *p);
size_t or_bsk_len(const or_params *p);
size_t or_pfpksk_len(const or_params *p);

/* LWE encryption of bit under the big key (ClientKey::encrypt, shortint_woppbs_1bit.rs:200-217),
 * randomness from the (seed, index) stream of the keygen spec. out: [K+1] */
void or_encrypt_bit(const or_client_key *ck, const uint8_t seed[32], uint64_t index, uint64_t bit,
                    uint64_t *out);
uint64_t or_decrypt_bit(const or_client_key *ck, const uint64_t *ct);
uint64_t or_decrypt_phase(const or_client_key *ck, const uint64_t *ct);
uint64_t or_decrypt_small_phase(const or_client_key *ck, const uint64_t *ct);
void or_glwe_decrypt(const or_client_key *ck, const uint64_t *glwe, uint64_t *plain /*[N]*/);

/* ---------------- hot-path primitives ---------------- */
/* keyswitch_lwe_ciphertext: in [K+1] -> out [n+1] */
void or_keyswitch(const or_server_key *sk, const uint64_t *in, uint64_t *out);
/* add_external_product_assign: out += ggsw (Fourier, [lev][k+1][k+1][M]) [x] in */
void or_external_product_add(const or_server_key *sk, const or_c64 *ggsw, int levels, int base_log,
                             const uint64_t *in, uint64_t *out);
/* cmux(ct0, ct1, ggsw): ct1 -= ct0; ct0 += ggsw [x] ct1 */
void or_cmux(const or_server_key *sk, uint64_t *ct0, uint64_t *ct1, const or_c64 *ggsw, int levels,
             int base_log);
/* FourierLweBootstrapKey::bootstrap: lwe_in [n+1], acc [(k+1)N] (trivial LUT) -> lwe_out [K+1] */
void or_bootstrap(const or_server_key *sk, const uint64_t *lwe_in, const uint64_t *acc,
                  uint64_t *lwe_out);
/* wop_pbs::homomorphic_shift_boolean for cbs level `level` (1-based) */
void or_homomorphic_shift_boolean(const or_server_key *sk, const uint64_t *lwe_in, int level,
                                  uint64_t *lwe_out);
/* private_functional_keyswitch_lwe_ciphertext_into_glwe_ciphertext with key p: in [K+1] */
void or_pfks(const or_server_key *sk, int p, const uint64_t *in, uint64_t *glwe_out);
/* circuit_bootstrap_boolean: small lwe [n+1] -> GGSW [cbs_l][k+1][(k+1)N] standard domain */
void or_circuit_bootstrap_boolean(const or_server_key *sk, const uint64_t *lwe_in, uint64_t *ggsw);
/* fill_with_forward_fourier for a cbs GGSW -> [cbs_l][k+1][k+1][M] */
void or_ggsw_to_fourier(const or_server_key *sk, const uint64_t *ggsw, int levels, or_c64 *out);
/* vertical_packing: lut [n_polys*N] (n_polys = 2^tree), ggsw list [n_in] Fourier -> lwe [K+1] */
void or_vertical_packing(const or_server_key *sk, const uint64_t *lut, int n_polys,
                         const or_c64 *ggsws, int n_in, uint64_t *lwe_out);
/* FheContext::circuit_bootstrap: bits [n_in][K+1], lut [n_out][small_len], out [n_out][K+1] */
void or_circuit_bootstrap(const or_server_key *sk, const uint64_t *bits, int n_in,
                          const uint64_t *lut, int n_out, uint64_t *out);

/* circuit_bootstrap_boolean_vertical_packing on small-key bits [n_in][n+1] (no keyswitch) */
void or_cbs_vp_small(const or_server_key *sk, const uint64_t *bits, int n_in, const uint64_t *lut, int n_out,
                     uint64_t *out);

/* ---------------- 8-bit model (param id 4: shortint_woppbs_8bit.rs:39-86) ---------------- */
void or_encrypt_small_bit(const or_client_key *ck, const uint8_t seed[32], uint64_t index, uint64_t bit,
                          uint64_t *out /*[n+1]*/);
uint64_t or_decrypt_small_bit(const or_client_key *ck, const uint64_t *ct);
void or_encrypt_int(const or_client_key *ck, const uint8_t seed[32], uint64_t index, uint64_t value,
                    uint64_t *out /*[K+1]*/);
uint64_t or_decrypt_int(const or_client_key *ck, const uint64_t *ct);
void or_generate_lut_without_padding(int N, const uint64_t *f_table /*[256]*/, uint64_t *out /*[max(N,256)]*/);
void or_extract_bits(const or_server_key *sk, const uint64_t *lwe_in, int delta_log, int nbits, uint64_t *out);
/* ---------------- shortint_1bit model (param id 5: src/tfhe/shortint_1bit.rs) ---------------- */
/* shortint encrypt / decrypt, message modulus 2, carry 1, EncryptionKeyChoice::Small: [n+1] */
void or_s1_encrypt(const or_client_key *ck, const uint8_t seed[32], uint64_t index, uint64_t bit, uint64_t *out);
uint64_t or_s1_decrypt(const or_client_key *ck, const uint64_t *ct);
/* test_vector_from_cleartext_fn (:349-373): trivial GLWE, boxes f(0) / f(1) rotated left by N/4 */
void or_s1_tv_from_fn(int k, int N, uint64_t f0, uint64_t f1, uint64_t *glwe);
/* keyswitch_lwe_ciphertext_into_glwe_ciphertext with the packing keyswitch key: [n+1] -> [(k+1)N] */
void or_s1_pks(const or_server_key *sk, const uint64_t *in, uint64_t *glwe);
/* keyswitch_lwe_ciphertext_list_and_pack_in_glwe_ciphertext (FheContext::packing_keyswitch :240-254) */
void or_s1_pack(const or_server_key *sk, const uint64_t *cts, int count, uint64_t *glwe);
/* test_vector_from_ciphertexts (:392-492) */
void or_s1_tv_from_cts(const or_server_key *sk, const uint64_t *ct0, const uint64_t *ct1, uint64_t *glwe);
/* FheContext::bootstrap / bootstrap_assign (:257-291): PBS with a test vector, then keyswitch back to the small key */
void or_s1_bootstrap(const or_server_key *sk, const uint64_t *in, const uint64_t *tv, uint64_t *out);
/* calculate_multivariate_function (:538-547, apply_selectors_rec :549-576) over bits [nbits][n+1] (MSB first) with the test vectors of
 * generate_multivariate_test_vector (:519-536) for f_table [2^nbits] (0/1 values) */
void or_s1_multivariate(const or_server_key *sk, const uint64_t *bits, int nbits, const uint64_t *f_table,
                        uint64_t *out);
void or_bootstrap_with_lut8(const or_server_key *sk, const uint64_t *bits, const uint64_t *lut, uint64_t *out);
void or_gf_256_mul_terms(uint8_t b, int coef[8][8]);
void or_mix_column_terms(int coef[32][32]);
void or_sub_bytes8(const or_server_key *sk, const uint64_t *state, int n_bytes, int threads, uint64_t *out);
void or_aes8_encrypt_block(const or_server_key *sk, const uint64_t *rk, const uint64_t *block, int rounds,
                           int threads, uint64_t *out);

/* generate_multivariate_luts: f_table[1<<input_bits]; out [output_bits][N << tree_bits] */
size_t or_lut_small_len(int N, int input_bits);
void or_generate_lut(int N, int input_bits, int output_bits, const uint64_t *f_table, uint64_t *out);

/* ---------------- AES (fhe_sbox_gal_mul_pbs) ---------------- */
/* encrypt_block_for_rounds on ciphertext arrays: rk [44*32][K+1], block [128][K+1] (MSB-first
 * bits, block byte order), out [128][K+1]. threads: worker threads over the 16 bytes. */
void or_aes_encrypt_block(const or_server_key *sk, const uint64_t *rk, const uint64_t *block,
                          int rounds, int threads, uint64_t *out);
/* one AES round of the FHE driver, exposed for the CPU baseline: SubBytes+GF for `n_bytes` bytes
 * of a state (threads over bytes). */
void or_sub_bytes_gal_mul(const or_server_key *sk, const uint64_t *state_bytes, int n_bytes,
                          int threads, uint64_t *out /*[n_bytes][24][K+1]*/);
/* plain AES (plain.rs:75-132 semantics incl. reduced rounds with rk[40..44] last) */
void or_plain_key_schedule(const uint8_t key[16], uint8_t rk[176]);
void or_plain_encrypt_block(const uint8_t rk[176], const uint8_t in[16], int rounds, uint8_t out[16]);
uint8_t or_gf_256_mul_quirk(uint8_t a, uint8_t b);
extern const uint8_t or_sbox[256];

#ifdef __cplusplus
}
#endif
#endif
