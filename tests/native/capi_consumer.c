/* A plain C99 consumer of the C-ABI (include/tfhe_aes_gpu.h): the calls a foreign-language binding of
 * the reference's ShortintWoppbs1BitSboxGalMulPbsAesEncrypt path makes, with no
 * Python, torch or HIP types involved.  Built with gcc -std=c99 -pedantic -Werror by
 * tests/test_capi_consumer.py, which also checks that the header is valid C.
 *
 *   capi_consumer host  -- host-only entry points (parameters, static noise schedule, client key,
 *                          encrypt / decrypt round trip); without a GPU, context creation must fail
 *                          loudly with TAE_E_NODEV (there is no CPU fallback)
 *   capi_consumer gpu   -- the above, then FIPS-197 C.1 end to end on device 0: FHE key schedule
 *                          (fhe_sbox_gal_mul_pbs.rs:134-164) on the encrypted key, 10 rounds of the
 *                          GalMul driver on the encrypted block, decrypted to 69c4e0d8...b4c55a
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tfhe_aes_gpu.h"

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        int rc_ = (x);                                                                            \
        if (rc_ != TAE_OK) {                                                                      \
            fprintf(stderr, "%s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_, tae_last_error()); \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)
#define EXPECT(c)                                                              \
    do {                                                                       \
        if (!(c)) {                                                            \
            fprintf(stderr, "%s:%d: expectation failed: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                          \
        }                                                                      \
    } while (0)

/* a byte is 8 bit ciphertexts, MSB first (src/util.rs:33-42) */
static void bytes_to_bits(const uint8_t *bytes, size_t n, uint8_t *bits) {
    size_t i;
    int b;
    for (i = 0; i < n; i++)
        for (b = 0; b < 8; b++) bits[8 * i + b] = (uint8_t)((bytes[i] >> (7 - b)) & 1);
}

static void bits_to_bytes(const uint8_t *bits, size_t n, uint8_t *bytes) {
    size_t i;
    int b;
    for (i = 0; i < n; i++) {
        bytes[i] = 0;
        for (b = 0; b < 8; b++) bytes[i] = (uint8_t)((bytes[i] << 1) | (bits[8 * i + b] & 1));
    }
}

static const uint8_t SEED[32] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16,
                                 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32};

static int host_checks(void) {
    tae_params p;
    size_t len = 0, i;
    tae_client_key *ck = NULL;
    uint8_t bits[16], back[16];
    uint64_t *cts;
    EXPECT(tae_version() != NULL);
    CHECK(tae_get_params(TAE_PARAMS_SQRD_LVL_64, &p));
    EXPECT(p.n == 677 && p.k == 4 && p.N == 512 && p.model == 1);
    CHECK(tae_bit_len(TAE_PARAMS_SQRD_LVL_64, &len));
    EXPECT(len == (size_t)p.k * p.N + 1);
    EXPECT(tae_get_params(99, &p) == TAE_E_PARAM || tae_get_params(99, &p) == TAE_E_ARG);
    /* the reference's noise rules, decided before any device work */
    CHECK(tae_aes_noise_schedule_check(TAE_PARAMS_SQRD_LVL_64, TAE_DRIVER_GAL_MUL, 10));
    EXPECT(tae_aes_noise_schedule_check(TAE_PARAMS_SQRD_LVL_64, TAE_DRIVER_SBOX_PBS, 2) == TAE_E_INDEP);
    /* client key from a seed, raw encrypt / decrypt on the host */
    CHECK(tae_client_key_from_seed(TAE_PARAMS_SQRD_LVL_64, SEED, &ck));
    cts = (uint64_t *)malloc(sizeof(uint64_t) * 16 * len);
    EXPECT(cts != NULL);
    for (i = 0; i < 16; i++) bits[i] = (uint8_t)((0xA53Cu >> i) & 1);
    CHECK(tae_encrypt_bits_raw(ck, bits, 16, 1000, cts));
    CHECK(tae_decrypt_bits_raw(ck, cts, 16, back));
    EXPECT(memcmp(bits, back, 16) == 0);
    /* an index range reaching 2^63 is refused (indices select the ChaCha streams) */
    EXPECT(tae_encrypt_bits_raw(ck, bits, 16, (uint64_t)1 << 63, cts) == TAE_E_ARG);
    free(cts);
    tae_client_key_free(ck);
    return 0;
}

static int no_fallback_check(void) {
    tae_client_key *ck = NULL;
    tae_context *ctx = NULL;
    const int rc = tae_generate_keys(TAE_PARAMS_SQRD_LVL_64, SEED, 0, 1, &ck, &ctx);
    EXPECT(rc == TAE_E_NODEV);
    EXPECT(ck == NULL && ctx == NULL);
    printf("no GPU: %s\n", tae_last_error());
    return 0;
}

static int fips197_c1(void) {
    static const uint8_t key[16] = {0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07,
                                    0x08, 0x09, 0x0a, 0x0b, 0x0c, 0x0d, 0x0e, 0x0f};
    static const uint8_t pt[16] = {0x00, 0x11, 0x22, 0x33, 0x44, 0x55, 0x66, 0x77,
                                   0x88, 0x99, 0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff};
    static const uint8_t want[16] = {0x69, 0xc4, 0xe0, 0xd8, 0x6a, 0x7b, 0x04, 0x30,
                                     0xd8, 0xcd, 0xb7, 0x80, 0x70, 0xb4, 0xc5, 0x5a};
    tae_client_key *ck = NULL;
    tae_context *ctx = NULL;
    size_t len = 0;
    uint8_t bits[128], got_bits[128], got[16];
    uint64_t *key_cts, *rk, *blk, *out;
    int i;
    CHECK(tae_bit_len(TAE_PARAMS_SQRD_LVL_64, &len));
    CHECK(tae_generate_keys(TAE_PARAMS_SQRD_LVL_64, SEED, 0, 16, &ck, &ctx));
    key_cts = (uint64_t *)malloc(sizeof(uint64_t) * 128 * len);
    rk = (uint64_t *)malloc(sizeof(uint64_t) * 44 * 32 * len);
    blk = (uint64_t *)malloc(sizeof(uint64_t) * 128 * len);
    out = (uint64_t *)malloc(sizeof(uint64_t) * 128 * len);
    EXPECT(key_cts && rk && blk && out);
    bytes_to_bits(key, 16, bits);
    CHECK(tae_encrypt_bits_raw(ck, bits, 128, 0, key_cts));
    CHECK(tae_aes_key_schedule_raw(ctx, key_cts, rk, TAE_MEM_HOST));
    bytes_to_bits(pt, 16, bits);
    CHECK(tae_encrypt_bits_raw(ck, bits, 128, 128, blk));
    CHECK(tae_aes_encrypt_blocks_raw(ctx, rk, blk, 1, 10, out, TAE_MEM_HOST));
    CHECK(tae_decrypt_bits_raw(ck, out, 128, got_bits));
    bits_to_bytes(got_bits, 16, got);
    printf("FIPS-197 C.1 under FHE: ");
    for (i = 0; i < 16; i++) printf("%02x", got[i]);
    printf("\n");
    EXPECT(memcmp(got, want, 16) == 0);
    free(key_cts);
    free(rk);
    free(blk);
    free(out);
    tae_context_free(ctx);
    tae_client_key_free(ck);
    return 0;
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "host";
    if (host_checks()) return 1;
    if (strcmp(mode, "host") == 0) {
        int count = 0;
        if (tae_device_count(&count) != TAE_OK || count == 0) {
            if (no_fallback_check()) return 1;
        }
    } else if (strcmp(mode, "gpu") == 0) {
        if (fips197_c1()) return 1;
    } else {
        fprintf(stderr, "usage: %s host|gpu\n", argv[0]);
        return 2;
    }
    printf("OK\n");
    return 0;
}
