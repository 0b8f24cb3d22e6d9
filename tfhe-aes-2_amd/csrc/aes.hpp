// AES-128 constants and byte-level helpers used by the FHE round driver.
// Reference: src/aes_128.rs (SBOX :18-35, RC :37-39, ROUNDS :16, gf_256_mul :42-56),
// src/aes_128/plain.rs:106-132 (key schedule, for host-side checks).
#pragma once
#include <cstdint>

namespace tae {

extern const uint8_t kSbox[256];
extern const uint8_t kRcon[11];
constexpr int kAesRounds = 10;

// gf_256_mul exactly as the reference writes it, including its reduction quirk (it XORs 0x1b
// when the high bit is CLEAR, aes_128.rs:50).  The x2/x3 LUT outputs inherit the quirk; the two
// 0x1b terms cancel inside every MixColumns output, so full AES stays correct.
uint8_t gf_256_mul(uint8_t a, uint8_t b);

// fhe_sbox_pbs::gf_256_mul (fhe_sbox_pbs.rs:33-53) on bits: the byte is shifted and XORed bit by
// bit (MSB-first, reduce by x^8 = x^4 + x^3 + x + 1).  terms[o][i] = how often input bit i is added
// into output bit o (LWE additions: nothing cancels).  mix_column_terms: MixColumns (:56-73) as
// a 32 x 32 map on one column, out byte r = 2 s_r + s_{r+3} + s_{r+2} + 3 s_{r+1}.
void gf_256_mul_bit_terms(uint8_t b, int terms[8][8]);
void mix_column_terms(int terms[32][32]);

// plain key expansion into 176 bytes (word-major), plain.rs:106-132
void plain_key_schedule(const uint8_t key[16], uint8_t rk[176]);

}  // namespace tae
