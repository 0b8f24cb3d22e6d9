// Parameter sets of the 1-bit WoP-PBS model, the 8-bit model's single set and the shortint_1bit model's.
// Reference: src/tfhe/shortint_woppbs_1bit/parameters.rs:29-205 (WopbsParameters +
// max_noise_level_squared).  Default for the AES path: params_sqrd_lvl_64 (main.rs:82-83).
#pragma once
#include <cstddef>
#include <cstdint>

namespace tae {

struct Params {
    int id;
    int n;  // lwe_dimension (small key)
    int k;  // glwe_dimension
    int N;  // polynomial_size
    int pbs_l, pbs_b;
    int ks_l, ks_b;
    int cbs_l, cbs_b;
    int pfks_l, pfks_b;
    double lwe_std, glwe_std, pfks_std;
    uint64_t max_noise_sq;  // 1-bit model: max noise^2; 8-bit model: shortint MaxNoiseLevel
    int model = 1;          // 1: shortint_woppbs_1bit (bits under the big key); 8: shortint_woppbs_8bit
                            //    (bits under the small key, bytes bootstrapped through an 8-bit int);
                            // 2: shortint_1bit (shortint bits under the small key, classic PBS with test
                            //    vectors; the third server key is the packing keyswitch key)

    int K() const { return k * N; }                    // big LWE dimension
    int M() const { return N / 2; }                    // Fourier coefficients per polynomial
    size_t big_len() const { return (size_t)K() + 1; }  // big LWE size
    size_t small_len() const { return (size_t)n + 1; }
    size_t glwe_len() const { return (size_t)(k + 1) * N; }
    size_t ksk_len() const { return (size_t)K() * ks_l * small_len(); }
    size_t bsk_len() const { return (size_t)n * pbs_l * (k + 1) * glwe_len(); }
    size_t bsk_fourier_len() const { return (size_t)n * pbs_l * (k + 1) * (k + 1) * M(); }
    size_t pfpksk_len() const {
        if (model == 2) return (size_t)n * pfks_l * glwe_len();  // packing keyswitch key [n][pfks_l][glwe]
        return (size_t)(k + 1) * big_len() * pfks_l * glwe_len();
    }
    size_t bit_len() const { return model == 1 ? big_len() : small_len(); }  // one bit ciphertext
    size_t cbs_ggsw_len() const { return (size_t)cbs_l * (k + 1) * glwe_len(); }
    size_t cbs_ggsw_fourier_len() const { return (size_t)cbs_l * (k + 1) * (k + 1) * M(); }
};

enum ParamSet { SQRD_LVL_1 = 0, SQRD_LVL_4 = 1, SQRD_LVL_64 = 2, SQRD_LVL_256 = 3, WOPPBS_8BIT = 4, SHORTINT_1BIT = 5 };

inline bool get_params(int id, Params &p) {
    switch (id) {
    case SQRD_LVL_1:  // parameters.rs:29-61
        p = {id, 671, 2, 1024, 2, 15, 4, 3, 1, 10, 1, 24,
             4.7280002450549286e-05, 3.162026630747649e-16, 3.162026630747649e-16, 1};
        return true;
    case SQRD_LVL_4:  // parameters.rs:77-109
        p = {id, 679, 2, 1024, 2, 15, 4, 3, 1, 11, 2, 16,
             4.7280002450549286e-05, 3.162026630747649e-16, 3.162026630747649e-16, 4};
        return true;
    case SQRD_LVL_64:  // parameters.rs:125-157
        p = {id, 677, 4, 512, 3, 12, 4, 3, 1, 13, 2, 16,
             4.7280002450549286e-05, 0.00000000000000022148688116005568,
             0.00000000000000022148688116005568, 64};
        return true;
    case SQRD_LVL_256:  // parameters.rs:173-205
        p = {id, 665, 2, 1024, 4, 9, 6, 2, 1, 14, 3, 12,
             4.7280002450549286e-05, 3.162026630747649e-16, 3.162026630747649e-16, 256};
        return true;
    case WOPPBS_8BIT:  // src/tfhe/shortint_woppbs_8bit.rs:39-86 (message modulus 256, carry 1,
                       // MaxNoiseLevel::new(11))
        p = {id, 785, 2, 1024, 6, 7, 8, 2, 4, 6, 3, 12,
             1.5140301927925663e-05, 0.00000000000000022148688116005568,
             0.00000000000000022148688116005568, 11, 8};
        return true;
    case SHORTINT_1BIT:  // src/tfhe/shortint_1bit.rs:62-83 (ClassicPBSParameters, "testing parameters":
                         // n 640, k 4, N 512, PBS 7 x 2^6, KS 2 x 2^6, message modulus 2, carry 1,
                         // MaxNoiseLevel 11, EncryptionKeyChoice::Small).  The packing keyswitch key of
                         // generate_keys_with_params (:186-196) takes (ks_l, ks_b) and the lwe noise: stored
                         // as (pfks_l, pfks_b, pfks_std).  No circuit bootstrap (cbs_l = 0).
        p = {id, 640, 4, 512, 7, 6, 2, 6, 0, 0, 2, 6,
             4.728000245054929e-7, 2.845267479601915e-15, 4.728000245054929e-7, 11, 2};
        return true;
    default:
        return false;
    }
}

}  // namespace tae
