// Device engine: server keys resident in HBM and the batched hot-path stages as HIP kernels.
//
// Reference hot path: FheContext::circuit_bootstrap
// (src/tfhe/shortint_woppbs_1bit.rs:292-336) = per input bit extract_dual_bit_from_bit
// (:339-363 -> tfhe extract_bits = one LWE keyswitch), then tfhe
// circuit_bootstrap_boolean_vertical_packing (homomorphic_shift_boolean PBS, k+1 private
// functional keyswitches into a GGSW, forward FFT of the GGSW, vertical-packing blind rotation,
// sample extraction).  Every stage here is batched over all bits of all SBOXes of a round.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "client.hpp"
#include "cplx.hpp"
#include "kslots.hpp"
#include "params.hpp"

namespace tae {

struct HipError {
    std::string msg;
};

void hip_check(hipError_t e, const char *what);

// Timing of the most recent batched call, per stage (ms, HIP events on the engine stream).
struct StageTimes {
    float keyswitch = 0, pbs = 0, pfks = 0, ggsw_fft = 0, vertical_packing = 0, extract = 0, linear = 0;
    int pbs_launches = 0;  // CBS-level PBS launches (one homomorphic_shift_boolean batch each)
    // the throughput blind-rotation kernel alone (br512x4 launches inside the PBS stage, without the
    // br512lat remainder) and the ciphertexts those launches processed
    float pbs_main = 0;
    double pbs_main_cts = 0;
    // clock mode (set_timing(2)): median effective shader clock over the workgroups of each throughput
    // blind-rotation launch (br512x4, or br1024 with two ciphertexts per workgroup), summed over launches
    double pbs_clock_ghz_sum = 0;
    int pbs_clock_launches = 0;
};
enum Stage { ST_KS = 0, ST_PBS, ST_PFKS, ST_FFT, ST_VP, ST_EXTRACT, ST_LINEAR, ST_PBS_MAIN };

class Engine {
  public:
    // Uploads the standard-domain keys and converts the BSK to the Fourier domain on device.
    Engine(const ServerKeyRaw &keys, int device);
    // Attach to keys already resident on this device (e.g. broadcast over RCCL); the standard
    // BSK is converted in place into an engine-owned Fourier buffer.  Pointers must stay valid.
    Engine(const Params &p, int device, const uint64_t *d_ksk, const uint64_t *d_bsk,
           const uint64_t *d_pfpksk);
    ~Engine();
    Engine(const Engine &) = delete;
    Engine &operator=(const Engine &) = delete;

    const Params &params() const { return p_; }
    int device() const { return device_; }
    hipStream_t stream() const { return stream_; }

    // ---- batched stages, all pointers device-resident ----
    // keyswitch_lwe_ciphertext: [B][K+1] -> [B][n+1]
    void keyswitch(const uint64_t *d_in, uint64_t *d_out, size_t B);
    // homomorphic_shift_boolean at cbs level `level`: [B][n+1] -> [B][K+1]
    void pbs_shift_boolean(const uint64_t *d_small, uint64_t *d_big, size_t B, int level);
    // generic FourierLweBootstrapKey::bootstrap with LUT GLWEs [(k+1)N]: ciphertext b takes
    // d_lut_glwe + (b % lut_mod) (k+1)N (lut_mod 1: one LUT for the batch; lut_mod > 1, a test vector per
    // ciphertext, runs on br512x4<7, true, 6> for shortint_1bit and on the generic pbs_kernel otherwise)
    void bootstrap(const uint64_t *d_small, const uint64_t *d_lut_glwe, uint64_t *d_big, size_t B,
                   uint64_t body_add, uint64_t out_add, size_t lut_mod = 1);
    // private functional keyswitches of level `level`: [B][K+1] -> GGSW rows of that level in
    // d_ggsw [B][cbs_l][k+1][(k+1)N]
    void pfks_into_ggsw(const uint64_t *d_big, uint64_t *d_ggsw, size_t B, int level);
    // fill_with_forward_fourier: [B][cbs_l][k+1][(k+1)N] -> [B][cbs_l][k+1][k+1][M]
    void ggsw_to_fourier(const uint64_t *d_ggsw, cplx *d_ggsw_f, size_t B);
    // vertical_packing for each group of n_in GGSWs: d_ggsw_f [G][n_in][...], d_lut
    // [n_out][N], out [G][n_out][K+1]
    void vertical_packing(const cplx *d_ggsw_f, size_t G, int n_in, const uint64_t *d_lut, int n_out,
                          uint64_t *d_out);
    // LUTs with input_bits > log2 N: CMux tree over the first `tree` GGSWs, then the blind rotation
    void vertical_packing_tree(const cplx *d_ggsw_f, size_t G, int n_in, int tree, const uint64_t *d_lut, int n_out,
                               uint64_t *d_out);
    // FheContext::circuit_bootstrap over G groups: bits [G][n_in][K+1] -> [G][n_out][K+1]
    void circuit_bootstrap(const uint64_t *d_bits, size_t G, int n_in, const uint64_t *d_lut,
                           int n_out, uint64_t *d_out);
    // circuit_bootstrap_boolean_vertical_packing on small-key bits (no keyswitch):
    // [G][n_in][n+1] -> [G][n_out][K+1]  (8-bit model: WopbsKey::circuit_bootstrapping_vertical_packing)
    void cbs_vp(const uint64_t *d_small_bits, size_t G, int n_in, const uint64_t *d_lut, int n_out,
                uint64_t *d_out);
    // tfhe wop_pbs::extract_bits: big-key [B][K+1] -> small-key bits [B][nbits][n+1], MSB first
    // (8-bit model extract_bits_from_ciphertext, shortint_woppbs_8bit.rs:268-296)
    void extract_bits(const uint64_t *d_in, size_t B, int delta_log, int nbits, uint64_t *d_out);
    // Byte::bootstrap_with_lut (fhe_impls/shortint_woppbs_8bit.rs:37-42) over G bytes:
    // [G][8][n+1] -> [G][8][n+1] through one 8-bit int ciphertext per byte
    void bootstrap_bytes8(const uint64_t *d_bytes, size_t G, const uint64_t *d_lut, uint64_t *d_out);
    // fhe_sbox_pbs::encrypt_block_for_rounds over nb blocks of small-key bits (8-bit model):
    // rk [44*32][n+1], blocks [nb][128][n+1]
    void aes8_encrypt_blocks(const uint64_t *d_rk, const uint64_t *d_blocks, size_t nb, int rounds,
                             uint64_t *d_out);

    // ---- AES driver (fhe_sbox_gal_mul_pbs::encrypt_block_for_rounds over many blocks) ----
    // rk [44*32][K+1] (expanded key words, word-major, MSB-first bits), blocks [nb][128][K+1]
    void aes_encrypt_blocks(const uint64_t *d_rk, const uint64_t *d_blocks, size_t nb, int rounds,
                            uint64_t *d_out);

    // ---- shortint_1bit model (src/tfhe/shortint_1bit.rs; param set SHORTINT_1BIT) ----
    // FheContext::bootstrap / bootstrap_assign (:257-291): PBS with test vector d_tvs + (b % lut_mod) (k+1)N, then the keyswitch
    // back to the small key: [B][n+1] -> [B][n+1]
    void s1_bootstrap(const uint64_t *d_in, const uint64_t *d_tvs, size_t lut_mod, uint64_t *d_out, size_t B);
    // keyswitch_lwe_ciphertext_into_glwe_ciphertext with the packing key, per ciphertext: [B][n+1] -> [B][(k+1)N]
    void s1_pks(const uint64_t *d_in, size_t B, uint64_t *d_out);
    // test_vector_from_ciphertexts (:392-492) over P pairs of packing keyswitches [2P][(k+1)N] -> [P][(k+1)N]
    void s1_tv_from_pks(const uint64_t *d_pks, size_t P, uint64_t *d_tv);
    // FheContext::packing_keyswitch (:240-254): count ciphertexts into one GLWE, #j at X^j
    void s1_pack(const uint64_t *d_in, int count, uint64_t *d_out);
    // calculate_multivariate_function (:538-547) / apply_selectors_rec (:549-576) for n_fn functions of the same nbits bits, over G groups:
    // bits [G][nbits][n+1] (MSB first), d_tvs [n_fn][2^(nbits-1)][(k+1)N] (generate_multivariate_test_vector)
    // -> [G][n_fn][n+1]; one batched bootstrap + packing step per selector level
    void s1_multivariate(const uint64_t *d_bits, size_t G, int nbits, const uint64_t *d_tvs, int n_fn, uint64_t *d_out);
    void s1_multivariate_chunk(const uint64_t *d_bits, size_t G, int nbits, const uint64_t *d_tvs, int n_fn,
                               uint64_t *d_out);
    // Shortint1BitSboxPbsAesEncrypt::encrypt_block_for_rounds over nb blocks: rk [44*32][n+1], blocks [nb][128][n+1]
    void s1_aes_encrypt_blocks(const uint64_t *d_rk, const uint64_t *d_blocks, size_t nb, int rounds, uint64_t *d_out);
    const uint64_t *s1_sbox_tvs() const { return d_s1_sbox_tv_; }  // [8][128][(k+1)N]
    const uint64_t *s1_identity_tv() const { return d_s1_id_tv_; }  // [(k+1)N]

    // ---- element-wise helpers ----
    void lwe_add(uint64_t *d_a, const uint64_t *d_b, size_t count);  // a += b (count u64)

    void synchronize();
    // Device-resident caller buffers (TAE_MEM_DEVICE) may have been written on any stream of the
    // caller (torch's current stream, an RCCL stream): wait for all device work before the engine's
    // non-blocking stream reads them.
    void order_after_caller();
    // TAE_MEM_DEVICE ordering: nullptr (default) = device-wide synchronize; otherwise the engine stream
    // waits on an event recorded on this caller stream (no host sync, other streams not waited for)
    void set_caller_stream(hipStream_t s) { caller_stream_ = s; }
    const StageTimes &last_times() const { return times_; }
    // 0 off, 1 HIP-event stage times, 2 stage times + in-kernel clock stamps of the blind rotations
    // (a diagnostic mode: each stamped launch is read back synchronously)
    void set_timing(int mode) {
        timing_ = mode != 0;
        clock_ = mode == 2;
    }

    // scratch sizing: reserve buffers for a circuit_bootstrap of `bits` input bits
    void reserve(size_t bits, size_t outputs);

    const uint64_t *lut_galmul() const { return d_lut24_; }  // 8 -> 24 (S, 2S', 3S')
    const uint64_t *lut_sbox() const { return d_lut8_; }     // 8 -> 8 SBOX
    // 8-bit model LUTs without padding (SBOX, identity), [N]
    const uint64_t *lut8_sbox() const { return d_wlut_sbox_; }
    const uint64_t *lut8_identity() const { return d_wlut_id_; }

  private:
    void init_common();
    void bsk_to_fourier(const uint64_t *d_bsk_std);
    void *alloc(size_t bytes);
    template <class T>
    T *grow(T *&ptr, size_t &cap, size_t count);

    Params p_;
    int device_;
    hipStream_t stream_ = nullptr;
    hipStream_t caller_stream_ = nullptr;
    hipEvent_t caller_ev_ = nullptr;
    bool owns_keys_ = false;
    uint64_t *d_ksk_ = nullptr, *d_pfpksk_ = nullptr;
    cplx *d_bsk_f_ = nullptr;
    cplx *d_twist_ = nullptr, *d_untwist_ = nullptr, *d_w_ = nullptr;
    uint64_t *d_lut_shift_ = nullptr;  // per cbs level: trivial GLWE with body = -alpha
    uint64_t *d_lut24_ = nullptr, *d_lut8_ = nullptr;
    uint64_t *d_wlut_sbox_ = nullptr, *d_wlut_id_ = nullptr;  // 8-bit model
    uint64_t *d_lut_x_ = nullptr;                             // extract_bits accumulators [nbits][glwe]
    int lut_x_delta_ = -1, lut_x_bits_ = 0;
    uint64_t *d_xbuf_ = nullptr, *d_xsh_ = nullptr, *d_xks_ = nullptr, *d_xpbs_ = nullptr, *d_ints_ = nullptr;
    size_t cap_xbuf_ = 0, cap_xsh_ = 0, cap_xks_ = 0, cap_xpbs_ = 0, cap_ints_ = 0;
    int8_t mix_idx_[32][8] = {};
    // shortint_1bit: S-box / identity test vectors and tree-level scratch
    uint64_t *d_s1_sbox_tv_ = nullptr, *d_s1_id_tv_ = nullptr, *d_s1_in_ = nullptr, *d_s1_out_ = nullptr,
             *d_s1_pks_ = nullptr, *d_s1_tv_ = nullptr;
    size_t cap_s1_in_ = 0, cap_s1_out_ = 0, cap_s1_pks_ = 0, cap_s1_tv_ = 0;
    void require_s1() const;
    void cbs_vp_stages(const uint64_t *d_small_bits, size_t G, int n_in, const uint64_t *d_lut, int n_out,
                       uint64_t *d_out);
    // scratch
    uint64_t *d_small_ = nullptr, *d_big_ = nullptr, *d_ggsw_ = nullptr, *d_state_ = nullptr,
             *d_muls_ = nullptr;
    cplx *d_ggsw_f_ = nullptr;
    size_t cap_small_ = 0, cap_big_ = 0, cap_ggsw_ = 0, cap_ggsw_f_ = 0, cap_state_ = 0, cap_muls_ = 0;
    // stage timing (HIP events around each stage call on the engine stream, summed in collect_times)
    struct Span {
        hipEvent_t a, b;
        int stage;
    };
    std::vector<hipEvent_t> ev_pool_;
    size_t ev_used_ = 0;
    std::vector<Span> spans_;
    hipEvent_t next_event();
    template <class F>
    void timed(int stage, F fn);
    void collect_times();
    // int8 MFMA keyswitches (ksgemm.hpp): key limb matrices + digit scratch
    bool mfma_ks_ = false;
    // PFKS GEMM in the K layout (ksgemm.hpp KSlots) from pf_kl_min_ ciphertexts on, the 6-bit
    // row-tile limbs below (shorter K: 2.4x fewer K steps per tile, for batches too small to fill the
    // chip either way); TAE_PFKS_LAYOUT=k / rows forces one (the parity tests run both)
    bool pf_kl_ = false;
    long pf_kl_min_ = 2048;
    int kp_pf_kl_ = 0;
    ksgemm::KSlots pf_slots_;
    int8_t *d_pf_bt_kl_ = nullptr;
    uint64_t *d_pf_corr_ = nullptr;  // [ncols] digit-offset correction of the K layout
    uint32_t *d_pf_flags_ = nullptr;  // [B][words] clamped-digit flags of the K layout (kslots_build)
    size_t cap_pf_flags_ = 0;
    int8_t *d_pf_bt_ = nullptr, *d_ks_bt_ = nullptr, *d_digits_ = nullptr;
    size_t cap_digits_ = 0;
    int kp_pf_ = 0, kp_ks_ = 0;
    void prepare_mfma_keys();
    // batched N=1024, k=2 blind rotation (br1024.hpp) for this set's (levels, base_log), or nullptr
    void (*br1024_pbs_)(const uint64_t *, int, const uint64_t *, int, const cplx *, int, uint64_t *, long, uint64_t,
                        uint64_t, const cplx *, const cplx *, const cplx *, const double *, uint64_t *) = nullptr;
    decltype(br1024_pbs_) br1024_vp_ = nullptr;
    decltype(br1024_pbs_) br1024_pbs1_ = nullptr;  // one ciphertext per workgroup (small batches)
    decltype(br1024_pbs_) br1024_occ2_ = nullptr;  // A/B: one per workgroup, two workgroups per CU
    int br1024_pbs1_lp_ = 1;                       // its levels per pass
    bool lf1k_ = false;                            // the 8-bit model's PBS: the N = 1024 fused transform (lf1k.hpp)
    bool b1kw_ = false;                            // ... on br1024w (four ciphertexts per workgroup, ACC stash)
    uint64_t *d_acc_w_ = nullptr;                  // br1024w's ACC stash [B][k+1][N]
    size_t cap_acc_w_ = 0;
    // latency blind rotation, one ciphertext per 1024-thread workgroup (br1024lat.hpp), or nullptr
    void (*br1024lat_)(const uint64_t *, int, const uint64_t *, const cplx *, uint64_t *, long, uint64_t, uint64_t,
                       const cplx *, const double *) = nullptr;
    size_t br1024lat_lds_ = 0;
    bool x4_512_ = false;     // PBS N = 512, k = 4, 3 x 2^12 (lvl_64): br512x4 / br512lat on the fused transform
    bool x4_vp_ = false;      // ... and cbs 1 x 2^13: vertical packing on br512x4<1, false, 13>
    bool lf512_ = false;      // N = 512, k = 4: the fused transform, conj(E2)-rescaled BSK (oracle lf_set)
    bool x4_s1_ = false;      // shortint_1bit PBS 7 x 2^6: br512x4<7, true, 6> with per-ciphertext test vectors
    long lat_max_ = 256;      // batch size up to which br512lat runs (TAE_BR_LAT_MAX)
    bool p16_ = false;        // lvl_64 PBS batches on br512p16 (two ciphertexts per workgroup) instead of br512x4
                              // (TAE_PBS_KERNEL = p16 / x4)
    int num_cu_ = 256;
    double *d_lf_ = nullptr;  // the fused-twiddle transform's table (lf512.hpp: params_sqrd_lvl_64, lf1k.hpp: 8-bit)
    bool timing_ = false, clock_ = false;
    uint64_t *d_clk_ = nullptr;
    size_t cap_clk_ = 0;
    uint64_t *clock_buffer(size_t wgs);                   // nullptr unless clock mode is on
    void record_clock(const uint64_t *clk, size_t wgs);  // median GHz of one stamped launch
    StageTimes times_;
};

}  // namespace tae
