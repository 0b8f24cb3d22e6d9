// extern "C" boundary (include/tfhe_aes_gpu.h).  Each entry point maps a reference trait method
// or tfhe-rs call to the host model (model.cpp) and the device Engine (kernels.hip); panics of the
// reference become status codes, HIP failures TAE_E_HIP.
#include <hip/hip_runtime.h>

#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "../../include/tfhe_aes_gpu.h"
#include "client.hpp"
#include "engine.hpp"
#include "cplx.hpp"
#include "model.hpp"

struct tae_client_key {
    tae::ClientKey ck;
};
struct tae_context {
    std::unique_ptr<tae::Context> ctx;
};
struct tae_bit {
    tae::BitCt b;
};
struct tae_lut {
    tae::Lut l;
};

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

template <class F>
int guarded(F &&fn) {
    try {
        fn();
        return TAE_OK;
    } catch (const tae::ModelError &e) {
        return fail(e.code, e.msg);
    } catch (const tae::HipError &e) {
        return fail(TAE_E_HIP, e.msg);
    } catch (const std::bad_alloc &) {
        return fail(TAE_E_ARG, "out of host memory");
    } catch (const std::exception &e) {
        return fail(TAE_E_PARAM, e.what());
    }
}

void require(bool cond, const char *msg) {
    if (!cond) throw tae::ModelError{TAE_E_ARG, msg};
}

tae::Params params_of(int param_set) {
    tae::Params p;
    if (!tae::get_params(param_set, p)) throw tae::ModelError{TAE_E_PARAM, "unknown parameter set"};
    return p;
}

void fill(tae_params *o, const tae::Params &p) {
    *o = {p.n, p.k, p.N, p.pbs_l, p.pbs_b, p.ks_l, p.ks_b, p.cbs_l, p.cbs_b, p.pfks_l, p.pfks_b,
          p.lwe_std, p.glwe_std, p.pfks_std, p.max_noise_sq, p.model};
}

void require_device(int device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        throw tae::ModelError{TAE_E_NODEV, "no GPU available: the HIP path has no CPU fallback"};
    if (device < 0 || device >= count) throw tae::ModelError{TAE_E_NODEV, "device index out of range"};
}

std::vector<const tae::BitCt *> unwrap(const tae_bit *const *bits, size_t n) {
    std::vector<const tae::BitCt *> v(n);
    for (size_t i = 0; i < n; i++) {
        require(bits[i] != nullptr, "null bit handle");
        v[i] = &bits[i]->b;
    }
    return v;
}

// run `fn(d_in, d_out, d_aux)` with host staging when mem == TAE_MEM_HOST.  `aux` (aux_bytes, may
// be null) is a second input in the same memory kind, staged the same way (a LUT).
template <class TI, class TO, class F>
void staged(tae_context const *ctx, const TI *in, size_t in_bytes, TO *out, size_t out_bytes, int mem, F fn,
            const uint64_t *aux = nullptr, size_t aux_bytes = 0) {
    tae::Context &c = *ctx->ctx;
    std::lock_guard<std::mutex> g(c.mutex());
    tae::Engine &e = c.engine();
    tae::hip_check(hipSetDevice(e.device()), "hipSetDevice");
    struct Dev {
        void *p = nullptr;
        ~Dev() {
            if (p) hipFree(p);
        }
    } daux;
    if (aux && mem != TAE_MEM_DEVICE) {
        tae::hip_check(hipMalloc(&daux.p, std::max<size_t>(aux_bytes, 16)), "hipMalloc");
        tae::hip_check(hipMemcpyAsync(daux.p, aux, aux_bytes, hipMemcpyHostToDevice, e.stream()), "upload aux");
        aux = static_cast<const uint64_t *>(daux.p);
    }
    auto call = [&](const TI *a, TO *b) { fn(a, b, aux); };
    if (mem == TAE_MEM_DEVICE) {
        e.order_after_caller();
        call(in, out);
        e.synchronize();
        return;
    }
    void *di = nullptr, *dout = nullptr;
    tae::hip_check(hipMalloc(&di, std::max<size_t>(in_bytes, 16)), "hipMalloc");
    if (hipMalloc(&dout, std::max<size_t>(out_bytes, 16)) != hipSuccess) {
        hipFree(di);
        throw tae::HipError{"hipMalloc"};
    }
    try {
        // everything on the engine stream, in order.  The output is cleared first: not every stage
        // writes every word (tae_stage_pfks_ggsw fills only the rows of the requested level), and the
        // caller must get zeros there, not uninitialized device memory.
        tae::hip_check(hipMemcpyAsync(di, in, in_bytes, hipMemcpyHostToDevice, e.stream()), "upload");
        tae::hip_check(hipMemsetAsync(dout, 0, out_bytes, e.stream()), "clear output");
        call(static_cast<const TI *>(di), static_cast<TO *>(dout));
        tae::hip_check(hipMemcpyAsync(out, dout, out_bytes, hipMemcpyDeviceToHost, e.stream()), "download");
        e.synchronize();
    } catch (...) {
        hipFree(di);
        hipFree(dout);
        throw;
    }
    hipFree(di);
    hipFree(dout);
}

void emit(const std::vector<tae::BitCt> &res, tae_bit **out) {
    for (size_t i = 0; i < res.size(); i++) out[i] = new tae_bit{res[i]};
}

}  // namespace

extern "C" {

const char *tae_last_error(void) { return g_last_error.c_str(); }
const char *tae_version(void) { return "tfhe-aes-2_amd 0.1 (gfx950)"; }

int tae_device_count(int *count) {
    return guarded([&] {
        require(count, "null");
        *count = 0;
        if (hipGetDeviceCount(count) != hipSuccess) *count = 0;
    });
}

int tae_get_params(int param_set, tae_params *out) {
    return guarded([&] {
        require(out, "null");
        fill(out, params_of(param_set));
    });
}

int tae_bit_len(int param_set, size_t *len) {
    return guarded([&] {
        require(len, "null");
        const tae::Params p = params_of(param_set);
        *len = p.bit_len();
    });
}

int tae_server_key_sizes(int param_set, size_t *ksk_len, size_t *bsk_len, size_t *pfpksk_len) {
    return guarded([&] {
        const tae::Params p = params_of(param_set);
        if (ksk_len) *ksk_len = p.ksk_len();
        if (bsk_len) *bsk_len = p.bsk_len();
        if (pfpksk_len) *pfpksk_len = p.pfpksk_len();
    });
}

int tae_generate_keys_raw(int param_set, const uint8_t seed[32], int threads, tae_client_key **client_key,
                          uint64_t *ksk, uint64_t *bsk, uint64_t *pfpksk) {
    return guarded([&] {
        require(seed && client_key, "null argument");
        const tae::Params p = params_of(param_set);
        auto ck = std::make_unique<tae_client_key>();
        tae::ServerKeyRaw sk;
        tae::generate_keys(p, seed, threads, ck->ck, sk);
        if (ksk) std::memcpy(ksk, sk.ksk.data(), sk.ksk.size() * 8);
        if (bsk) std::memcpy(bsk, sk.bsk.data(), sk.bsk.size() * 8);
        if (pfpksk) std::memcpy(pfpksk, sk.pfpksk.data(), sk.pfpksk.size() * 8);
        *client_key = ck.release();
    });
}

int tae_generate_keys(int param_set, const uint8_t seed[32], int device, int threads, tae_client_key **client_key,
                      tae_context **context) {
    return guarded([&] {
        require(seed && client_key && context, "null argument");
        const tae::Params p = params_of(param_set);
        require_device(device);
        auto ck = std::make_unique<tae_client_key>();
        tae::ServerKeyRaw sk;
        tae::generate_keys(p, seed, threads, ck->ck, sk);
        auto ctx = std::make_unique<tae_context>();
        ctx->ctx = std::make_unique<tae::Context>(std::make_unique<tae::Engine>(sk, device));
        *client_key = ck.release();
        *context = ctx.release();
    });
}

int tae_client_key_from_seed(int param_set, const uint8_t seed[32], tae_client_key **client_key) {
    return guarded([&] {
        require(seed && client_key, "null argument");
        auto ck = std::make_unique<tae_client_key>();
        tae::generate_client_key(params_of(param_set), seed, ck->ck);
        *client_key = ck.release();
    });
}

extern "C++" {
namespace tae {
namespace keyio {
void save(const char *path, const Params &p, int param_set, const ClientKey *ck, const uint64_t *ksk,
          const uint64_t *bsk, const uint64_t *pfpksk);
void load(const char *path, int *param_set, uint32_t *flags, ClientKey *ck, uint64_t *ksk, uint64_t *bsk,
          uint64_t *pfpksk);
}  // namespace keyio
}  // namespace tae
}

int tae_keys_save(const char *path, int param_set, const tae_client_key *client_key, const uint64_t *ksk,
                  const uint64_t *bsk, const uint64_t *pfpksk) {
    return guarded([&] {
        require(path, "null path");
        const tae::Params p = params_of(param_set);
        if (client_key) {
            const tae::Params &q = client_key->ck.p;
            require(q.n == p.n && q.k == p.k && q.N == p.N && q.model == p.model,
                    "client key does not belong to the parameter set");
        }
        tae::keyio::save(path, p, param_set, client_key ? &client_key->ck : nullptr, ksk, bsk, pfpksk);
    });
}

int tae_keys_file_info(const char *path, int *param_set, int *flags) {
    return guarded([&] {
        require(path && param_set && flags, "null argument");
        uint32_t fl = 0;
        tae::keyio::load(path, param_set, &fl, nullptr, nullptr, nullptr, nullptr);
        *flags = (int)fl;
    });
}

int tae_keys_load(const char *path, tae_client_key **client_key, uint64_t *ksk, uint64_t *bsk, uint64_t *pfpksk) {
    return guarded([&] {
        require(path, "null path");
        require(client_key || ksk || bsk || pfpksk, "nothing to load");
        int ps = 0;
        uint32_t fl = 0;
        std::unique_ptr<tae_client_key> ck = client_key ? std::make_unique<tae_client_key>() : nullptr;
        tae::keyio::load(path, &ps, &fl, ck ? &ck->ck : nullptr, ksk, bsk, pfpksk);
        if (client_key) *client_key = ck.release();
    });
}

int tae_context_create_raw(int param_set, int device, const uint64_t *ksk, const uint64_t *bsk,
                           const uint64_t *pfpksk, int mem, tae_context **context) {
    return guarded([&] {
        require(ksk && bsk && pfpksk && context, "null argument");
        const tae::Params p = params_of(param_set);
        require_device(device);
        auto ctx = std::make_unique<tae_context>();
        if (mem == TAE_MEM_DEVICE) {
            ctx->ctx = std::make_unique<tae::Context>(std::make_unique<tae::Engine>(p, device, ksk, bsk, pfpksk));
        } else {
            tae::ServerKeyRaw sk;
            sk.p = p;
            sk.ksk.assign(ksk, ksk + p.ksk_len());
            sk.bsk.assign(bsk, bsk + p.bsk_len());
            sk.pfpksk.assign(pfpksk, pfpksk + p.pfpksk_len());
            ctx->ctx = std::make_unique<tae::Context>(std::make_unique<tae::Engine>(sk, device));
        }
        *context = ctx.release();
    });
}

void tae_context_free(tae_context *ctx) { delete ctx; }
void tae_client_key_free(tae_client_key *ck) { delete ck; }

int tae_client_key_secrets(const tae_client_key *ck, uint64_t *lwe_sk, uint64_t *glwe_sk) {
    return guarded([&] {
        require(ck, "null");
        if (lwe_sk) std::memcpy(lwe_sk, ck->ck.lwe_sk.data(), ck->ck.lwe_sk.size() * 8);
        if (glwe_sk) std::memcpy(glwe_sk, ck->ck.glwe_sk.data(), ck->ck.glwe_sk.size() * 8);
    });
}

int tae_context_params(const tae_context *ctx, tae_params *out) {
    return guarded([&] {
        require(ctx && out, "null");
        fill(out, ctx->ctx->params());
    });
}

int tae_encrypt(const tae_client_key *ck, uint64_t bit, tae_bit **out) {
    return guarded([&] {
        require(ck && out, "null");
        if (bit > 1) throw tae::ModelError{TAE_E_ARG, "cleartext out of bounds: " + std::to_string(bit)};
        auto &c = const_cast<tae_client_key *>(ck)->ck;
        auto b = std::make_unique<tae_bit>();
        b->b.ct.assign(c.bit_len(), 0);
        c.encrypt_model_bit_at(bit, tae::kAutoIndexBase + c.next_index.fetch_add(1), b->b.ct.data());
        // BitCt::fresh (1-bit model: noise^2 1 + a new component id; 8-bit: NoiseLevel::NOMINAL)
        b->b.noise = c.p.model == 8   ? tae::NoiseLevel{1, {}}
                     : c.p.model == 2 ? tae::NoiseLevel{}  // shortint_1bit: unchecked adds, nothing tracked
                                      : tae::NoiseLevel::with_noise_level(1, tae::next_ct_id());
        b->b.max_noise_sq = c.p.max_noise_sq;
        *out = b.release();
    });
}

int tae_decrypt(const tae_client_key *ck, const tae_bit *bit, uint64_t *out) {
    return guarded([&] {
        require(ck && bit && out, "null");
        require(bit->b.ct.size() == ck->ck.bit_len(), "ciphertext size mismatch");
        *out = ck->ck.decrypt_model_bit(bit->b.ct.data());
    });
}

int tae_trivial(const tae_context *ctx, uint64_t bit, tae_bit **out) {
    return guarded([&] {
        require(ctx && out, "null");
        *out = new tae_bit{ctx->ctx->trivial(bit)};
    });
}

// Resolve the encryption indices of a raw call: TAE_INDEX_AUTO reserves `count` fresh indices from
// the key's counter (the region tae_encrypt uses); an explicit range must lie below kAutoIndexBase.
static uint64_t raw_index_range(const tae_client_key *ck, size_t count, uint64_t start_index) {
    if (start_index == TAE_INDEX_AUTO) return tae::kAutoIndexBase + const_cast<tae_client_key *>(ck)->ck.next_index.fetch_add(count);
    require(start_index < tae::kAutoIndexBase && count <= tae::kAutoIndexBase - start_index,
            "explicit encryption indices must lie below 2^63 (use TAE_INDEX_AUTO for fresh ones)");
    return start_index;
}

int tae_encrypt_bits_raw(const tae_client_key *ck, const uint8_t *bits, size_t count, uint64_t start_index,
                         uint64_t *out) {
    return guarded([&] {
        require(ck && (bits || !count) && (out || !count), "null");
        for (size_t i = 0; i < count; i++) require(bits[i] < 2, "cleartext out of bounds");
        const uint64_t first = raw_index_range(ck, count, start_index);
        const size_t L = ck->ck.bit_len();
        for (size_t i = 0; i < count; i++) ck->ck.encrypt_model_bit_at(bits[i], first + i, out + i * L);
    });
}

int tae_encrypt_ints_raw(const tae_client_key *ck, const uint8_t *values, size_t count, uint64_t start_index,
                         uint64_t *out) {
    return guarded([&] {
        require(ck && (values || !count) && (out || !count), "null");
        const uint64_t first = raw_index_range(ck, count, start_index);
        const size_t L = ck->ck.p.big_len();
        for (size_t i = 0; i < count; i++) ck->ck.encrypt_int_at(values[i], first + i, out + i * L);
    });
}

int tae_decrypt_ints_raw(const tae_client_key *ck, const uint64_t *cts, size_t count, uint8_t *values) {
    return guarded([&] {
        require(ck && (cts || !count) && (values || !count), "null");
        const size_t L = ck->ck.p.big_len();
        for (size_t i = 0; i < count; i++) values[i] = (uint8_t)ck->ck.decrypt_int(cts + i * L);
    });
}

int tae_decrypt_bits_raw(const tae_client_key *ck, const uint64_t *cts, size_t count, uint8_t *bits) {
    return guarded([&] {
        require(ck && (cts || !count) && (bits || !count), "null");
        const size_t L = ck->ck.bit_len();
        for (size_t i = 0; i < count; i++) bits[i] = (uint8_t)ck->ck.decrypt_model_bit(cts + i * L);
    });
}

int tae_bit_clone(const tae_bit *bit, tae_bit **out) {
    return guarded([&] {
        require(bit && out, "null");
        *out = new tae_bit{bit->b};
    });
}

void tae_bit_free(tae_bit *bit) { delete bit; }

int tae_bit_xor_assign(tae_bit *lhs, const tae_bit *rhs) {
    return guarded([&] {
        require(lhs && rhs, "null");
        lhs->b.xor_assign(rhs->b);
    });
}

int tae_bit_noise_level(const tae_bit *bit, uint64_t *nl) {
    return guarded([&] {
        require(bit && nl, "null");
        *nl = bit->b.noise.noise_level_squared;
    });
}

int tae_bit_data(const tae_bit *bit, uint64_t *out, size_t len) {
    return guarded([&] {
        require(bit && out, "null");
        require(len == bit->b.ct.size(), "length mismatch");
        std::memcpy(out, bit->b.ct.data(), len * 8);
    });
}

int tae_bit_from_data(const tae_context *ctx, const uint64_t *data, size_t len, uint64_t nl, tae_bit **out) {
    return guarded([&] {
        require(ctx && data && out, "null");
        require(len == ctx->ctx->bit_len(), "length mismatch");
        *out = new tae_bit{ctx->ctx->wrap(std::vector<uint64_t>(data, data + len), nl)};
    });
}

int tae_generate_lookup_table(const tae_context *ctx, int input_bits, int output_bits, const uint64_t *f_values,
                              tae_lut **out) {
    return guarded([&] {
        require(ctx && f_values && out, "null");
        *out = new tae_lut{ctx->ctx->generate_lookup_table(input_bits, output_bits, f_values)};
    });
}

void tae_lut_free(tae_lut *lut) { delete lut; }

int tae_generate_multivariate_luts(int poly_size, int input_bits, int output_bits, const uint64_t *f_values,
                                   uint64_t *out, size_t out_len) {
    return guarded([&] {
        require(f_values && out, "null");
        require(poly_size >= 2 && (poly_size & (poly_size - 1)) == 0 && poly_size <= (1 << 16),
                "polynomial size must be a power of two");
        require(input_bits >= 1 && input_bits <= 16 && output_bits >= 1 && output_bits <= 64, "bit counts out of range");
        require(out_len == tae::lut_small_len(poly_size, input_bits) * (size_t)output_bits, "length mismatch");
        tae::generate_lut(poly_size, input_bits, output_bits, f_values, out);
    });
}

int tae_xor_batch(const tae_context *ctx, uint64_t *lhs, const uint64_t *rhs, size_t count,
                  const uint64_t *lhs_noise_sq, const uint64_t *rhs_noise_sq, uint64_t *out_noise_sq, int mem) {
    return guarded([&] {
        require(ctx && (lhs || !count) && (rhs || !count), "null");
        require((lhs_noise_sq == nullptr) == (rhs_noise_sq == nullptr), "give both noise arrays or neither");
        const uint64_t max_sq = ctx->ctx->params().max_noise_sq;
        if (lhs_noise_sq) {
            // BitXorAssign's noise rule (shortint_woppbs_1bit.rs:134-142, NoiseLevelWithComponents::add
            // + MaxNoiseLevel::validate): squared noise levels add and must stay <= max_noise_level^2
            for (size_t i = 0; i < count; i++) {
                const uint64_t l = lhs_noise_sq[i], r = rhs_noise_sq[i];
                const uint64_t s = l + r;
                if (l > max_sq || r > max_sq - l)  // no wrap-around: l + r <= max_sq exactly
                    throw tae::ModelError{TAE_E_NOISE, "NoiseTooBig: noise level squared " + std::to_string(s) +
                                                           " above " + std::to_string(max_sq) + " at element " +
                                                           std::to_string(i)};
            }
        }
        const size_t words = count * ctx->ctx->bit_len();
        if (count) {
            tae::Context &c = *ctx->ctx;
            std::lock_guard<std::mutex> g(c.mutex());
            tae::Engine &e = c.engine();
            tae::hip_check(hipSetDevice(e.device()), "hipSetDevice");
            if (mem == TAE_MEM_DEVICE) {
                e.order_after_caller();
                e.lwe_add(lhs, rhs, words);
                e.synchronize();
            } else {
                void *da = nullptr, *db = nullptr;
                tae::hip_check(hipMalloc(&da, words * 8), "hipMalloc");
                if (hipMalloc(&db, words * 8) != hipSuccess) {
                    hipFree(da);
                    throw tae::HipError{"hipMalloc"};
                }
                try {
                    tae::hip_check(hipMemcpyAsync(da, lhs, words * 8, hipMemcpyHostToDevice, e.stream()), "upload");
                    tae::hip_check(hipMemcpyAsync(db, rhs, words * 8, hipMemcpyHostToDevice, e.stream()), "upload");
                    e.lwe_add(static_cast<uint64_t *>(da), static_cast<const uint64_t *>(db), words);
                    tae::hip_check(hipMemcpyAsync(lhs, da, words * 8, hipMemcpyDeviceToHost, e.stream()), "download");
                    e.synchronize();
                } catch (...) {
                    hipFree(da);
                    hipFree(db);
                    throw;
                }
                hipFree(da);
                hipFree(db);
            }
        }
        if (out_noise_sq && lhs_noise_sq)
            for (size_t i = 0; i < count; i++) out_noise_sq[i] = lhs_noise_sq[i] + rhs_noise_sq[i];
    });
}

int tae_lut_data(const tae_lut *lut, uint64_t *out, size_t len, size_t *needed) {
    return guarded([&] {
        require(lut, "null");
        if (needed) *needed = lut->l.data.size();
        if (out) {
            require(len == lut->l.data.size(), "length mismatch");
            std::memcpy(out, lut->l.data.data(), len * 8);
        }
    });
}

int tae_circuit_bootstrap(const tae_context *ctx, const tae_bit *const *bits, size_t n_bits, const tae_lut *lut,
                          tae_bit **out) {
    return guarded([&] {
        require(ctx && bits && lut && out, "null");
        emit(ctx->ctx->circuit_bootstrap(unwrap(bits, n_bits), lut->l), out);
    });
}

int tae_circuit_bootstrap_raw(const tae_context *ctx, const uint64_t *bits, size_t groups, int n_in,
                              const tae_lut *lut, uint64_t *out, int mem) {
    return guarded([&] {
        require(ctx && bits && lut && out, "null");
        ctx->ctx->circuit_bootstrap_raw(bits, groups, n_in, lut->l, out, mem == TAE_MEM_DEVICE);
    });
}

int tae_bootstrap_from_bits_raw(const tae_context *ctx, const uint64_t *bits, size_t groups, const tae_lut *lut,
                                uint64_t *out, int mem) {
    return guarded([&] {
        require(ctx && bits && lut && out, "null");
        ctx->ctx->bootstrap_from_bits_raw(bits, groups, lut->l, out, mem == TAE_MEM_DEVICE);
    });
}

int tae_extract_bits_raw(const tae_context *ctx, const uint64_t *ints, size_t groups, uint64_t *out, int mem) {
    return guarded([&] {
        require(ctx && ints && out, "null");
        ctx->ctx->extract_bits_raw(ints, groups, out, mem == TAE_MEM_DEVICE);
    });
}

int tae_aes_key_schedule_raw(const tae_context *ctx, const uint64_t *key, uint64_t *expanded, int mem) {
    return guarded([&] {
        require(ctx && key && expanded, "null");
        ctx->ctx->aes_key_schedule_raw(key, expanded, mem == TAE_MEM_DEVICE);
    });
}

int tae_aes_encrypt_block_for_rounds(const tae_context *ctx, const tae_bit *const *expanded_key,
                                     const tae_bit *const *block, int rounds, tae_bit **out) {
    return guarded([&] {
        require(ctx && expanded_key && block && out, "null");
        emit(ctx->ctx->aes_encrypt_blocks(unwrap(expanded_key, 44 * 32), unwrap(block, 128), 1, rounds), out);
    });
}

int tae_aes_encrypt_blocks(const tae_context *ctx, const tae_bit *const *expanded_key, const tae_bit *const *blocks,
                           size_t n_blocks, int rounds, tae_bit **out) {
    return guarded([&] {
        require(ctx && expanded_key && blocks && out, "null");
        emit(ctx->ctx->aes_encrypt_blocks(unwrap(expanded_key, 44 * 32), unwrap(blocks, 128 * n_blocks), n_blocks,
                                          rounds),
             out);
    });
}

int tae_aes_key_schedule(const tae_context *ctx, const tae_bit *const *key, tae_bit **expanded) {
    return guarded([&] {
        require(ctx && key && expanded, "null");
        emit(ctx->ctx->aes_key_schedule(unwrap(key, 128)), expanded);
    });
}

int tae_aes_encrypt_blocks_raw(const tae_context *ctx, const uint64_t *rk, const uint64_t *blocks, size_t n_blocks,
                               int rounds, uint64_t *out, int mem) {
    return guarded([&] {
        require(ctx && rk && blocks && out, "null");
        ctx->ctx->aes_encrypt_blocks_raw(rk, blocks, n_blocks, rounds, out, mem == TAE_MEM_DEVICE);
    });
}

int tae_aes_sbox_pbs_encrypt_blocks(const tae_context *ctx, const tae_bit *const *expanded_key,
                                    const tae_bit *const *blocks, size_t n_blocks, int rounds, tae_bit **out) {
    return guarded([&] {
        require(ctx && expanded_key && blocks && out, "null");
        emit(ctx->ctx->aes_encrypt_blocks(unwrap(expanded_key, 44 * 32), unwrap(blocks, 128 * n_blocks), n_blocks,
                                          rounds, tae::AesDriver::SboxPbs),
             out);
    });
}

int tae_aes_sbox_pbs_key_schedule(const tae_context *ctx, const tae_bit *const *key, tae_bit **expanded) {
    return guarded([&] {
        require(ctx && key && expanded, "null");
        emit(ctx->ctx->aes_key_schedule(unwrap(key, 128), tae::AesDriver::SboxPbs), expanded);
    });
}

int tae_aes_sbox_pbs_encrypt_blocks_raw(const tae_context *ctx, const uint64_t *rk, const uint64_t *blocks,
                                        size_t n_blocks, int rounds, uint64_t *out, int mem) {
    return guarded([&] {
        require(ctx && rk && blocks && out, "null");
        ctx->ctx->aes_encrypt_blocks_raw(rk, blocks, n_blocks, rounds, out, mem == TAE_MEM_DEVICE,
                                         tae::AesDriver::SboxPbs);
    });
}

int tae_aes_sbox_pbs_key_schedule_raw(const tae_context *ctx, const uint64_t *key, uint64_t *expanded, int mem) {
    return guarded([&] {
        require(ctx && key && expanded, "null");
        ctx->ctx->aes_key_schedule_raw(key, expanded, mem == TAE_MEM_DEVICE, tae::AesDriver::SboxPbs);
    });
}

int tae_aes_noise_schedule_check(int param_set, int driver, int rounds) {
    return guarded([&] {
        const tae::Params p = params_of(param_set);
        require(driver == TAE_DRIVER_GAL_MUL || driver == TAE_DRIVER_SBOX_PBS, "unknown driver");
        if (rounds < 1 || rounds > 10) throw tae::ModelError{TAE_E_PARAM, "rounds must be in 1..=10"};
        if (p.model == 2) return;  // shortint_1bit: unchecked adds, no bookkeeping to fail
        std::vector<tae::NoiseLevel> rk(44 * 32), blk(128);
        for (auto &x : rk) x = p.model == 8 ? tae::NoiseLevel{1, {}} : tae::NoiseLevel::with_noise_level(1, tae::next_ct_id());
        for (auto &x : blk) x = p.model == 8 ? tae::NoiseLevel{1, {}} : tae::NoiseLevel::with_noise_level(1, tae::next_ct_id());
        if (p.model == 8)
            tae::aes8_noise_schedule(rk, blk, rounds, p.max_noise_sq);
        else if (driver == TAE_DRIVER_SBOX_PBS)
            tae::sbox_pbs_noise_schedule(rk, blk, rounds, p.max_noise_sq);
        else
            tae::aes_noise_schedule(rk, blk, rounds, p.max_noise_sq);
    });
}


/* ---- shortint_1bit model ---- */
int tae_s1_test_vector_from_fn(int param_set, uint64_t f0, uint64_t f1, uint64_t *tv) {
    return guarded([&] {
        require(tv, "null");
        const tae::Params p = params_of(param_set);
        require(p.model == 2, "test vectors belong to the shortint_1bit parameter set");
        require(f0 <= 1 && f1 <= 1, "function values must be 0 or 1");
        tae::s1_test_vector(p, f0, f1, tv);
    });
}

int tae_s1_bootstrap(const tae_context *ctx, const uint64_t *in, size_t count, const uint64_t *tvs, size_t n_tv,
                     uint64_t *out, int mem) {
    return guarded([&] {
        require(ctx && (in || !count) && tvs && (out || !count), "null");
        if (count) ctx->ctx->s1_bootstrap_raw(in, count, tvs, n_tv, out, mem == TAE_MEM_DEVICE);
    });
}

int tae_s1_packing_keyswitch(const tae_context *ctx, const uint64_t *cts, size_t count, uint64_t *glwe, int mem) {
    return guarded([&] {
        require(ctx && cts && glwe, "null");
        ctx->ctx->s1_packing_keyswitch_raw(cts, count, glwe, mem == TAE_MEM_DEVICE);
    });
}

int tae_s1_test_vectors_from_ciphertexts(const tae_context *ctx, const uint64_t *ct0, const uint64_t *ct1, size_t count,
                                         uint64_t *tvs, int mem) {
    return guarded([&] {
        require(ctx && (count == 0 || (ct0 && ct1 && tvs)), "null");
        if (count) ctx->ctx->s1_test_vectors_from_ciphertexts_raw(ct0, ct1, count, tvs, mem == TAE_MEM_DEVICE);
    });
}

int tae_s1_multivariate(const tae_context *ctx, const uint64_t *bits, size_t groups, int nbits,
                        const uint64_t *f_tables, int n_fn, uint64_t *out, int mem) {
    return guarded([&] {
        require(ctx && f_tables && (groups == 0 || (bits && out)), "null");
        if (groups) ctx->ctx->s1_multivariate_raw(bits, groups, nbits, f_tables, n_fn, out, mem == TAE_MEM_DEVICE);
    });
}

int tae_stage_keyswitch(const tae_context *ctx, const uint64_t *in, size_t count, uint64_t *out, int mem) {
    return guarded([&] {
        require(ctx && in && out, "null");
        const auto &p = ctx->ctx->params();
        staged(ctx, in, count * p.big_len() * 8, out, count * p.small_len() * 8, mem,
               [&](const uint64_t *a, uint64_t *b, const uint64_t *) { ctx->ctx->engine().keyswitch(a, b, count); });
    });
}

int tae_stage_pbs_shift_boolean(const tae_context *ctx, const uint64_t *small, size_t count, int level, uint64_t *big,
                                int mem) {
    return guarded([&] {
        require(ctx && small && big, "null");
        const auto &p = ctx->ctx->params();
        require(level >= 1 && level <= p.cbs_l, "level out of range");
        staged(ctx, small, count * p.small_len() * 8, big, count * p.big_len() * 8, mem,
               [&](const uint64_t *a, uint64_t *b, const uint64_t *) { ctx->ctx->engine().pbs_shift_boolean(a, b, count, level); });
    });
}

int tae_stage_bootstrap(const tae_context *ctx, const uint64_t *small, size_t count, const uint64_t *lut_glwe,
                        uint64_t *big, int mem) {
    return guarded([&] {
        require(ctx && small && lut_glwe && big, "null");
        const auto &p = ctx->ctx->params();
        staged(
            ctx, small, count * p.small_len() * 8, big, count * p.big_len() * 8, mem,
            [&](const uint64_t *a, uint64_t *b, const uint64_t *lut) { ctx->ctx->engine().bootstrap(a, lut, b, count, 0, 0); },
            lut_glwe, p.glwe_len() * 8);
    });
}

int tae_stage_pfks_ggsw(const tae_context *ctx, const uint64_t *big, size_t count, int level, uint64_t *ggsw, int mem) {
    return guarded([&] {
        require(ctx && big && ggsw, "null");
        const auto &p = ctx->ctx->params();
        require(level >= 1 && level <= p.cbs_l, "level out of range");
        staged(ctx, big, count * p.big_len() * 8, ggsw, count * p.cbs_ggsw_len() * 8, mem,
               [&](const uint64_t *a, uint64_t *b, const uint64_t *) { ctx->ctx->engine().pfks_into_ggsw(a, b, count, level); });
    });
}

int tae_stage_ggsw_fourier(const tae_context *ctx, const uint64_t *ggsw, size_t count, double *ggsw_f, int mem) {
    return guarded([&] {
        require(ctx && ggsw && ggsw_f, "null");
        const auto &p = ctx->ctx->params();
        staged(ctx, ggsw, count * p.cbs_ggsw_len() * 8, ggsw_f, count * p.cbs_ggsw_fourier_len() * 16, mem,
               [&](const uint64_t *a, double *b, const uint64_t *) {
                   ctx->ctx->engine().ggsw_to_fourier(a, reinterpret_cast<tae::cplx *>(b), count);
               });
    });
}

int tae_stage_vertical_packing(const tae_context *ctx, const double *ggsw_f, size_t groups, int n_in,
                               const uint64_t *lut, int n_out, uint64_t *out, int mem) {
    return guarded([&] {
        require(ctx && ggsw_f && lut && out, "null");
        const auto &p = ctx->ctx->params();
        staged(
            ctx, ggsw_f, groups * n_in * p.cbs_ggsw_fourier_len() * 16, out, groups * n_out * p.big_len() * 8, mem,
            [&](const double *a, uint64_t *b, const uint64_t *l) {
                ctx->ctx->engine().vertical_packing(reinterpret_cast<const tae::cplx *>(a), groups, n_in, l, n_out, b);
            },
            lut, (size_t)n_out * p.N * 8);
    });
}

int tae_synchronize(const tae_context *ctx) {
    return guarded([&] {
        require(ctx, "null");
        ctx->ctx->engine().synchronize();
    });
}

int tae_set_caller_stream(tae_context *ctx, void *stream) {
    return guarded([&] {
        require(ctx, "null");
        std::lock_guard<std::mutex> g(ctx->ctx->mutex());  // the context's entry points hold the same lock
        ctx->ctx->engine().set_caller_stream((hipStream_t)stream);
    });
}

int tae_set_timing(const tae_context *ctx, int on) {
    return guarded([&] {
        require(ctx, "null");
        require(on >= 0 && on <= 2, "timing mode is 0, 1 or 2");
        ctx->ctx->engine().set_timing(on);
    });
}

int tae_last_stage_times_v4(const tae_context *ctx, double *v12) {
    return guarded([&] {
        require(ctx && v12, "null");
        const auto &t = ctx->ctx->engine().last_times();
        const double v[12] = {t.keyswitch, t.pbs,    t.pfks,         t.ggsw_fft, t.vertical_packing,
                              t.extract,   t.linear, (double)t.pbs_launches, t.pbs_main, t.pbs_main_cts,
                              t.pbs_clock_launches ? t.pbs_clock_ghz_sum / t.pbs_clock_launches : 0.0,
                              (double)t.pbs_clock_launches};
        for (int i = 0; i < 12; i++) v12[i] = v[i];
    });
}

int tae_last_stage_times_v2(const tae_context *ctx, float *ms8) {
    return guarded([&] {
        require(ctx && ms8, "null");
        const auto &t = ctx->ctx->engine().last_times();
        const float v[8] = {t.keyswitch, t.pbs, t.pfks, t.ggsw_fft, t.vertical_packing, t.extract, t.linear,
                            (float)t.pbs_launches};
        for (int i = 0; i < 8; i++) ms8[i] = v[i];
    });
}

int tae_last_stage_times_v3(const tae_context *ctx, double *v10) {
    return guarded([&] {
        require(ctx && v10, "null");
        const auto &t = ctx->ctx->engine().last_times();
        const double v[10] = {t.keyswitch, t.pbs,    t.pfks,         t.ggsw_fft, t.vertical_packing,
                              t.extract,   t.linear, (double)t.pbs_launches, t.pbs_main, t.pbs_main_cts};
        for (int i = 0; i < 10; i++) v10[i] = v[i];
    });
}

int tae_last_stage_times(const tae_context *ctx, float *ms5) {
    return guarded([&] {
        require(ctx && ms5, "null");
        const auto &t = ctx->ctx->engine().last_times();
        ms5[0] = t.keyswitch;
        ms5[1] = t.pbs;
        ms5[2] = t.pfks;
        ms5[3] = t.ggsw_fft;
        ms5[4] = t.vertical_packing;
    });
}

}  // extern "C"
