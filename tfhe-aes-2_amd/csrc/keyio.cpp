// On-disk key files.  The reference keeps keys in memory only (its tests regenerate them per run,
// SURVEY.md §8f-2); a service needs to persist a client key and ship server keys to evaluation
// nodes.  One self-describing little-endian file holds either or both:
//
//   "TAEKEY02"                     8-byte magic + format version
//   u32 param_set, u32 flags       flags: 1 = client key, 2 = server keys
//   [flags & 1] u8 seed[32], u64 next_index
//                                  the client key is re-derived from its seed (generate_client_key,
//                                  the same LWE_SK / GLWE_SK streams as keygen); next_index is the
//                                  encryption counter, so a reloaded key never reuses randomness
//   [flags & 2] u64 ksk_len, bsk_len, pfpksk_len, then the three standard-domain u64 arrays
//                                  (the lengths must equal tae_server_key_sizes(param_set))
//   u64 checksum                   word-wise FNV-1a over every preceding byte
//
// Version 01 (round 2 and earlier) stored a client counter whose tae_encrypt ciphertexts used the LOW
// indices [0, next_index); tae_encrypt now draws from 2^63 + next_index and explicit raw ranges may use
// anything below 2^63, so a reloaded 01 client key could reuse those streams.  01 files are therefore
// still read for their server keys, but a 01 file holding a client key is rejected (re-save it).
//
// A file is rejected (TAE_E_ARG) on a bad magic, unknown flags or parameter set, a size mismatch,
// truncation or a checksum mismatch; nothing is returned from a rejected file.
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>

#include "../../include/tfhe_aes_gpu.h"
#include "client.hpp"
#include "model.hpp"

namespace tae {
namespace keyio {

constexpr char kMagic[8] = {'T', 'A', 'E', 'K', 'E', 'Y', '0', '2'};
constexpr char kMagicV1[8] = {'T', 'A', 'E', 'K', 'E', 'Y', '0', '1'};
constexpr uint32_t kClient = 1, kServer = 2;

struct Hash {
    uint64_t h = 0xcbf29ce484222325ull;
    uint64_t pend = 0;  // bytes not yet folded (< 8), little-endian
    int npend = 0;
    void bytes(const void *p, size_t n) {
        const uint8_t *b = static_cast<const uint8_t *>(p);
        while (n && npend) {
            pend |= (uint64_t)*b++ << (8 * npend);
            n--;
            if (++npend == 8) word(pend), pend = 0, npend = 0;
        }
        for (; n >= 8; n -= 8, b += 8) {
            uint64_t w;
            std::memcpy(&w, b, 8);
            word(w);
        }
        for (; n; n--) pend |= (uint64_t)*b++ << (8 * npend++);
    }
    void word(uint64_t w) { h = (h ^ w) * 0x100000001b3ull; }
    uint64_t final() {
        if (npend) word(pend ^ ((uint64_t)npend << 56)), npend = 0, pend = 0;
        return h;
    }
};

struct File {
    FILE *f = nullptr;
    ~File() {
        if (f) fclose(f);
    }
};

[[noreturn]] void bad(const std::string &msg) { throw ModelError{TAE_E_ARG, "key file: " + msg}; }

void put(File &f, Hash &h, const void *p, size_t n) {
    h.bytes(p, n);
    if (fwrite(p, 1, n, f.f) != n) bad("write failed");
}

void get(File &f, Hash &h, void *p, size_t n) {
    if (fread(p, 1, n, f.f) != n) bad("truncated");
    h.bytes(p, n);
}

void skip(File &f, Hash &h, size_t n) {  // hashed, not kept
    std::unique_ptr<uint8_t[]> buf(new uint8_t[1 << 20]);
    while (n) {
        const size_t c = n < (1u << 20) ? n : (1u << 20);
        get(f, h, buf.get(), c);
        n -= c;
    }
}

void save(const char *path, const Params &p, int param_set, const ClientKey *ck, const uint64_t *ksk,
          const uint64_t *bsk, const uint64_t *pfpksk) {
    const bool server = ksk || bsk || pfpksk;
    if (server && !(ksk && bsk && pfpksk)) bad("server keys need ksk, bsk and pfpksk");
    if (!ck && !server) bad("nothing to save");
    File f;
    f.f = fopen(path, "wb");
    if (!f.f) bad(std::string("cannot create ") + path);
    Hash h;
    put(f, h, kMagic, 8);
    const uint32_t hdr[2] = {(uint32_t)param_set, (ck ? kClient : 0u) | (server ? kServer : 0u)};
    put(f, h, hdr, sizeof(hdr));
    if (ck) {
        put(f, h, ck->seed.data(), 32);
        const uint64_t next = ck->next_index.load();
        put(f, h, &next, 8);
    }
    if (server) {
        const uint64_t lens[3] = {p.ksk_len(), p.bsk_len(), p.pfpksk_len()};
        put(f, h, lens, sizeof(lens));
        put(f, h, ksk, lens[0] * 8);
        put(f, h, bsk, lens[1] * 8);
        put(f, h, pfpksk, lens[2] * 8);
    }
    const uint64_t sum = h.final();
    if (fwrite(&sum, 1, 8, f.f) != 8 || fflush(f.f) != 0) bad("write failed");
}

// Reads the header; with `out_*` set also the payload.  The checksum is verified before the call
// returns, so a caller only keeps what a valid file held (server arrays are written in place and
// must be discarded on error).
void load(const char *path, int *param_set, uint32_t *flags, ClientKey *ck, uint64_t *ksk, uint64_t *bsk,
          uint64_t *pfpksk) {
    File f;
    f.f = fopen(path, "rb");
    if (!f.f) bad(std::string("cannot open ") + path);
    Hash h;
    char magic[8];
    get(f, h, magic, 8);
    const bool v1 = std::memcmp(magic, kMagicV1, 8) == 0;
    if (!v1 && std::memcmp(magic, kMagic, 8) != 0) bad("not a TAEKEY02 file");
    uint32_t hdr[2];
    get(f, h, hdr, sizeof(hdr));
    Params p;
    if (!get_params((int)hdr[0], p)) bad("unknown parameter set");
    if (hdr[1] == 0 || (hdr[1] & ~(kClient | kServer))) bad("unknown flags");
    if (v1 && (hdr[1] & kClient))
        bad("legacy TAEKEY01 client key: its counter does not reserve the indices it used; re-save the key");
    *param_set = (int)hdr[0];
    *flags = hdr[1];
    const bool header_only = !ck && !ksk && !bsk && !pfpksk;
    uint8_t seed[32];
    uint64_t next = 0;
    if (hdr[1] & kClient) {
        get(f, h, seed, 32);
        get(f, h, &next, 8);
    }
    if (hdr[1] & kServer) {
        uint64_t lens[3];
        get(f, h, lens, sizeof(lens));
        if (lens[0] != p.ksk_len() || lens[1] != p.bsk_len() || lens[2] != p.pfpksk_len())
            bad("server key sizes do not match the parameter set");
        if (header_only) return;
        if (ksk || bsk || pfpksk) {
            if (!(ksk && bsk && pfpksk)) bad("ksk, bsk and pfpksk buffers are required together");
            get(f, h, ksk, lens[0] * 8);
            get(f, h, bsk, lens[1] * 8);
            get(f, h, pfpksk, lens[2] * 8);
        } else {
            skip(f, h, (lens[0] + lens[1] + lens[2]) * 8);
        }
    } else if (ksk || bsk || pfpksk) {
        bad("the file holds no server keys");
    }
    if (header_only) return;
    uint64_t sum;
    if (fread(&sum, 1, 8, f.f) != 8) bad("truncated");
    if (sum != h.final()) bad("checksum mismatch");
    char extra;
    if (fread(&extra, 1, 1, f.f) != 0) bad("trailing bytes");
    if (ck && !(hdr[1] & kClient)) bad("the file holds no client key");
    if ((hdr[1] & kClient) && ck) {
        generate_client_key(p, seed, *ck);
        ck->next_index.store(next);
    }
}

}  // namespace keyio
}  // namespace tae
