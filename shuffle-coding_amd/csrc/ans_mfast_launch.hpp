// ans_mfast_launch.hpp — launchers of the ans_mfast.hpp skeletons, shared by ans_codecs.hip
// (Uniform, LogUniform) and the Independent<Categorical> units ans_codecs_indep_{enc,dec}.hip,
// which hold that codec's many instantiations (norm range x renorm screen x symbol width) so
// they compile in parallel.
#pragma once

#include "ans_mfast.hpp"

namespace shuffle_coding {
namespace mfast {

inline unsigned mgrid(uint64_t nfull) { return static_cast<unsigned>((nfull + kLanes - 1) / kLanes); }

template <class M, typename Sym, int SPP, int kL = kLanes>
void menc(const M& md, const void* syms, const uint8_t* tids, uint64_t L, uint64_t nfull, uint8_t* slots, uint64_t cap,
          uint32_t* lens, uint32_t* st, ChunkInit ini, uint32_t lds, hipStream_t s) {
    k_menc<M, Sym, SPP, kL><<<static_cast<unsigned>((nfull + kL - 1) / kL), kL, lds, s>>>(
        md, static_cast<const Sym*>(syms), tids, L, nfull, slots, cap, lens, st, ini);
}
template <class M, typename Sym, int SPP, int kL = kLanes>
void mdec(const M& md, const uint8_t* in, uint64_t cap, const uint64_t* offs, const uint32_t* lens, const uint8_t* tids,
          uint64_t L, uint64_t nfull, int gen_kind, void* out, uint32_t* st, ChunkInit ini, uint32_t lds, hipStream_t s) {
    k_mdec<M, Sym, SPP, kL><<<static_cast<unsigned>((nfull + kL - 1) / kL), kL, lds, s>>>(
        md, in, cap, offs, lens, tids, L, nfull, gen_kind, static_cast<Sym*>(out), st, ini);
}

// An Independent<Categorical> set's fast-kernel images (built by ans_codecs.hip build_indep_fast).
struct IndepFast {
    bool usable = false;
    bool rare = false;  // some row needs the exact renorm screen (IndepModel<true>)
    uint32_t kmax = 0;  // most bytes one push emits
    int nr = 0;         // the tables' norm range (ans_fast.hpp kNormStd / kNormSmall / kNormBig)
    void* d_mem = nullptr;
    IndepModel<false> md;  // device pointers (every IndepModel instantiation has the same fields)
    // the 1,024-lane decoder's image (tables at LDS offset 0, DecLayout<kLanesW>), when the set fits
    // its 28 KiB; decodes of at least ncu * 1,024 chains use it (one such workgroup per CU)
    const uint4* dec_img_w = nullptr;
    uint32_t dec_bytes_w = 0;
    int ncu = 256;
    int lanes = 0;  // 0: by the call's size; 256 / 1,024: that layout where it exists (ans_gpu_tableset_lanes)
    bool lean = false, lean_w = false;  // IndepModel kLean for the 256- / 1,024-lane decoder image
    bool enc_wide = false;              // the encoder image fits the 1,024-lane layout (kEncTabW)
    // the 1,024-lane layouts when the call has the chains for one such workgroup per CU
    bool wide(uint64_t nfull) const { return lanes ? lanes == kLanesW : nfull >= static_cast<uint64_t>(ncu) * kLanesW; }
};

// the full chunks of a fixed-chunk Independent call (ans_codecs_indep_enc.hip / _dec.hip)
void indep_fast_encode(const IndepFast& f, const void* syms, int w, const uint8_t* tids, uint64_t L, uint64_t nfull,
                       uint8_t* slots, uint64_t cap, uint32_t* lens, uint32_t* st, ChunkInit ini, hipStream_t s);
void indep_fast_decode(const IndepFast& f, const uint8_t* in, uint64_t cap, const uint64_t* offs, const uint32_t* lens,
                       const uint8_t* tids, uint64_t L, uint64_t nfull, int gen_kind, void* out, int w, uint32_t* st,
                       ChunkInit ini, hipStream_t s);

}  // namespace mfast
}  // namespace shuffle_coding
