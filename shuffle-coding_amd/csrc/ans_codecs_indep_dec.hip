// Independent<Categorical> (src/codec.rs:366-403) on the fast decoder (ans_mfast.hpp k_mdec with
// IndepModel): the instantiations per norm range and symbol width.  (The decoder's renorm handles
// the bidirectional cases whatever the set: no screen variant.)
#include "ans_mfast_launch.hpp"

namespace shuffle_coding {
namespace mfast {
namespace {

template <int NR, int kL, bool kLean>
void dec_m(const IndepFast& f, const uint8_t* in, uint64_t cap, const uint64_t* offs, const uint32_t* lens,
           const uint8_t* tids, uint64_t L, uint64_t nfull, int gen_kind, void* out, int w, uint32_t* st, ChunkInit ini,
           hipStream_t s) {
    using M = IndepModel<false, NR, DecLayout<kL>::kTab, kLean>;
    const bool wide = kL == kLanesW;
    const M m{f.md.enc_img, wide ? f.dec_img_w : f.md.dec_img, f.md.nsym, f.md.enc_bytes,
              wide ? f.dec_bytes_w : f.md.dec_bytes, f.md.k_off, f.md.ro, f.md.no, f.md.so};
    const uint32_t lds = wide ? kLdsMax : kDecTab + m.dec_bytes;
    if (w == 1 && f.kmax * 16 <= 60) mdec<M, uint8_t, 16, kL>(m, in, cap, offs, lens, tids, L, nfull, gen_kind, out, st, ini, lds, s);
    else if (w == 1) mdec<M, uint8_t, 8, kL>(m, in, cap, offs, lens, tids, L, nfull, gen_kind, out, st, ini, lds, s);
    else if (w == 2) mdec<M, uint16_t, 8, kL>(m, in, cap, offs, lens, tids, L, nfull, gen_kind, out, st, ini, lds, s);
    else mdec<M, uint32_t, 4, kL>(m, in, cap, offs, lens, tids, L, nfull, gen_kind, out, st, ini, lds, s);
}
template <int NR, int kL>
void dec_l(const IndepFast& f, const uint8_t* in, uint64_t cap, const uint64_t* offs, const uint32_t* lens,
           const uint8_t* tids, uint64_t L, uint64_t nfull, int gen_kind, void* out, int w, uint32_t* st, ChunkInit ini,
           hipStream_t s) {
    if (kL == kLanesW ? f.lean_w : f.lean)
        dec_m<NR, kL, true>(f, in, cap, offs, lens, tids, L, nfull, gen_kind, out, w, st, ini, s);
    else
        dec_m<NR, kL, false>(f, in, cap, offs, lens, tids, L, nfull, gen_kind, out, w, st, ini, s);
}
// the 1,024-lane layout when the set has its image and the call the chains for one such
// workgroup per CU (four waves per SIMD); below that, 256-lane workgroups spread over more CUs
template <int NR>
void dec_w(const IndepFast& f, const uint8_t* in, uint64_t cap, const uint64_t* offs, const uint32_t* lens,
           const uint8_t* tids, uint64_t L, uint64_t nfull, int gen_kind, void* out, int w, uint32_t* st, ChunkInit ini,
           hipStream_t s) {
    if (f.dec_img_w && f.wide(nfull))
        dec_l<NR, kLanesW>(f, in, cap, offs, lens, tids, L, nfull, gen_kind, out, w, st, ini, s);
    else
        dec_l<NR, kLanes>(f, in, cap, offs, lens, tids, L, nfull, gen_kind, out, w, st, ini, s);
}

}  // namespace

void indep_fast_decode(const IndepFast& f, const uint8_t* in, uint64_t cap, const uint64_t* offs, const uint32_t* lens,
                       const uint8_t* tids, uint64_t L, uint64_t nfull, int gen_kind, void* out, int w, uint32_t* st,
                       ChunkInit ini, hipStream_t s) {
    if (f.nr == fast::kNormSmall) dec_w<fast::kNormSmall>(f, in, cap, offs, lens, tids, L, nfull, gen_kind, out, w, st, ini, s);
    else if (f.nr == fast::kNormBig) dec_w<fast::kNormBig>(f, in, cap, offs, lens, tids, L, nfull, gen_kind, out, w, st, ini, s);
    else dec_w<fast::kNormStd>(f, in, cap, offs, lens, tids, L, nfull, gen_kind, out, w, st, ini, s);
}

}  // namespace mfast
}  // namespace shuffle_coding
