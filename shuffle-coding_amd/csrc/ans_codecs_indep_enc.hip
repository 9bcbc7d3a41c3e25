// Independent<Categorical> (src/codec.rs:366-403) on the fast encoder (ans_mfast.hpp k_menc with
// IndepModel): the instantiations per norm range, renorm screen and symbol width.
#include "ans_mfast_launch.hpp"

namespace shuffle_coding {
namespace mfast {
namespace {

template <bool R, int NR, int kL>
void enc_l(const IndepFast& f, const void* syms, int w, const uint8_t* tids, uint64_t L, uint64_t nfull, uint8_t* slots,
           uint64_t cap, uint32_t* lens, uint32_t* st, ChunkInit ini, hipStream_t s) {
    using M = IndepModel<R, NR, kDecTab, false, EncLayout<kL>::kTab>;
    const M m{f.md.enc_img, f.md.dec_img, f.md.nsym, f.md.enc_bytes, f.md.dec_bytes, f.md.k_off, f.md.ro, f.md.no, f.md.so};
    const uint32_t lds = kL == kLanesW ? kLdsMax : kEncTab + m.enc_bytes;
    // a point per 16 u8 symbols needs at most 4 bytes each (64 between points), else per 8
    if (w == 1 && f.kmax * 16 <= 60) menc<M, uint8_t, 16, kL>(m, syms, tids, L, nfull, slots, cap, lens, st, ini, lds, s);
    else if (w == 1) menc<M, uint8_t, 8, kL>(m, syms, tids, L, nfull, slots, cap, lens, st, ini, lds, s);
    else if (w == 2) menc<M, uint16_t, 8, kL>(m, syms, tids, L, nfull, slots, cap, lens, st, ini, lds, s);
    else menc<M, uint32_t, 4, kL>(m, syms, tids, L, nfull, slots, cap, lens, st, ini, lds, s);
}
// the 1,024-lane layout (one shared table image, four waves per SIMD) when the set's image fits
// it and the call has the chains for one such workgroup per CU
template <bool R, int NR>
void enc_w(const IndepFast& f, const void* syms, int w, const uint8_t* tids, uint64_t L, uint64_t nfull, uint8_t* slots,
           uint64_t cap, uint32_t* lens, uint32_t* st, ChunkInit ini, hipStream_t s) {
    if (f.enc_wide && f.wide(nfull)) enc_l<R, NR, kLanesW>(f, syms, w, tids, L, nfull, slots, cap, lens, st, ini, s);
    else enc_l<R, NR, kLanes>(f, syms, w, tids, L, nfull, slots, cap, lens, st, ini, s);
}
template <int NR>
void enc_nr(const IndepFast& f, const void* syms, int w, const uint8_t* tids, uint64_t L, uint64_t nfull,
            uint8_t* slots, uint64_t cap, uint32_t* lens, uint32_t* st, ChunkInit ini, hipStream_t s) {
    if (f.rare) enc_w<true, NR>(f, syms, w, tids, L, nfull, slots, cap, lens, st, ini, s);
    else enc_w<false, NR>(f, syms, w, tids, L, nfull, slots, cap, lens, st, ini, s);
}

}  // namespace

void indep_fast_encode(const IndepFast& f, const void* syms, int w, const uint8_t* tids, uint64_t L, uint64_t nfull,
                       uint8_t* slots, uint64_t cap, uint32_t* lens, uint32_t* st, ChunkInit ini, hipStream_t s) {
    if (f.nr == fast::kNormSmall) enc_nr<fast::kNormSmall>(f, syms, w, tids, L, nfull, slots, cap, lens, st, ini, s);
    else if (f.nr == fast::kNormBig) enc_nr<fast::kNormBig>(f, syms, w, tids, L, nfull, slots, cap, lens, st, ini, s);
    else enc_nr<fast::kNormStd>(f, syms, w, tids, L, nfull, slots, cap, lens, st, ini, s);
}

}  // namespace mfast
}  // namespace shuffle_coding
