// ans_wide.hpp — fast kernels for large alphabets (nsym > 256: C4's 65,536-symbol table).
//
// Same messages and bytes as ans_fast.hpp (one lane = one chunk = one reference Message:
// src/ans.rs:292 zeros, src/codec.rs:415-424 IID, src/ans.rs:96-116 push/pop,
// src/ans.rs:255-264 flatten/unflatten); what differs is where the table lives.  A table of
// 65,536 rows does not fit in LDS, and a random 4-16 B gather from the L2 costs one L2 request
// whatever its width: tools/l2rand.hip measures ~265-300 G lane-requests/s chip-wide for
// tables of 256 KiB-2 MiB (any load width, any cache-policy bit), i.e. a whole 128-B line
// per request.  So these kernels cut L2 requests per symbol:
//  * the table is the bare cdf array (u32 cdf(0..nsym+5), 256 KiB for C4): a symbol's row is
//    the 8-B pair (cdf(s), cdf(s+1)), one request, and the smaller array keeps more of itself
//    in each CU's 32-KiB L1;
//  * the LDS holds a prefix of that array beside the byte ring, so every symbol below the
//    prefix bound (37% of C4's symbols in the encoder, ~24% of its probability in the
//    decoder) never leaves the CU;
//  * the encoder forms 1/p from v_rcp_f64 plus one Newton step instead of reading it
//    (error <= 2^-44 relative: the quotient estimate of DESIGN.md §4 holds for norm >= 2^22);
//  * streams move 128 B per lane per global access (aligned page pairs): a 128-B L2 line is
//    fetched once instead of once per 64-B half (profiles/r02_hbm_calib.txt).
#pragma once

#include "ans_fast.hpp"

namespace shuffle_coding {
namespace fast {

// ---- encoder LDS.  Plain prefix: the byte ring at offset 0 (64 KiB, 512 lanes), the cdf
// prefix after it.  Packed prefix: the per-mass renorm shifts first when kSa (kWideSaBytes at
// offset 0, so a shift's address is the mass itself), the block bases (kWideBBytes, below 64 KiB
// so their base folds into the ds offset field), the ring, then the low halves.
constexpr uint32_t kWideRing = 0;
constexpr uint32_t kWideEncCum = kEncRingBytes;
constexpr uint32_t kWideEncCumMax = (160u * 1024u - kWideEncCum) / 4u;  // staged cdf entries
constexpr uint32_t kWideNormMin = 1u << 22;  // one Newton step suffices above (see k_encode_w)
constexpr uint32_t kWideSaMax = 4096;        // largest mass with a shift byte (12-bit masses)
constexpr uint32_t kWideSaBytes = 4352;      // (kWideSaMax + 1) bytes, rounded up to 256
static_assert(kWideSaBytes >= kWideSaMax + 1 && kWideSaBytes % 256 == 0, "shift table");
constexpr uint32_t kWideBBytes = 10752;      // packed block bases: up to 2,688 (43,000 symbols)
template <bool kSa, bool kPack>
struct WideEncLds {
    static constexpr uint32_t b = kSa ? kWideSaBytes : 0;               // packed: block bases
    static constexpr uint32_t ring = kPack ? b + kWideBBytes : kWideRing;
    static constexpr uint32_t cum = ring + kEncRingBytes;               // plain cdf / packed low halves
};
// the packed prefix's capacity: nl symbols need (nl/16 + 2) bases and nl + 2 low halves
constexpr uint32_t wide_pack_nl_max(bool sa) {
    const uint32_t o_bytes = 160u * 1024u - ((sa ? kWideSaBytes : 0) + kWideBBytes + kEncRingBytes);
    const uint32_t by_o = (o_bytes / 4u) * 2u - 2u, by_b = ((kWideBBytes / 4u) - 2u) * 16u;
    return (by_o < by_b ? by_o : by_b) & ~15u;
}
static_assert(WideEncLds<true, true>::cum + ((2u * (wide_pack_nl_max(true) + 2u) + 3u) & ~3u) <= 160u * 1024u &&
                  WideEncLds<false, true>::cum + ((2u * (wide_pack_nl_max(false) + 2u) + 3u) & ~3u) <= 160u * 1024u &&
                  4u * ((wide_pack_nl_max(false) >> 4) + 2u) <= kWideBBytes && WideEncLds<true, true>::ring <= 65535u,
              "packed prefix regions fit one CU's LDS (the ring base in the 16-bit ds offsets)");

typedef unsigned v2u32 __attribute__((ext_vector_type(2)));
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }

// (cdf(s), cdf(s+1)) from the global cdf array: one 8-B load at a 4-B aligned address
__device__ __forceinline__ v2u32 cum_pair_global(const uint32_t* cum, uint32_t s) {
    typedef __attribute__((address_space(1))) const v2u32 gv2;
    return *reinterpret_cast<gv2*>(reinterpret_cast<uintptr_t>(cum + s));
}
// ... and from the LDS prefix (ds_read2_b32: any dword alignment)
__device__ __forceinline__ v2u32 cum_pair_lds(uint32_t base, uint32_t s) {
    const lds_u32* p = reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(base + 4 * s));
    return v2u32{p[0], p[1]};
}

// fl(1/p) to within 2^-44 relative: v_rcp_f64 (tools/rcp_check.hip measures up to 2^28 ulp,
// ~2^-24 relative) and one Newton step r' = r + r(1 - p r), whose error is the square of that
// plus two roundings.  With x < 2^64 and norm >= 2^22, x/p < 2^42, so the estimate of
// qest_m1 stays within 2^42 * (2^-44 + 2^-52) < 1/2 of x/p: q_m in {q - 1, q} as before.
__device__ __forceinline__ double rcp_newton(uint32_t p) {
    const double d = static_cast<double>(p);
    const double r = __builtin_amdgcn_rcp(d);
    const double e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(r, e, r);
}

// Encoder for nsym > 256 (u16 / u32 symbols): rows from the LDS prefix or the global cdf.
// Groups of 128 B of symbols (8 units of 16 B) per lane, walked last to first; each unit's rows
// are requested at the point before it (LDS or global, per lane), so their latency hides behind
// one unit of work.  Points and the byte funnel are ans_fast.hpp's.
// kPack: the LDS prefix is the packed image (FastTable::enc_pack): a row costs a ds_read_b32 of
// the block base and two ds_read_u16 of low halves plus 3 VALU (lrow), for ~1.8x the prefix
// (64% of C4's symbols instead of 37%; the rest is the L2 request each).
// kSa: every mass is at most kWideSaMax (FastTable::enc_sa) and its renorm shift sa(p) is one
// LDS byte at address p: k = sa/8 - 1 + [head >= p*K << sa] (ans_renorm.hpp enc_sa), one 64-bit
// shift and compare where the bit-length renorm takes three v_ffbh, two v_min, four adds, the
// shift and the compare.  The unit's eight shift bytes are read before its first push.
// kVar: chunk c holds vlen[c] <= chunk_len symbols at the start of its chunk_len-symbol stride
// (a staged ragged or variable-length chunk, ans_kernels.hip launch_staged): its last group is
// partial, and it is the first one coded, so the pushes past vlen[c] are skipped there.
// (A push emits at most 4 bytes whatever the table, and the renorm never loops over j, so the
// kernel has no KMAX parameter: one unit of 8 u16 / 4 u32 symbols completes at most one page.)
// kNR: kNormStd, or kNormBig (2^31 < norm < 2^32: a mass may reach 2^31, where the 32-bit
// remainder test cannot tell r - p from r, so those rows always take the exact 64-bit branch, as
// in ans_fast.hpp push_one; the quotient is below 2^33 there, so the estimate is as tight).
// kNormSmall tables never come here (norm < 2^16 < kWideNormMin).
template <typename Sym, bool kK32, bool kPack, bool kSa, bool kVar = false, int kNR = kNormStd>
__global__ __launch_bounds__(kBlock, 2) void k_encode_w(FastTable t, const Sym* __restrict__ syms, uint64_t chunk_len,
                                                         uint64_t nfull, uint8_t* __restrict__ slots, uint64_t slot_cap,
                                                         uint32_t* __restrict__ lens, uint32_t* __restrict__ status,
                                                         ChunkInit ini, const uint32_t* __restrict__ vlen = nullptr) {
    static_assert(!kSa || kPack, "the shift table comes with the packed prefix");
    static_assert(kNR != kNormSmall, "norm < 2^16: the global-row k_encode");
    using Lay = WideEncLds<kSa, kPack>;
    extern __shared__ __align__(16) unsigned char lds[];
    {
        uint32_t* lc = reinterpret_cast<uint32_t*>(lds + Lay::cum);
        if constexpr (kPack) {  // the image's bases and low halves to their two regions
            uint32_t* lb = reinterpret_cast<uint32_t*>(lds + Lay::b);
            const uint32_t nb = t.enc_pack_ooff / 4;
            for (uint32_t i = threadIdx.x; i < t.enc_pack_bytes / 4; i += kBlock) {
                if (i < nb) lb[i] = t.enc_pack_img[i];
                else lc[i - nb] = t.enc_pack_img[i];
            }
        } else {
            for (uint32_t i = threadIdx.x; i <= t.enc_nl; i += kBlock) lc[i] = t.cum[i];
        }
        if constexpr (kSa) {
            uint32_t* ls = reinterpret_cast<uint32_t*>(lds);
            for (uint32_t i = threadIdx.x; i < kWideSaBytes / 4; i += kBlock) ls[i] = t.enc_sa_img[i];
        }
    }
    const RingT<Lay::ring> ring{4 * threadIdx.x};
    __syncthreads();
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (c >= nfull) return;

    constexpr int U = 16 / static_cast<int>(sizeof(Sym));
    constexpr int GU = 8;  // units per 128-B group
    const uint4* src = reinterpret_cast<const uint4*>(syms + c * chunk_len);
    constexpr int GS = 128 / static_cast<int>(sizeof(Sym));  // symbols per group
    const uint32_t nvalid = kVar ? vlen[c] : static_cast<uint32_t>(chunk_len);
    const int ngroups = kVar ? static_cast<int>((nvalid + GS - 1) / GS) : static_cast<int>(chunk_len * sizeof(Sym) / 128);
    uint8_t* dst = slots + c * slot_cap;
    const uint32_t npages_cap = static_cast<uint32_t>(slot_cap / 64);
    const uint64_t K = t.K;
    const uint32_t norm = t.norm;
    const uint32_t nsym = t.nsym;  // out-of-range symbols read the zero-mass pair (cdf(nsym), cdf(nsym+1))
    const uint32_t nl = t.enc_nl;
    const uint32_t exp_norm = 0x43300000u * norm;
    const uint32_t* gcum = t.cum;

    uint64_t head = ini.head(c);  // Message::zeros() / random(seed + c)
    FunnelT<Lay::ring> f{0, 0, 0, ring.col, ring.col};
    PageOut<Lay::ring> pout;
    uint32_t fp = 0, over = 0;
    uint32_t minmass = ~0u;

    auto flush = [&]() __attribute__((always_inline)) {
        if ((f.pos8 >> 9) > fp) {  // at most one page completes per unit (U * KMAX <= 64 bytes)
            if (fp < npages_cap) pout.page(ring, fp, dst);
            else over = 1;
            ++fp;
        }
    };
    // a unit's rows: every lane reads the LDS pair of min(s, nl) (always in range) and the lanes
    // whose symbol lies past the prefix also load the global pair, into separate registers (a
    // shared destination would make each LDS read wait for every outstanding global load)
    // A unit's rows land in ONE pair of registers per symbol whichever part of the table holds
    // them: every lane reads the LDS prefix at min(s, nl), then the lanes with s >= nl overwrite
    // those registers from global memory with a row that the same combination (lrow) turns into
    // (cdf(s), pmf(s)), so process selects nothing (packed: FastTable::enc_grow; plain: (cdf(s),
    // cdf(s+1))).  The global loads follow all of the unit's LDS reads: the compiler orders a
    // load after a pending LDS write to the same registers with an lgkmcnt wait, once per unit
    // where interleaving them would wait once per symbol.  (Separate registers took a select,
    // which the compiler made an exec-masked branch per symbol: six SALU and a v_mov.)
    // Packed rows: (B, O(s) | O(s+1) << 16), the two low halves in one register (lrow reads
    // them by halves; as separate u32 values each took a v_and).
    using LRow = v2u32;
    // kPack: the global rows load on every lane, into their own registers, with no exec mask: a
    // lane in the prefix reads row nl - 1, all zero, and a lane past it the row XORed with its
    // LDS read C = row nl (FastTable::enc_grow), so lbuf ^ gbuf is the symbol's row either way
    auto request_g = [&](const uint4& unit, LRow* gbuf) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t s = umin(sym_of<Sym>(unit, j), nsym);
            gbuf[j] = cum_pair_global(t.enc_grow, 2 * umax(s, nl - 1));
        }
    };
    auto request = [&](const uint4& unit, LRow* lbuf) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t sp = umin(umin(sym_of<Sym>(unit, j), nsym), nl);
            if constexpr (kPack) {
                const uint32_t b = *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(Lay::b + 4 * (sp >> 4)));
                uint32_t oa;  // Lay::cum + 2 sp in one v_lshl_add (the base lies past the 16-bit ds
                              // offsets; from C++ the compiler formed oa and oa + 2 with two v_add)
                asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(oa) : "v"(sp), "s"(Lay::cum));
                us2 o;
                o.x = *reinterpret_cast<const lds_u16*>(static_cast<uintptr_t>(oa));
                o.y = *reinterpret_cast<const lds_u16*>(static_cast<uintptr_t>(oa + 2));
                lbuf[j] = v2u32{b, __builtin_bit_cast(uint32_t, o)};
            } else {
                lbuf[j] = cum_pair_lds(Lay::cum, sp);
            }
        }
        if constexpr (!kPack) {
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const uint32_t s = umin(sym_of<Sym>(unit, j), nsym);
                if (s >= nl) lbuf[j] = cum_pair_global(gcum, s);
            }
        }
    };
    // (cdf(s), pmf(s)) of a symbol.  Packed (ans_kernels.hip build_fast_table): B = cdf(16 b) of
    // its block and the low halves O(s) = cdf(s) mod 2^16, O(s + 1); within a block cdf(s) - B
    // < 2^16 and every mass is below 2^16, so cdf(s) = B + ((O(s) - B) mod 2^16) and pmf(s) =
    // (O(s + 1) - O(s)) mod 2^16: a 16-bit subtract, an SDWA add of its low half and a 16-bit
    // subtract, with no select at block ends (offsets from each block's base needed the next
    // block's base for s = 16 b + 15).  A global row (B = cdf(s)) gives the same.
    auto lrow = [&](const LRow& r) __attribute__((always_inline)) {
        if constexpr (kPack) {
            uint32_t d, cum, p;  // (d: only its low half is defined and read)
            asm("v_sub_u16 %0, %1, %2" : "=v"(d) : "v"(r.y), "v"(r.x));
            asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
                : "=v"(cum) : "v"(r.x), "v"(d));
            asm("v_sub_u16_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0"
                : "=v"(p) : "v"(r.y), "v"(r.y));
            return v2u32{cum, p};
        } else {
            return v2u32{r.x, r.y - r.x};
        }
    };
    // renorm(p*K) (src/ans.rs:100,246-253): k = #{j >= 1 : (head >> 8j) >= p*K} bytes out
    // From bit lengths: with d = bitlen(head) - bitlen(pK) >= 0 (head >= norm*K >= pK before a
    // push), every j with 8j < d holds and every j with 8j > d fails, so k = m - 1 + [(head >> 8m)
    // >= pK] for m = ceil(d / 8): one 64-bit shift and compare where testing each j took KMAX
    // (8m <= 40: pK >= K >= 2^25 in the fast range, so d <= 39).  head >= 2^55 here, so its
    // high word is never zero.
    auto bytes_out8 = [&](uint64_t pK) __attribute__((always_inline)) {
        uint32_t fh, fp0, fp1;
        asm("v_ffbh_u32 %0, %1" : "=v"(fh) : "v"(hi32(head)));
        asm("v_ffbh_u32 %0, %1" : "=v"(fp1) : "v"(hi32(pK)));
        asm("v_ffbh_u32 %0, %1" : "=v"(fp0) : "v"(lo32(pK)));
        const uint32_t clz_pk = umin(fp1, fp0 + 32u);  // ffbh(0) = ~0: the low word's count then wins
        const uint32_t m8 = (clz_pk - fh + 7u) & ~7u;  // 8 * ceil(d / 8)
        return (head >> m8) >= pK ? m8 : m8 - 8u;
    };
    // the row of symbol j of a unit: cdf(x), pmf(x) (src/codec.rs:63-64)
    auto process = [&](const LRow* lbuf, const LRow* gbuf, uint32_t upos) __attribute__((always_inline)) {
        auto row_of = [&](int j) __attribute__((always_inline)) {
            if constexpr (kPack) return lrow(lbuf[j] ^ gbuf[j]);
            else return lrow(lbuf[j]);
        };
        // kSa: the unit's rows and shift bytes first (p <= kWideSaMax: the byte at LDS address p)
        v2u32 rows[U];
        uint32_t sas[U];
        if constexpr (kSa) {
#pragma unroll
            for (int j = U - 1; j >= 0; --j) {
                rows[j] = row_of(j);
                sas[j] = *reinterpret_cast<const lds_u8*>(static_cast<uintptr_t>(rows[j].y));
            }
        }
#pragma unroll
        for (int j = U - 1; j >= 0; --j) {  // IID::push: last symbol first (src/codec.rs:417)
            if (kVar && upos + j >= nvalid) continue;  // past the chunk (its first, partial group)
            __builtin_amdgcn_s_setprio(2);  // the push at raised wave priority (encode -0.4%, A/B)
            const v2u32 row = kSa ? rows[j] : row_of(j);
            const uint32_t cum = row.x, p = row.y;
            const uint64_t pK = kK32 ? static_cast<uint64_t>(p) * static_cast<uint32_t>(K) : static_cast<uint64_t>(p) * K;
            uint32_t k8;
            if constexpr (kSa) {
                const uint32_t sa = sas[j];
                k8 = head >= (pK << sa) ? sa : sa - 8u;
            } else {
                k8 = bytes_out8(pK);
            }
            f.push(lo32(head), k8);
            head >>= k8;
            // q = head / p, r = head % p (src/ans.rs:101-102), head = norm*q + cdf(x, r)
            // (src/ans.rs:103-104): ans_fast.hpp push_one's form, with 1/p from rcp_newton.
            // The estimate is rounded to nearest (qest_half) and the rare lanes where it is not q
            // take the exact 64-bit remainder on a voted branch: rcp_newton is within 2^-47.9 of
            // 1/p (v_rcp_f64 within 2^-24, squared by the Newton step, plus roundings) and
            // head/p < 2^64 / norm <= 2^42, so the estimate is within 2^-5.9 of head/p (C4,
            // norm 2^27: 2^-10.9, the branch in ~7% of wave steps) and q_est is q - 1, q or
            // q + 1.  The estimate from below (qest_m1) needed a borrow-select on every push.
            uint64_t qb = qest_half(head, rcp_newton(p));
            uint32_t rm = lo32(head) - lo32(qb) * p;
            const bool fix = kNR == kNormBig ? (rm >= p || static_cast<int32_t>(p) < 0) : rm >= p;
            if (__builtin_expect(__builtin_amdgcn_ballot_w64(fix) != 0, 0)) {
                if (fix) {  // a zero-mass push (p = 0: rm >= 0 = p) always lands here
                    minmass = min(minmass, p);
                    const int64_t r = static_cast<int64_t>(head - (qb - 0x4330000000000000ull) * p);
                    // (kNormBig's forced rows may be right already)
                    const int64_t d = r < 0 ? -1 : (kNR != kNormBig || r >= static_cast<int64_t>(p) ? 1 : 0);
                    qb += static_cast<uint64_t>(d);
                    rm = static_cast<uint32_t>(r - d * static_cast<int64_t>(p));
                }
            }
            const uint32_t a = cum + rm;
            const uint64_t lo64 = static_cast<uint64_t>(lo32(qb)) * norm + a;
            uint32_t hq;
            asm("v_mul_lo_u32 %0, %1, %2" : "=v"(hq) : "v"(hi32(qb)), "s"(norm));
            head = mk64(hi32(lo64) + hq - exp_norm, lo32(lo64));
            __builtin_amdgcn_s_setprio(0);
        }
    };

    uint4 n[GU];
#pragma unroll
    for (int i = 0; i < GU; ++i) n[i] = make_uint4(0, 0, 0, 0);
    if (ngroups > 0) {  // (an empty staged chunk codes no symbol)
        const uint4* gsrc = src + GU * (ngroups - 1);
#pragma unroll
        for (int i = 0; i < GU; ++i) n[i] = gsrc[i];
    }
    // r06: the packed rows' global loads on every lane (request_g) measured encode -1.2/-2.3% in a
    // same-box A/B against the exec-masked loads; requesting them TWO units ahead with the
    // compiler's own vmcnt waits instead of the points' (four rotating sets) +2.2%
    // (profiles/r06l_ab_c4_enc_two_ahead_rejected.txt)
    LRow la[U], lb[U], ga[U], gb[U];
    wait_vm();
    request(n[GU - 1], la);
    if constexpr (kPack) request_g(n[GU - 1], ga);
    for (int g = ngroups - 1; g >= 0; --g) {
        uint4 cc[GU];
#pragma unroll
        for (int i = 0; i < GU; ++i) cc[i] = n[i];
#pragma unroll
        for (int u = GU - 1; u >= 0; --u) {
            // point: the rows of unit u (requested one unit ago) have landed; the group prefetch
            // issued after them at u = GU-1 may stay in flight through the next point
            if (u == GU - 2) wait_vm_n<GU>();
            else wait_vm();
            flush();
            const bool odd = (u & 1) != 0;
            if (u > 0) {
                request(cc[u - 1], odd ? lb : la);
                if constexpr (kPack) request_g(cc[u - 1], odd ? gb : ga);
            }
            if (u == GU - 1 && g > 0) {
                const uint4* gsrc = src + GU * (g - 1);
#pragma unroll
                for (int i = 0; i < GU; ++i) n[i] = gsrc[i];
            }
            if (u == 0) {  // unit GU-1 of group g-1 (landed units ago)
                request(n[GU - 1], la);
                if constexpr (kPack) request_g(n[GU - 1], ga);
            }
            process(odd ? la : lb, odd ? ga : gb, static_cast<uint32_t>(g * GS + u * U));
        }
    }
    wait_vm();
    flush();  // the last unit's completed page: the flatten's 8 bytes may reach the ring slot it holds

    // flatten (src/ans.rs:255-260): all significant head bytes, low first (7 or 8 here)
    const uint32_t nb = (71u - static_cast<uint32_t>(__builtin_clzll(head))) >> 3;
    f.push(lo32(head), 32);
    f.push(hi32(head), 8 * (nb - 4));
    f.finish();
    const uint32_t len = f.len();
    for (const uint32_t last = (len + 63) / 64; fp < last; ++fp) {
        if (fp < npages_cap) pout.page(ring, fp, dst);
        else over = 1;
    }
    if (!over) pout.finish(fp, dst);
    if (minmass == 0) {  // classify like the reference: out-of-range index (codec.rs:63) or p == 0 (ans.rs:98)
        uint32_t sym_err = 0;
        for (uint64_t k = 0; k < nvalid; ++k)
            sym_err |= static_cast<uint32_t>(syms[c * chunk_len + k]) >= t.nsym ? 1u : 0u;
        atomicOr(status, 1u << (sym_err ? ANS_E_SYMBOL : ANS_E_ZERO_MASS));
    }
    if (over) atomicOr(status, 1u << ANS_E_LEN);
    lens[c] = (over || minmass == 0) ? 0u : len;
}

// ====================================================================== decode, large alphabets
// One chain per lane as in ans_fast.hpp k_decode; the icdf (src/codec.rs:65-68) splits by cf:
//  * cf < cpre = cdf(nlp) (a prefix of the alphabet staged in LDS): bucket cf >> shp gives
//    s0 = icdf(bucket start) from a u16 array, then cdf(s0..s0+4) from the staged cdf prefix
//    (three ds_read2_b32) resolve four candidates; cf >= cdf(s0+4) scans the staged cdf (voted);
//  * otherwise the global DecBucketG of cf >> dec_shift (cdf(s0..s0+5) and s0, 32 B in one
//    128-B line: one L2 request), with the global cdf scan past its fifth candidate (voted).
// The stream ring holds two 64-B pages per lane (33 rows x 512 lanes, row 32 mirroring row 0);
// the next aligned 128-B page pair waits in registers and lands one page per point.  A point
// comes every 16 symbols (at most 64 B, KMAX <= 4), so reads never reach an unlanded page, and
// one global page fetch per 128 B exposes its HBM latency once per ~64 symbols (gfx9 retires
// vector-memory operations in issue order, so a page fetch delays the next bucket load).
constexpr int kWideDecRows = 33;
// 512 lanes: 1,024 (four waves per SIMD, 25 KiB of tables) measured 40% slower on C4, its
// smaller LDS prefix sending more lookups to L2
constexpr uint32_t kWideDecLanes = 512;
constexpr uint32_t kWideDecRowShift = 11;  // log2 of a ring row's bytes
static_assert((1u << kWideDecRowShift) == kWideDecLanes * 4, "row bytes");
constexpr uint32_t kWideDecTab = kWideDecRows * kWideDecLanes * 4;  // 67,584 B of ring, then the tables
static_assert(kWideDecTab % 256 == 0, "table base");
constexpr uint32_t kWideDecTabBytes = 160u * 1024u - kWideDecTab;
constexpr uint32_t kWideDecBktLds = kWideDecTabBytes / 16;  // compact buckets staged beside the ring
__device__ const uint4 kZeroPair[8] = {};  // 128 zero bytes: pages below the stream start

struct DecChainW {
    uint32_t col;  // 4 * lane
    const uint8_t* src;
    uint4 Q[8];    // the page pair (2m, 2m+1) not yet landed
    int32_t low, P, sh;  // sh: the stream start within its 128-B line
    uint32_t wx, wy, W;
    uint64_t head;
    uint64_t qq;
    uint32_t cf, cum, nxt, sx;
    bool far;

    __device__ __forceinline__ lds_u32& row(int32_t r) const {
        return *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>((static_cast<uint32_t>(r) << kWideDecRowShift) + col));
    }
    // positions count from the stream's first byte (ans_fast.hpp DecChain::fetch_pair): pairs
    // below the top one lie inside the stream and are read with unaligned 16-B loads
    __device__ __forceinline__ void fetch_pair(int32_t m) {
        typedef __attribute__((address_space(1), aligned(1))) const v4u32 gv4;
        const uint4* g = m >= 0 ? reinterpret_cast<const uint4*>(src + 128ll * m) : kZeroPair;
        const gv4* gg = reinterpret_cast<const gv4*>(reinterpret_cast<uintptr_t>(g));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const v4u32 v = gg[k];
            Q[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
    }
    // page p (its half of Q) into ring slot p & 1: eight ds_write2st64_b32 from the lane's
    // column (rows 2 KiB apart are 8 st64 units, rows 0..31 within the 8-bit offset fields);
    // pages count from the stream's start, so none holds another stream's bytes
    template <int R0>
    __device__ __forceinline__ void land_half(uint4 a0, uint4 a1, uint4 a2, uint4 a3) {
        constexpr int o = 8 * R0;
        asm volatile(
            "ds_write2st64_b32 %0, %1, %2 offset0:%17 offset1:%18\n\t"
            "ds_write2st64_b32 %0, %3, %4 offset0:%19 offset1:%20\n\t"
            "ds_write2st64_b32 %0, %5, %6 offset0:%21 offset1:%22\n\t"
            "ds_write2st64_b32 %0, %7, %8 offset0:%23 offset1:%24\n\t"
            "ds_write2st64_b32 %0, %9, %10 offset0:%25 offset1:%26\n\t"
            "ds_write2st64_b32 %0, %11, %12 offset0:%27 offset1:%28\n\t"
            "ds_write2st64_b32 %0, %13, %14 offset0:%29 offset1:%30\n\t"
            "ds_write2st64_b32 %0, %15, %16 offset0:%31 offset1:%32"
            :
            : "v"(col), "v"(a0.x), "v"(a0.y), "v"(a0.z), "v"(a0.w), "v"(a1.x), "v"(a1.y), "v"(a1.z), "v"(a1.w),
              "v"(a2.x), "v"(a2.y), "v"(a2.z), "v"(a2.w), "v"(a3.x), "v"(a3.y), "v"(a3.z), "v"(a3.w),
              "i"(o), "i"(o + 8), "i"(o + 16), "i"(o + 24), "i"(o + 32), "i"(o + 40), "i"(o + 48), "i"(o + 56),
              "i"(o + 64), "i"(o + 72), "i"(o + 80), "i"(o + 88), "i"(o + 96), "i"(o + 104), "i"(o + 112), "i"(o + 120)
            : "memory");
    }
    __device__ __forceinline__ void land(int32_t p) {
        if (p & 1) {
            land_half<16>(Q[4], Q[5], Q[6], Q[7]);
        } else {
            land_half<0>(Q[0], Q[1], Q[2], Q[3]);
            row(32) = Q[0].x;  // row 32 mirrors row 0
        }
    }
    __device__ __forceinline__ void read_window() {
        const uint32_t a = ((static_cast<uint32_t>(P) << (kWideDecRowShift - 2)) & (31u << kWideDecRowShift)) | col;  // row (P >> 2) & 31
        wy = *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(a));
        wx = *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(a + kWideDecLanes * 4));
    }
    __device__ __forceinline__ void form_window() { W = ab(wx, wy, static_cast<uint32_t>(P)); }
    // the top pair, which may reach past the stream's end: the aligned dwords holding stream
    // bytes, funnelled to the stream's alignment (ans_fast.hpp DecChain::fetch_top)
    __device__ __forceinline__ void fetch_top(int32_t m, int32_t len) {
        typedef __attribute__((address_space(1))) const uint32_t gu32;
        const uintptr_t a = reinterpret_cast<uintptr_t>(src) + 128ll * m;
        const gu32* d0 = reinterpret_cast<const gu32*>(a & ~uintptr_t(3));
        const uint32_t b = static_cast<uint32_t>(a & 3u);
        const int32_t last = static_cast<int32_t>(((reinterpret_cast<uintptr_t>(src) + len - 1) >> 2) - (a >> 2));
        uint32_t d[33];
#pragma unroll
        for (int q = 0; q < 33; ++q) d[q] = q <= last ? d0[q] : 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            Q[k] = make_uint4(ab(d[4 * k + 1], d[4 * k], b), ab(d[4 * k + 2], d[4 * k + 1], b),
                              ab(d[4 * k + 3], d[4 * k + 2], b), ab(d[4 * k + 4], d[4 * k + 3], b));
    }
    // the top two pages land before decoding starts; the pair below them is requested.
    // s: the stream's first byte, at any alignment (a dense container); positions count from s
    // itself (sh = 0), so the lanes of a wave land pages at nearly the same symbols in a dense
    // container as in slots (ans_fast.hpp DecChain::start)
    __device__ __forceinline__ void start(const uint8_t* s, int32_t slen) {
        sh = 0;
        src = s;
        const int32_t len = slen;
        const int32_t top = len > 0 ? (len - 1) >> 6 : 0;
        if (len > 0) fetch_top(top >> 1, len);
        else fetch_pair(-1);
        wait_vm();
        land(top);
        if (top & 1) {
            land(top - 1);
            fetch_pair((top >> 1) - 1);  // holds top-3, top-2
        } else {
            fetch_pair((top >> 1) - 1);  // holds top-2, top-1
            wait_vm();
            land(top - 1);                // top-2 stays in the low half
        }
        low = top - 1;
        lim = 64 * low + 60;
        P = len - 4;
        read_window();
        head = 0;
    }
    __device__ __forceinline__ void pull_until(uint64_t bound) {
        for (int g = 0; g < 9 && head < bound; ++g) {
            form_window();
            head = (head << 8) | (W >> 24);
            P -= 1;
            read_window();
        }
    }
    // at a point (after s_waitcnt vmcnt(0)): land page low-1 once page low+1 is no longer read
    // (((P >> 2) + 1) >> 4 <= low  <=>  P < lim = 64 low + 60: one compare per point)
    int32_t lim;
    __device__ __forceinline__ void point() {
        if (P < lim) {
            land(low - 1);
            --low;
            lim -= 64;
            if (!(low & 1)) fetch_pair((low >> 1) - 1);  // the next page (low-1, odd) opens a new pair
        }
    }
    template <int kNR = kNormStd>
    __device__ __forceinline__ void renorm_div(uint64_t L, uint32_t hL8, uint32_t norm, double rcp_norm,
                                               double neg_norm = 0.0) {
        form_window();
        P -= static_cast<int32_t>(renorm_up(head, W, L, hL8));
        read_window();  // for the next step; kept ahead of this step's lookups
        __builtin_amdgcn_sched_barrier(0);
        div_norm<kNR>(head, norm, rcp_norm, qq, cf, neg_norm);
    }
    // head = p*q + r; with every mass below 2^24 (kP24) the high word's product is one
    // v_mad_u32_u24 (hi32(q) < 2^24 for norm > 256), as in ans_fast.hpp DecChain::update
    template <bool kP24>
    __device__ __forceinline__ void update(uint32_t p, uint32_t r) {
        if constexpr (kP24) {
            const uint64_t lo = static_cast<uint64_t>(lo32(qq)) * p + r;
            uint32_t hi;
            asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(hi) : "v"(hi32(qq)), "v"(p), "v"(hi32(lo)));
            head = mk64(hi, lo32(lo));
        } else {
            head = qq * p + r;
        }
    }
};

// kCompact: the global buckets are DecBucketC (16 B, one L2 request), else DecBucketG (32 B).
// kPrefix: resolve cf below dec_w_cpre from the LDS prefix, else every lookup is global (the
// compact tables: a wave step waits on L2 as soon as one of its 64 lanes misses the prefix,
// which for C4 is nearly every step, so the prefix only added VALU to the chain).
// kVar: chunk c decodes vlen[c] <= chunk_len symbols into the start of its chunk_len-symbol
// stride (staged output: the rest of its last 128-B line is garbage).
// kP24: every mass is below 2^24 and the norm above 256 (DecChainW::update: hi32(q) < 2^24).
// kNR: the norm range of div_norm (kNormSmall: more than 256 symbols below 2^16, a count-built
// label table; kNormBig: 2^31 < norm < 2^32).
template <typename Sym, bool kCompact, bool kPrefix, bool kVar = false, bool kP24 = false, int kNR = kNormStd>
__global__ __launch_bounds__(kWideDecLanes, 2) void k_decode_w(FastTable t, const uint8_t* __restrict__ slots,
                                                         uint64_t slot_cap, const uint64_t* __restrict__ offsets,
                                                         const uint32_t* __restrict__ lens,
                                                         uint64_t chunk_len, uint64_t nfull, int gen_kind,
                                                         Sym* __restrict__ out, uint32_t* __restrict__ status,
                                                         ChunkInit ini, const uint32_t* __restrict__ vlen = nullptr) {
    extern __shared__ __align__(16) unsigned char lds[];
    if (kPrefix) {  // the prefix tables: bucket s0 values (u16), then cdf(0 .. nlp + 5)
        const uint32_t* gs = reinterpret_cast<const uint32_t*>(t.dec_w_s0);
        uint32_t* ls = reinterpret_cast<uint32_t*>(lds + kWideDecTab);
        for (uint32_t i = threadIdx.x; i < (t.dec_w_nbp + 1) / 2; i += kWideDecLanes) ls[i] = gs[i];
        uint32_t* lc = reinterpret_cast<uint32_t*>(lds + kWideDecTab + t.dec_w_cum_off);
        for (uint32_t i = threadIdx.x; i <= t.dec_w_nlp + 5; i += kWideDecLanes) lc[i] = t.cum[i];
    }
    // compact buckets without the prefix (C4): the first nlb = t.dec_c_nlb buckets are staged in
    // the LDS the ring leaves (up to kWideDecBktLds: 6,016 of C4's 65,704), so that share of the
    // lookups issues no L2 request (the decoder runs at ~0.87 of the L2 gather ceiling, DESIGN.md
    // §3.3).  The launcher sizes the dynamic LDS for them (ans_launch_impl.hpp wide_dec_lds).
    // Tables with more buckets than that stage theirs at twice the width (t.dbkt_cl, shift
    // dec_cl_shift = dec_c_shift + 1: C4 9.2% -> 18.3% of lookups); the 1/256 or less of a staged
    // bucket's cf beyond its five candidates re-fetches the lane's global bucket (far below).
    const uint32_t nlb = kCompact && !kPrefix ? t.dec_c_nlb : 0u;
    if constexpr (kCompact && !kPrefix) {
        const uint4* gb = reinterpret_cast<const uint4*>(t.dbkt_cl);
        uint4* lb = reinterpret_cast<uint4*>(lds + kWideDecTab);
        for (uint32_t i = threadIdx.x; i < nlb; i += kWideDecLanes) lb[i] = gb[i];
    }
    __syncthreads();
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kWideDecLanes + threadIdx.x;
    if (c >= nfull) return;  // no barrier below: lanes are independent
    if (!offsets && lens[c] > slot_cap) {  // foreign or corrupt stream: its pages would lie past the slot
        atomicOr(status, 1u << ANS_E_LEN);
        return;
    }

    constexpr int U = 16 / static_cast<int>(sizeof(Sym));
    constexpr int UPT = 16 / U;  // units per point: 16 symbols, at most 64 stream bytes
    const uint32_t nvalid = kVar ? vlen[c] : static_cast<uint32_t>(chunk_len);
    // a multiple of 4 (chunk bytes % 64 == 0), or for kVar the units holding the chunk
    const int nunit = static_cast<int>((nvalid + U - 1) / U);
    const uint64_t L = t.L;
    const uint32_t hL8 = renorm_screen(L);
    const uint32_t norm = t.norm;
    const double rcp_norm = t.rcp_norm;
    const uint32_t shift = t.dec_shift, shp = t.dec_w_shp, cpre = t.dec_w_cpre;
    const uint32_t lcum = kWideDecTab + t.dec_w_cum_off;  // LDS byte address of cdf(0)
    const DecBucketG* __restrict__ bkt = t.dbkt_g;
    const DecBucketC* __restrict__ bktc = t.dbkt_c;
    const uint32_t cshift = t.dec_c_shift, clshift = t.dec_cl_shift;
    const uint32_t* __restrict__ gcum = t.cum;
    uint4* dst = reinterpret_cast<uint4*>(out + c * chunk_len);

    DecChainW ch;
    ch.col = 4 * threadIdx.x;
    ch.start(slots + (offsets ? offsets[c] : c * slot_cap), static_cast<int32_t>(lens[c]));
    ch.pull_until(L);  // Message::unflatten: head 0, renorm_up pulls the flushed head

    // a compact bucket (c0 | s0, d0 | d1, d2 | d3, d4) resolved for cf: the pop's p = pmf(s), r = cf -
    // cdf(s) and s among s0 .. s0 + 4 (src/codec.rs:65-68); far: cf lies past the five candidates
    auto resolve_c = [](const uint4& g, uint32_t cf, uint32_t& p, uint32_t& r, uint32_t& sx, bool& far)
        __attribute__((always_inline)) {
        const uint32_t rel = cf - g.x;  // cf - cdf(s0); the candidates' offsets are cdf - cdf(s0)
        const uint32_t d0 = g.y >> 16, d1 = g.z & 0xFFFFu, d2 = g.z >> 16, d3 = g.w & 0xFFFFu, d4 = g.w >> 16;
        const bool b1 = rel >= d0, b2 = rel >= d1, b3 = rel >= d2, b4 = rel >= d3;
        // (lo, hi) = (d_{k-1}, d_k) as ONE packed word, selected among the five consecutive
        // 16-bit pairs of the sequence 0, d0, .., d4 (two of them funnelled by v_alignbit):
        // four selects where two chains of four selected lo and hi apart (r05)
        const uint32_t w1 = __builtin_amdgcn_alignbit(g.z, g.y, 16u);  // d0 | d1
        const uint32_t w3 = __builtin_amdgcn_alignbit(g.w, g.z, 16u);  // d2 | d3
        const uint32_t pr = b4 ? g.w : (b3 ? w3 : (b2 ? g.z : (b1 ? w1 : (g.y & 0xFFFF0000u))));
        p = (pr >> 16) - (pr & 0xFFFFu);
        r = rel - (pr & 0xFFFFu);
        sx = (g.y & 0xFFFFu) + (b1 ? 1u : 0u) + (b2 ? 1u : 0u) + (b3 ? 1u : 0u) + (b4 ? 1u : 0u);
        far = rel >= d4;
    };

    auto step = [&]() __attribute__((always_inline)) {
        // the chain's part up to the bucket loads at raised wave priority (ans_fast.hpp k_decode;
        // decode -1.4% in a same-box A/B)
        __builtin_amdgcn_s_setprio(2);
        ch.template renorm_div<kNR>(L, hL8, norm, rcp_norm, -static_cast<double>(norm));
        const uint32_t cf = ch.cf;
        const bool pre = kPrefix && cf < cpre;
        // global bucket (lanes past the prefix only): issued first, the longer round trip
        uint4 ga = make_uint4(0, 0, 0, 0), gb = make_uint4(0, 0, 0, 0);
        if (!pre) {
            if constexpr (kCompact && !kPrefix) {  // the LDS copy of the first nlb buckets, else L2
                // one load per lane into the same registers, L2 or LDS under complementary exec
                // masks (r05: the LDS read on every lane and a 4-dword select added 12 VALU per
                // symbol to the r04 decoder)
                const uint32_t bl = cf >> clshift;
                const uint4* gp = reinterpret_cast<const uint4*>(bktc + (cf >> cshift));  // c0 | s0, d0 | d1, d2 | d3, d4
                const uint4* lp = reinterpret_cast<const uint4*>(lds + kWideDecTab) + bl;  // (generic: the LDS aperture)
                ga = *(bl < nlb ? lp : gp);
            } else if constexpr (kCompact) {
                ga = *reinterpret_cast<const uint4*>(bktc + (cf >> cshift));  // c0 | s0, d0 | d1, d2 | d3, d4
            } else {
                const uint4* e = reinterpret_cast<const uint4*>(bkt + (cf >> shift));
                ga = e[0];
                gb = e[1];  // c0..c3 | c4, c5, s0, -
            }
        }
        __builtin_amdgcn_s_setprio(0);
        // LDS prefix (every lane; the bucket index clamped into the prefix)
        const uint32_t bi = umin(cf, cpre - 1) >> shp;
        const uint32_t s0 = *reinterpret_cast<const lds_u16*>(static_cast<uintptr_t>(kWideDecTab + 2 * bi));
        const uint32_t a0 = lcum + 4 * s0;
        const uint32_t c0 = *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(a0));
        const uint32_t c1 = *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(a0 + 4));
        const uint32_t c2 = *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(a0 + 8));
        const uint32_t c3 = *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(a0 + 12));
        const uint32_t c4 = *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(a0 + 16));
        // the pop's p = pmf(s) and r = cf - cdf(s) (src/codec.rs:65-68)
        uint32_t p, r, sx;
        bool far;
        if (pre) {
            const bool b1 = cf >= c1, b2 = cf >= c2, b3 = cf >= c3;
            const uint32_t cum = b3 ? c3 : (b2 ? c2 : (b1 ? c1 : c0));
            const uint32_t nxt = b3 ? c4 : (b2 ? c3 : (b1 ? c2 : c1));
            p = nxt - cum;
            r = cf - cum;
            sx = s0 + (b1 ? 1u : 0u) + (b2 ? 1u : 0u) + (b3 ? 1u : 0u);
            far = cf >= c4;
        } else if constexpr (kCompact) {
            asm volatile("" ::"v"(ga.x), "v"(ga.y), "v"(ga.z), "v"(ga.w));
            if constexpr (!kPrefix) {
                // lanes past a double-width LDS bucket's five candidates resolve on their global
                // bucket instead (screened before the resolve, so the step holds one resolve: two
                // inlined in each of the 64 unrolled steps stopped the unit loop unrolling and put
                // the symbol lines in scratch, decode +6%)
                const bool again = cf - ga.x >= (ga.w >> 16) && (cf >> clshift) < nlb && clshift != cshift;
                if (__builtin_expect(__any(again), 0)) {
                    if (again) ga = *reinterpret_cast<const uint4*>(bktc + (cf >> cshift));
                    asm volatile("" ::"v"(ga.x), "v"(ga.y), "v"(ga.z), "v"(ga.w));
                }
            }
            resolve_c(ga, cf, p, r, sx, far);
        } else {
            asm volatile("" ::"v"(ga.x), "v"(ga.y), "v"(ga.z), "v"(ga.w), "v"(gb.x), "v"(gb.y), "v"(gb.z));
            const bool b1 = cf >= ga.y, b2 = cf >= ga.z, b3 = cf >= ga.w, b4 = cf >= gb.x;
            const uint32_t cum = b4 ? gb.x : (b3 ? ga.w : (b2 ? ga.z : (b1 ? ga.y : ga.x)));
            const uint32_t nxt = b4 ? gb.y : (b3 ? gb.x : (b2 ? ga.w : (b1 ? ga.z : ga.y)));
            p = nxt - cum;
            r = cf - cum;
            sx = gb.z + (b1 ? 1u : 0u) + (b2 ? 1u : 0u) + (b3 ? 1u : 0u) + (b4 ? 1u : 0u);
            far = cf >= gb.y;
        }
        if (__builtin_expect(__any(far), 0)) {
            if (far) {  // more boundaries than candidates: scan the cdf (src/codec.rs:66 partition_point)
                sx += 1;
                uint32_t cum, nxt;
                if (pre) {
                    while (cf >= *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(lcum + 4 * (sx + 1)))) ++sx;
                    cum = *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(lcum + 4 * sx));
                    nxt = *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(lcum + 4 * (sx + 1)));
                } else {
                    while (cf >= gcum[sx + 1]) ++sx;
                    cum = gcum[sx];
                    nxt = gcum[sx + 1];
                }
                p = nxt - cum;
                r = cf - cum;
            }
        }
        ch.template update<kP24>(p, r);  // head = p*q + r (src/ans.rs:113-114)
        return sx;
    };

    // symbols leave in whole 128-B lines per lane (eight units; k_decode in ans_fast.hpp): the
    // last line of a chunk whose bytes are an odd multiple of 64 holds four units
    uint4 q[8];
    for (int u0 = 0; u0 < nunit; u0 += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (u0 + u < nunit) {  // (uniform)
                if (u % UPT == 0) {
                    wait_vm();  // point: retire what the previous point issued
                    if (u == 0 && u0 > 0) {
                        uint4* d = dst + (u0 - 8);
#pragma unroll
                        for (int k = 0; k < 8; ++k) d[k] = q[k];
                    }
                    ch.point();
                }
                uint4 outv = make_uint4(0, 0, 0, 0);
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    __builtin_amdgcn_sched_barrier(0);
                    if (kVar && static_cast<uint32_t>((u0 + u) * U + j) >= nvalid) continue;  // past the chunk
                    put_sym<Sym>(outv, j, step());
                }
                q[u] = outv;
            }
        }
    }
    wait_vm();
    if (nunit > 0) {
        const int rem = kVar ? 8 : ((nunit - 1) & 7) + 1;  // 4 or 8 (staged: the whole line)
        uint4* d = dst + ((nunit - 1) & ~7);
        if (rem == 8) {
#pragma unroll
            for (int k = 0; k < 8; ++k) d[k] = q[k];
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = q[k];
        }
    }
    // assert_eq!(initial, m) with initial = the chunk's initial message (src/ans.rs:56, 302-310)
    ch.pull_until(kMaxMinHead);
    const int32_t remaining = ch.P + 4 - ch.sh;  // < 0: generated
    if (remaining < 0 && gen_kind == ANS_GEN_EMPTY) atomicOr(status, 1u << ANS_E_EXHAUSTED);
    else if (ch.head != ini.head(c) || remaining != 0) atomicOr(status, 1u << ANS_E_MISMATCH);
}

}  // namespace fast
}  // namespace shuffle_coding
