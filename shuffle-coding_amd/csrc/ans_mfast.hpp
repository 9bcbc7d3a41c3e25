// ans_mfast.hpp — throughput kernels for the codecs beside IID<Categorical> (included by
// ans_codecs.hip): Independent<Categorical> (src/codec.rs:366-403) over a set of <= 256-symbol
// tables staged in LDS, IID<Uniform(size)> (src/codec.rs:13-49) and IID<LogUniform(E)>
// (src/codec.rs:561-611, the item of MaxBenfordIID, src/param_codec.rs:91-129).
//
// One lane = one chunk = one reference Message, exactly as in ans_fast.hpp, whose gfx950 idioms
// these kernels reuse: global memory touched only at wave-uniform points (s_waitcnt vmcnt(0)),
// whole 128-B lines per lane for symbols and stream pages, a per-lane [dword][lane] LDS ring
// for the stream, byte funnels through v_alignbyte / v_perm, the f64 quotient estimate with a
// voted exact fix-up.  What is new here is what these codecs need and IID<Categorical> does not:
//
//  * A model per codec (IndepModel, UniformModel, LogUniformModel below) supplies the per-symbol
//    push and pop; the skeletons (k_menc, k_mdec) own the chunk walk, the ring and the pages.
//  * 256-lane workgroups: the ring sits at LDS offset 0 (32 KiB encode, 33 KiB decode) and the
//    model's tables after it, so an Independent set of several 256-symbol tables still leaves
//    room for two workgroups per CU; 2^28 symbols in 4,096-symbol chunks (65,536 chains) then
//    fill every CU with one workgroup each.
//  * Codecs of different norms in one message (Independent, LogUniform's two Uniforms) make the
//    reference's renorm bidirectional (src/ans.rs:233-253): a push may first take back a byte it
//    pushed (renorm_up), a pop may hand one back (renorm_down).  Every head in the fast range is
//    >= 2^55 after a push (norm * K > 2^56 - norm), so either move is at most ONE byte, and the
//    stream position never falls more than one byte below its running maximum (encode) / rises
//    more than one above its running minimum (decode).  The encoder therefore flushes a page
//    only once the position is a byte past it (nothing flushed is ever taken back), and the
//    decoder's page landing (P < 64 low + 60) already leaves the byte above the window in the
//    ring.  Both moves are rare and run on wave-voted branches.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ans_fast.hpp"

namespace shuffle_coding {
namespace mfast {

using fast::ab;
using fast::ChunkInit;
using fast::hi32;
using fast::lds_ld128;
using fast::lds_ld32;
using fast::lds_ld64;
using fast::lds_u32;
using fast::lo32;
using fast::mk64;
using fast::shl16;
using fast::unroll_seq;
using fast::wait_vm;

constexpr int kLanes = 256;                       // chunks per workgroup
constexpr uint32_t kEncRingBytes = 32 * kLanes * 4;  // 128-B ring per lane: 32 KiB
constexpr uint32_t kDecRows = 33;                 // 32 ring rows + the mirror of row 0
constexpr uint32_t kDecRingBytes = kDecRows * kLanes * 4;  // 33 KiB
constexpr uint32_t kEncTab = kEncRingBytes;       // LDS offset of the encoder's model tables
constexpr uint32_t kDecTab = kDecRingBytes;       // LDS offset of the decoder's model tables
static_assert(kDecTab % 256 == 0, "tables 256-B aligned");
constexpr uint32_t kLdsMax = 160 * 1024;
constexpr uint64_t kMaxMinHead = 1ull << 56;  // src/ans.rs:19
// r05: the decoder's second layout, as ans_fast.hpp k_decode's: 1,024-lane workgroups (four
// waves per SIMD where a call has the chains: 2^30 u8 symbols in 4,096-symbol chunks is 1,024
// chains per CU) sharing ONE table image of at most kDecTabW bytes at LDS offset 0, the ring
// after it.  The 256-lane layout (ring at 0, tables after it) stays for images that do not fit.
constexpr int kLanesW = 1024;
constexpr uint32_t kDecTabW = 28672;
static_assert(kDecTabW + kDecRows * kLanesW * 4 == kLdsMax, "1,024 rings + the tables = one CU's LDS");
template <int kL>
struct DecLayout {
    static_assert(kL == kLanes || kL == kLanesW, "two layouts");
    static constexpr uint32_t kRing = kL == kLanes ? 0u : kDecTabW;   // LDS offset of ring row 0
    static constexpr uint32_t kTab = kL == kLanes ? kDecTab : 0u;     // LDS offset of the model's tables
    static constexpr uint32_t kRowShift = kL == kLanes ? 10u : 12u;   // log2 of a ring row's bytes
    static constexpr uint32_t kLds = kL == kLanes ? 0u : kLdsMax;     // (256 lanes: the caller's size)
};

// encoder error bits (lane-private; reported as ANS_E_* by the skeleton)
constexpr uint32_t kErrSymbol = 1;    // symbol outside the alphabet (src/codec.rs:63, LogUniform bits >= size)
constexpr uint32_t kErrZeroMass = 2;  // assert_ne!(p, 0) (src/ans.rs:98)
constexpr uint32_t kErrNormRange = 4; // Uniform::new(2^(bits-1)) beyond MAX_SIZE (src/codec.rs:35)
constexpr uint32_t kErrPulled = 8;    // a take-back reached past the stream's start (generator bytes)

// ====================================================================== encoder
// Two layouts, as the decoder's (DecLayout): 256 lanes with the ring at LDS offset 0 and the
// model's tables after it (kEncTab), or (r05) 1,024 lanes sharing ONE table image of at most
// kEncTabW bytes at offset 0 with the ring after it, four waves per SIMD where a call has the
// chains (1,024 per CU).  The stream's dword i lives in ring row i & 31: ((i & 31) << R) | 4 lane,
// R = log2 of a row's bytes.
constexpr uint32_t kEncTabW = 32768;
static_assert(kEncTabW + 32u * kLanesW * 4 == kLdsMax, "1,024 rings + the tables = one CU's LDS");
template <int kL>
struct EncLayout {
    static_assert(kL == kLanes || kL == kLanesW, "two layouts");
    static constexpr uint32_t kRing = kL == kLanes ? 0u : kEncTabW;
    static constexpr uint32_t kTab = kL == kLanes ? kEncTab : 0u;
    static constexpr uint32_t kRowShift = kL == kLanes ? 10u : 12u;
    static constexpr uint32_t kRowMask = 31u << kRowShift;
    static_assert(kL == kLanes || kRowShift == 12, "row_of's shift: (pos8 & 0x3E0) << 7");
    // the row address of stream bit position pos8 (dword pos8 >> 5), without the ring base
    static __device__ __forceinline__ uint32_t row_of(uint32_t pos8, uint32_t col) {
        if constexpr (kL == kLanes) {
            return (shl16<5>(pos8) & kRowMask) | col;  // (fits 16 bits)
        } else {  // the mask first, then one v_lshl_or (ans_fast.hpp DecChain::read_window)
            uint32_t a;
            asm("v_lshl_or_b32 %0, %1, 7, %2" : "=v"(a) : "v"(pos8 & 0x3E0u), "v"(col));
            return a;
        }
    }
};

template <int kL>
struct MRingT {
    using Lay = EncLayout<kL>;
    uint32_t col;
    __device__ __forceinline__ lds_u32& at(int32_t i) const {
        const uint32_t a = ((static_cast<uint32_t>(i) << Lay::kRowShift) & Lay::kRowMask) | col;
        return *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(a + Lay::kRing));
    }
};

// The byte funnel of ans_fast.hpp (FunnelT) on the ring, plus take_back: pos8 = 8 * stream bytes
// so far; X holds dword pos/4 with its pos&3 written bytes at the bottom; every dword below it
// is in the ring.  addr: the ring address (less the ring base) of dword pos/4.
template <int kL>
struct MFunnelT {
    using Lay = EncLayout<kL>;
    uint32_t X, pos8, neg8, addr, col;

    __device__ __forceinline__ void push(uint32_t lo, uint32_t k8) {
        uint32_t xv, d0, d1;
        asm("v_bfe_u32 %0, %1, 0, %2" : "=v"(xv) : "v"(X), "v"(pos8));
        asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(d0) : "v"(lo), "v"(pos8), "v"(xv));
        asm("v_lshrrev_b32 %0, %1, %2" : "=v"(d1) : "v"(neg8), "v"(lo));
        *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(addr + Lay::kRing)) = d0;
        pos8 += k8;
        neg8 -= k8;
        const uint32_t a = Lay::row_of(pos8, col);
        X = a != addr ? d1 : d0;
        addr = a;
    }
    // the last byte back (renorm_up during a push, src/ans.rs:239-243); pos8 > 0
    __device__ __forceinline__ uint32_t take_back() {
        pos8 -= 8;
        neg8 += 8;
        const uint32_t a = Lay::row_of(pos8, col);
        if (a != addr) {  // the byte lies in the dword below, which is in the ring
            X = *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(a + Lay::kRing));
            addr = a;
        }
        return (X >> (pos8 & 31u)) & 0xFFu;
    }
    __device__ __forceinline__ uint32_t len() const { return pos8 >> 3; }
    __device__ __forceinline__ void finish() {
        uint32_t xv;
        asm("v_bfe_u32 %0, %1, 0, %2" : "=v"(xv) : "v"(X), "v"(pos8));
        *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(addr + Lay::kRing)) = xv;
    }
};

// completed pages leave in aligned 128-B pairs (ans_fast.hpp PageOut)
struct MPageOut {
    uint4 h0, h1, h2, h3;
    template <class Ring>
    __device__ __forceinline__ void page(const Ring& ring, uint32_t p, uint8_t* dst) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = ring.at(static_cast<int32_t>(16 * p + i));
        const uint4 v0 = make_uint4(w[0], w[1], w[2], w[3]), v1 = make_uint4(w[4], w[5], w[6], w[7]);
        const uint4 v2 = make_uint4(w[8], w[9], w[10], w[11]), v3 = make_uint4(w[12], w[13], w[14], w[15]);
        if (p & 1) {
            uint4* d = reinterpret_cast<uint4*>(dst + 64ull * (p - 1));
            d[0] = h0;
            d[1] = h1;
            d[2] = h2;
            d[3] = h3;
            d[4] = v0;
            d[5] = v1;
            d[6] = v2;
            d[7] = v3;
        }
        h0 = v0;
        h1 = v1;
        h2 = v2;
        h3 = v3;
    }
    __device__ __forceinline__ void finish(uint32_t np, uint8_t* dst) {
        if (np & 1) {
            uint4* d = reinterpret_cast<uint4*>(dst + 64ull * (np - 1));
            d[0] = h0;
            d[1] = h1;
            d[2] = h2;
            d[3] = h3;
        }
    }
};

// One chain's encoder state, handed to the model's push.
template <int kL>
struct EncLaneT {
    uint64_t head;
    MFunnelT<kL> f;
    uint32_t err;
    // push the head's low 8k8/8 bytes (up to 8) and drop them from the head
    __device__ __forceinline__ void emit(uint32_t k8) {
        f.push(lo32(head), min(k8, 32u));
        if (k8 > 32u) f.push(hi32(head), k8 - 32u);
        head >>= k8;
    }
    __device__ __forceinline__ void emit4(uint32_t k8) {  // at most 4 bytes
        f.push(lo32(head), k8);
        head >>= k8;
    }
    // renorm_up: head = head << 8 | last byte while head < bound (src/ans.rs:239-243); at most one
    // byte for the fast range's heads, but exact whatever the count.  A take-back past the stream
    // start reads the tail generator; a byte container cannot carry that (kErrPulled).
    __device__ __forceinline__ void take_back_until(uint64_t bound) {
        for (int g = 0; g < 8 && head < bound; ++g) {
            uint32_t b = 0;
            if (f.pos8 == 0) err |= kErrPulled;
            else b = f.take_back();
            head = (head << 8) | b;
        }
    }
};
using MRing = MRingT<kLanes>;
using MFunnel = MFunnelT<kLanes>;
using EncLane = EncLaneT<kLanes>;

// 8 * #{j >= 1 : head >> 8j >= pK} (src/ans.rs:246-253), exact (the voted slow paths)
__device__ __forceinline__ uint32_t bytes_out8_exact(uint64_t head, uint64_t pK) {
    uint32_t k = 0;
    while (k < 7 && (head >> (8 * (k + 1))) >= pK) ++k;
    return 8 * k;
}

// symbol j of a 16-B unit (u8 / u16 / u32 in the low bits; u64 as (lo, hi))
template <typename Sym>
__device__ __forceinline__ void unit_sym(const uint4& v, int j, uint32_t& lo, uint32_t& hi) {
    if constexpr (sizeof(Sym) == 8) {
        lo = j == 0 ? v.x : v.z;
        hi = j == 0 ? v.y : v.w;
    } else {
        constexpr int per = 4 / static_cast<int>(sizeof(Sym));
        const int wi = j / per, sh = 8 * static_cast<int>(sizeof(Sym)) * (j % per);
        const uint32_t w = wi == 0 ? v.x : wi == 1 ? v.y : wi == 2 ? v.z : v.w;
        lo = sizeof(Sym) == 4 ? w : (w >> sh) & ((1u << (8 * sizeof(Sym))) - 1u);
        hi = 0;
    }
}
template <typename Sym>
__device__ __forceinline__ void unit_put(uint4& v, int j, uint32_t lo, uint32_t hi) {
    if constexpr (sizeof(Sym) == 8) {
        if (j == 0) {
            v.x = lo;
            v.y = hi;
        } else {
            v.z = lo;
            v.w = hi;
        }
    } else {
        constexpr int per = 4 / static_cast<int>(sizeof(Sym));
        const int wi = j / per, sh = 8 * static_cast<int>(sizeof(Sym)) * (j % per);
        uint32_t& w = wi == 0 ? v.x : wi == 1 ? v.y : wi == 2 ? v.z : v.w;
        w = (j % per) == 0 ? lo : (w | (lo << sh));
    }
}

// The encode skeleton.  Chunk c (< nfull: every chunk holds chunk_len symbols, chunk_len * w a
// multiple of 128) is IID / Independent::push of its symbols last first (src/codec.rs:388-391,
// 415-420) from the chunk's initial message, then flatten (src/ans.rs:255-260), into slot c.
// Symbols (and table ids) come in 128-B groups per lane (64 B for 1,024 lanes), walked last to first; a point (the
// page flush) precedes every SPP symbols, which emit at most 64 bytes between them.
// kL: the layout (EncLayout; the model's tables must be built for it, Model::kTabE).
template <class Model, typename Sym, int SPP, int kL = kLanes>
__global__ __launch_bounds__(kL, kL == kLanes ? 2 : 1) void k_menc(Model md, const Sym* __restrict__ syms,
                                                                   const uint8_t* __restrict__ tids, uint64_t chunk_len,
                                                                   uint64_t nfull, uint8_t* __restrict__ slots,
                                                                   uint64_t slot_cap, uint32_t* __restrict__ lens,
                                                                   uint32_t* __restrict__ status, ChunkInit ini) {
    extern __shared__ __align__(16) unsigned char lds[];
    static_assert(Model::kTabE == EncLayout<kL>::kTab, "the model's tables where the layout puts them");
    md.stage_enc(lds + EncLayout<kL>::kTab, kL);
    __syncthreads();
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kL + threadIdx.x;
    if (c >= nfull) return;

    constexpr int U = 16 / static_cast<int>(sizeof(Sym));  // symbols per 16-B unit
    static_assert(U % SPP == 0 || SPP % U == 0, "points split units evenly");
    // units per group: 128 B, each group requested while the one before it is coded (kPre),
    // except: 1,024 lanes (128 VGPRs) cannot hold two 128-B groups of symbols and table ids
    // beside the chain (the u8 encoder spilled 190), so there a 128-B group is loaded at its own
    // start, its latency covered by the SIMD's other three waves (r05: 64-B groups with the
    // prefetch read 4.1 GB per launch for 2.15 GB of symbols and ids at 2^30 u8, each line's
    // other half coming back from HBM after eviction); and u8 symbols without table ids
    // (Uniform / LogUniform, 16 symbols a unit: the 128 unrolled pushes of a 128-B group reached
    // 256 VGPRs and spilled 76) take 64-B groups
    constexpr bool kPre = kL == kLanes;
    constexpr int GU = (kL == kLanes && sizeof(Sym) == 1 && !Model::kTids) ? 4 : 8;
    constexpr int GS = GU * U;                               // symbols per group
    constexpr int TB = GS;                                   // table-id bytes per group
    const uint4* src = reinterpret_cast<const uint4*>(syms + c * chunk_len);
    const uint8_t* tsrc = Model::kTids ? tids + c * chunk_len : nullptr;
    uint8_t* dst = slots + c * slot_cap;
    const uint32_t npages_cap = static_cast<uint32_t>(slot_cap / 64);
    const int ngroups = static_cast<int>(chunk_len * sizeof(Sym) / (16 * GU));

    const MRingT<kL> ring{4 * threadIdx.x};
    MPageOut pout;
    EncLaneT<kL> e;
    e.head = ini.head(c);  // Message::zeros() / random(seed + c)
    e.f = MFunnelT<kL>{0, 0, 0, ring.col, ring.col};
    e.err = 0;
    uint32_t fp = 0, over = 0;
    // page fp leaves once the position is a byte past it: a take-back never reaches a flushed page
    auto flush_ready = [&]() __attribute__((always_inline)) {
        if (e.f.pos8 >= 512u * fp + 520u) {
            if (fp < npages_cap) pout.page(ring, fp, dst);
            else over = 1;
            ++fp;
        }
    };

    uint4 n[GU], tn[GU];
#pragma unroll
    for (int i = 0; i < GU; ++i) {
        n[i] = make_uint4(0, 0, 0, 0);
        tn[i] = make_uint4(0, 0, 0, 0);
    }
    auto load_group = [&](int g) __attribute__((always_inline)) {
        const uint4* gs = src + GU * g;
#pragma unroll
        for (int i = 0; i < GU; ++i) n[i] = gs[i];
        if constexpr (Model::kTids) {
            const uint4* gt = reinterpret_cast<const uint4*>(tsrc + static_cast<uint64_t>(TB) * g);
#pragma unroll
            for (int i = 0; i < TB / 16; ++i) tn[i] = gt[i];
        }
    };
    if (kPre && ngroups > 0) load_group(ngroups - 1);
    for (int g = ngroups - 1; g >= 0; --g) {
        if constexpr (!kPre) load_group(g);
        uint4 cc[GU], tc[GU];
#pragma unroll
        for (int i = 0; i < GU; ++i) {
            cc[i] = n[i];
            tc[i] = tn[i];
        }
        auto unit = [&](auto ic) __attribute__((always_inline)) {
            constexpr int u = GU - 1 - decltype(ic)::value;  // last unit first
            if (kPre && u == GU / 2 - 1 && g > 0) load_group(g - 1);
#pragma unroll
            for (int j = U - 1; j >= 0; --j) {  // last symbol first (src/codec.rs:417)
                if ((j + 1) % SPP == 0 || j == U - 1) flush_ready();
                __builtin_amdgcn_sched_barrier(0);
                // the symbol's words pass a volatile fence first, so that their unpacking stays
                // at the push (hoisted to the group's start, the unpacked symbols of a whole
                // group were held in registers and spilled)
                // (u8 / u16 symbols and the table ids: the field extract itself is the volatile
                // asm, where an empty "+v" fence on the word made the compiler copy the word, which
                // the later symbols of the unit still read: two v_mov per push, r05)
                uint32_t lo, hi;
                if constexpr (sizeof(Sym) <= 2) {
                    constexpr int per = 4 / static_cast<int>(sizeof(Sym));
                    const int wi = j / per;  // (folded: j is unrolled)
                    const uint32_t word = wi == 0 ? cc[u].x : wi == 1 ? cc[u].y : wi == 2 ? cc[u].z : cc[u].w;
                    asm volatile("v_bfe_u32 %0, %1, %2, %3"
                                 : "=v"(lo)
                                 : "v"(word), "i"(8 * static_cast<int>(sizeof(Sym)) * (j % per)),
                                   "i"(8 * static_cast<int>(sizeof(Sym))));
                    hi = 0;
                } else {
                    uint4 cv = cc[u];
                    if constexpr (sizeof(Sym) == 8) {
                        if (j == 0) asm volatile("" : "+v"(cv.x), "+v"(cv.y));
                        else asm volatile("" : "+v"(cv.z), "+v"(cv.w));
                    } else {
                        const int wi = j;  // (u32: a word per symbol)
                        if (wi == 0) asm volatile("" : "+v"(cv.x));
                        else if (wi == 1) asm volatile("" : "+v"(cv.y));
                        else if (wi == 2) asm volatile("" : "+v"(cv.z));
                        else asm volatile("" : "+v"(cv.w));
                    }
                    unit_sym<Sym>(cv, j, lo, hi);
                }
                uint32_t tid = 0;
                if constexpr (Model::kTids) {
                    const int tb = u * U + j;  // table-id byte of this symbol within the group
                    const uint4& tv = tc[tb / 16];
                    const int wi = (tb % 16) / 4;
                    const uint32_t w = wi == 0 ? tv.x : wi == 1 ? tv.y : wi == 2 ? tv.z : tv.w;
                    // (the low and the top byte by the fast-class v_and / v_lshrrev)
                    if (tb % 4 == 0) asm volatile("v_and_b32 %0, 0xff, %1" : "=v"(tid) : "v"(w));
                    else if (tb % 4 == 3) asm volatile("v_lshrrev_b32 %0, 24, %1" : "=v"(tid) : "v"(w));
                    else asm volatile("v_bfe_u32 %0, %1, %2, 8" : "=v"(tid) : "v"(w), "i"(8 * (tb % 4)));
                }
                md.template push<decltype(e), sizeof(Sym) == 1>(e, lo, hi, tid);
            }
        };
        unroll_seq(unit, std::make_integer_sequence<int, GU>{});
    }
    flush_ready();  // the flatten's 8 bytes then stay within the page after the held one

    // flatten (src/ans.rs:255-260): all significant head bytes, low first (7 or 8: head > 2^55)
    const uint32_t nb = (71u - static_cast<uint32_t>(__builtin_clzll(e.head))) >> 3;
    e.f.push(lo32(e.head), 32);
    e.f.push(hi32(e.head), 8 * (nb - 4));
    e.f.finish();
    const uint32_t len = e.f.len();
    for (const uint32_t last = (len + 63) / 64; fp < last; ++fp) {
        if (fp < npages_cap) pout.page(ring, fp, dst);
        else over = 1;
    }
    if (!over) pout.finish(fp, dst);
    uint32_t err = e.err;
    if (err & kErrZeroMass) err = md.classify(syms + c * chunk_len, tsrc, chunk_len, err);
    if (err) {
        const int code = (err & kErrSymbol) ? ANS_E_SYMBOL : (err & kErrNormRange) ? ANS_E_NORM_RANGE
                         : (err & kErrZeroMass) ? ANS_E_ZERO_MASS : ANS_E_MISMATCH;
        atomicOr(status, 1u << code);
    }
    if (over) atomicOr(status, 1u << ANS_E_LEN);
    lens[c] = (over || err) ? 0u : len;
}

// ====================================================================== decoder
// The ans_fast.hpp DecChain on a 256-lane ring at LDS offset 0 (33 rows, row 32 mirrors row 0),
// plus the renorm_down (push-back) of the bidirectional renorm and the two-round pull of codecs
// whose pops can take more than four bytes (Uniform and LogUniform sizes up to 2^46).
__device__ const uint4 kZeroPair[8] = {};  // the Zeros tail generator's bytes below a stream

template <int kL>
struct MChainT {
    using Lay = DecLayout<kL>;
    const uint8_t* src;
    uint4 Q[8];
    int32_t low, P8, lim8;
    uint32_t W, wx, wy, col;
    uint64_t head;
    bool bad;  // a pushed-back byte that differs from the stream's: corrupt (ANS_E_MISMATCH)

    // sixteen ring rows from one address: rows kL * 4 bytes = kL / 64 st64 units apart
    template <int R0>
    __device__ __forceinline__ uint32_t put_half(uint4 a0, uint4 a1, uint4 a2, uint4 a3) {
        constexpr int st = kL / 64;
        const uint32_t base = col + Lay::kRing + R0 * kL * 4;
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
            : "v"(base), "v"(a0.x), "v"(a0.y), "v"(a0.z), "v"(a0.w), "v"(a1.x), "v"(a1.y), "v"(a1.z), "v"(a1.w),
              "v"(a2.x), "v"(a2.y), "v"(a2.z), "v"(a2.w), "v"(a3.x), "v"(a3.y), "v"(a3.z), "v"(a3.w),
              "i"(0), "i"(st), "i"(2 * st), "i"(3 * st), "i"(4 * st), "i"(5 * st), "i"(6 * st), "i"(7 * st),
              "i"(8 * st), "i"(9 * st), "i"(10 * st), "i"(11 * st), "i"(12 * st), "i"(13 * st), "i"(14 * st),
              "i"(15 * st)
            : "memory");
        return a0.x;
    }
    __device__ __forceinline__ void put_page(int32_t p) {
        if (p & 1) {
            put_half<16>(Q[4], Q[5], Q[6], Q[7]);
        } else {
            const uint32_t r0 = put_half<0>(Q[0], Q[1], Q[2], Q[3]);
            *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(col + Lay::kRing + 32u * kL * 4)) = r0;  // mirror
        }
    }
    __device__ __forceinline__ void fetch_pair(int32_t m) {
        typedef __attribute__((address_space(1), aligned(1))) const fast::v4u32 gv4;
        const uint4* g = m >= 0 ? reinterpret_cast<const uint4*>(src + 128ll * m) : kZeroPair;
        const gv4* gg = reinterpret_cast<const gv4*>(reinterpret_cast<uintptr_t>(g));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const fast::v4u32 v = gg[k];
            Q[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
    }
    // the top pair as the aligned dwords holding stream bytes (no read past the stream's line)
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
    // ring row (P8 >> 5) & 31 of the lane's column (the ring base added by the caller / offsets)
    __device__ __forceinline__ uint32_t row_addr(int32_t p8) const {
        uint32_t a;
        asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(a) : "v"(static_cast<uint32_t>(p8) & 0x3E0u), "i"(Lay::kRowShift - 5), "v"(col));
        return a;
    }
    // W = stream bytes [P, P+4): ring rows (P>>2)&31 and the next; P8 = 8P
    __device__ __forceinline__ void read_window() {
        const uint32_t a = row_addr(P8);
        wy = lds_ld32(a + Lay::kRing);
        wx = lds_ld32(a + Lay::kRing + 4 * kL);
    }
    __device__ __forceinline__ void form_window() { W = __builtin_amdgcn_alignbit(wx, wy, static_cast<uint32_t>(P8)); }
    __device__ __forceinline__ void start(const uint8_t* s, int32_t len) {
        src = s;
        bad = false;
        const int32_t top = len > 0 ? (len - 1) >> 6 : 0;
        if (len > 0) fetch_top(top >> 1, len);
        else fetch_pair(-1);
        wait_vm();
        put_page(top);
        if (top & 1) {
            put_page(top - 1);
            fetch_pair((top >> 1) - 1);
        } else {
            fetch_pair((top >> 1) - 1);
            wait_vm();
            put_page(top - 1);
        }
        low = top - 1;
        lim8 = 8 * (64 * low + 60);
        P8 = 8 * (len - 4);
        read_window();
        head = 0;
    }
    __device__ __forceinline__ void pull_until(uint64_t bound) {
        for (int g = 0; g < 9 && head < bound; ++g) {
            form_window();
            head = (head << 8) | (W >> 24);
            P8 -= 8;
            read_window();
        }
    }
    __device__ __forceinline__ void point() {
        if (P8 < lim8) {
            put_page(low - 1);
            --low;
            lim8 -= 512;
            if (!(low & 1)) fetch_pair((low >> 1) - 1);
        }
    }
    // renorm(L) (src/ans.rs:233-253) from the window W: head = head << 8k | the top k bytes of W for
    // the least k in 0..4 that reaches L (ans_fast.hpp renorm_up8: byte permutes from the clz),
    // or, when head >> 8 >= L already (a codec of a smaller L before this one), renorm_down: the
    // head's low byte goes back onto the stream (P moves up one byte), where it must equal the
    // stream's own byte (checked against the ring; a mismatch is a corrupt stream).  Both rare
    // cases sit behind one 32-bit screen voted per wave.  Returns the bits the position moves down.
    // kJ4 = false: no pop leaves the high word zero (every row's p K >= 2^32, ans_fast.hpp
    // renorm_up8), so js = clz >> 3 needs no clamp
    static __device__ __forceinline__ uint64_t l_of(uint64_t L) { return L; }
    template <class F>
    static __device__ __forceinline__ uint64_t l_of(const F& f) { return f(); }
    // (L: the bound, or a callable that reads it: only the rare path needs it)
    template <bool kJ4 = true, class LT = uint64_t>
    __device__ __forceinline__ int32_t renorm_up8(const LT& L, uint32_t hL8) {
        const uint32_t h1 = hi32(head), h0 = lo32(head);
        uint32_t fb;
        asm("v_ffbh_u32 %0, %1" : "=v"(fb) : "v"(h1));
        const uint32_t m = kJ4 ? min(fb, 32u) & 0x38u : fb & 0x18u;  // 8 js
        const uint32_t sel = hi32(0x0706050403020100ull << m);
        const uint32_t xj1 = __builtin_amdgcn_perm(h1, h0, sel), xj0 = __builtin_amdgcn_perm(h0, W, sel);
        head = mk64(xj1, xj0);
        int32_t m8 = static_cast<int32_t>(m);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(xj1 >= hL8) != 0, 0)) {
            const uint32_t xm1 = xj1 >> 8, xm0 = ab(xj1, xj0, 1);
            if (xj1 >= hL8 && mk64(xm1, xm0) >= l_of(L)) {
                head = mk64(xm1, xm0);
                m8 -= 8;
                if (m == 0) {  // renorm_down: byte xj0 & 0xFF back onto the stream at P + 4
                    const int32_t p8 = P8 + 32;
                    const uint32_t byte = (lds_ld32(row_addr(p8) + Lay::kRing) >> (static_cast<uint32_t>(p8) & 31u)) & 0xFFu;
                    bad |= byte != (xj0 & 0xFFu);
                }
            }
        }
        return m8;
    }
    // renorm to L for heads that may need more than four bytes (a second round, voted)
    __device__ __forceinline__ void renorm_wide(uint64_t L, uint32_t hL8) {
        form_window();
        P8 -= renorm_up8(L, hL8);
        read_window();
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(head < L) != 0, 0)) {
            if (head < L) {
                form_window();
                P8 -= renorm_up8(L, hL8);
                read_window();
            }
        }
    }
};

using MChain = MChainT<kLanes>;

// The decode skeleton: chunk c's stream read from its end (Tail::pop, src/ans.rs:198-203),
// unflatten (src/ans.rs:262-264), then IID / Independent::pop forward (src/codec.rs:393-399,
// 422-424); the symbols leave in whole 128-B lines (64 B for 1,024 lanes); at the end the message must be back at the
// chunk's initial one (src/ans.rs:56).  A point precedes every SPP symbols (at most 60 stream
// bytes between points, so no window read reaches an unlanded page).
// kL: the layout (DecLayout: 256 lanes, or 1,024 sharing one table image at LDS offset 0; the
// model's tables must be built for it, Model::kTab).
template <class Model, typename Sym, int SPP, int kL = kLanes>
__global__ __launch_bounds__(kL, kL == kLanes ? 2 : 1) void k_mdec(Model md, const uint8_t* __restrict__ slots,
                                                                   uint64_t slot_cap,
                                                                   const uint64_t* __restrict__ offsets,
                                                                   const uint32_t* __restrict__ lens,
                                                                   const uint8_t* __restrict__ tids, uint64_t chunk_len,
                                                                   uint64_t nfull, int gen_kind, Sym* __restrict__ out,
                                                                   uint32_t* __restrict__ status, ChunkInit ini) {
    extern __shared__ __align__(16) unsigned char lds[];
    static_assert(Model::kTab == DecLayout<kL>::kTab, "the model's tables where the layout puts them");
    md.stage_dec(lds + DecLayout<kL>::kTab, kL);
    __syncthreads();
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kL + threadIdx.x;
    if (c >= nfull) return;

    constexpr int U = 16 / static_cast<int>(sizeof(Sym));
    static_assert(U % SPP == 0 || SPP % U == 0, "points split units evenly");
    const int nunit = static_cast<int>(chunk_len / U);  // chunk_len * w is a multiple of 128: whole lines
    uint4* dst = reinterpret_cast<uint4*>(out + c * chunk_len);
    const uint8_t* tsrc = Model::kTids ? tids + c * chunk_len : nullptr;

    if ((!offsets && lens[c] > slot_cap) || lens[c] >= (1u << 27)) {
        atomicOr(status, 1u << ANS_E_LEN);
        return;
    }
    MChainT<kL> ch;
    ch.col = 4 * threadIdx.x;
    ch.start(slots + (offsets ? offsets[c] : c * slot_cap), static_cast<int32_t>(lens[c]));
    ch.pull_until(md.first_bound(tsrc));  // Message::unflatten: head 0, the first pop's renorm_up
    typename Model::DecState ds;
    md.dec_init(ds);

    // a line: LU units of output (128 B; 64 B for 1,024 lanes, whose 128 VGPRs cannot hold two
    // 128-B id lines and an output line beside the chain: 40 VGPRs spilled)
    constexpr int LU = kL == kLanes ? 8 : 4;
    // the table ids of a line (LU * U bytes, one u32 word per four ids) and of the next line,
    // whose load is issued at the line's first point: whole lines per load (r05: 16-B loads a
    // unit apart left each lane's id line to be evicted between them, 5.3 GB read per launch for
    // 2.1 GB of stream and ids at 2^30 u8 symbols).
    // r06, 1,024 lanes (kPair): with one 64-B id load per 64-B output line, a line ahead, each
    // 128-B id line's second half came back from HBM 64 pops after its first (3.14 GB read per
    // launch for 2.11 GB, profiles/r05t_codecs_pmc.json).  Now the two halves of a 128-B id line
    // (the ids of lines 2m and 2m + 1) are fetched one unit (16 pops) apart: the even half in
    // the last unit of line 2m - 1, the odd half at the first point of line 2m, so the line is
    // still in L2 for the second.  The ids (< kIndMaxTables = 15 on these kernels: four bits) of
    // both lines are held packed, even line in the low nibble of each byte, odd in the high one:
    // each landed half is merged into its nibbles (two VALU per word, 1/4 VALU per pop for u8),
    // 16 VGPRs for the pair as for one line before (holding a whole 128-B load spilled at 1,024
    // lanes' 128 VGPRs), and a line's id is one v_bfe at nibble 4 * (line & 1).  (Not for
    // kNormSmall sets, Model::kPairIds: their longer pop leaves no room for it, 12-20 B spilled.)
    constexpr bool kPair = Model::kTids && kL == kLanesW && Model::kPairIds;
    constexpr int TW = LU * U / 4;  // u32 words of ids per line
    uint32_t tl[TW], tn[TW];
#pragma unroll
    for (int k = 0; k < TW; ++k) tl[k] = tn[k] = 0;
    auto load_ids = [&](int line, uint32_t* w) __attribute__((always_inline)) {
        const uint4* g = reinterpret_cast<const uint4*>(tsrc + static_cast<int64_t>(LU) * U * line);
#pragma unroll
        for (int k = 0; k < TW / 4; ++k) {
            const uint4 v = g[k];
            w[4 * k] = v.x;
            w[4 * k + 1] = v.y;
            w[4 * k + 2] = v.z;
            w[4 * k + 3] = v.w;
        }
    };
    auto merge_ids = [&](bool odd) __attribute__((always_inline)) {  // tn (landed) -> tl's nibbles
#pragma unroll
        for (int k = 0; k < TW; ++k) {
            if constexpr (kPair) {
                uint32_t w;
                if (odd) asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(w) : "v"(0xF0F0F0F0u), "v"(tn[k] << 4), "v"(tl[k]));
                else asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(w) : "v"(0x0F0F0F0Fu), "v"(tn[k]), "v"(tl[k]));
                tl[k] = w;
            } else {
                tl[k] = tn[k];
            }
        }
    };
    if constexpr (Model::kTids) {
        if (nunit > 0) load_ids(0, tn);
    }
    uint4 q[LU];
    for (int u0 = 0; u0 < nunit; u0 += LU) {
        const uint32_t par = kPair ? static_cast<uint32_t>(u0 / LU) & 1u : 0u;  // (uniform) line parity
        auto unit = [&](auto ic) __attribute__((always_inline)) {
            constexpr int uu = decltype(ic)::value;
            uint4 outv = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int j = 0; j < U; ++j) {
                if (j % SPP == 0) {
                    wait_vm();  // point
                    if constexpr (Model::kTids && !kPair) {
                        if (j == 0 && uu == 0) {
                            merge_ids(false);  // this line's ids (landed at this point)
                            if (u0 + LU < nunit) load_ids(u0 / LU + 1, tn);  // the next line's
                        }
                    }
                    if constexpr (kPair) {
                        if (j == 0 && uu == 0 && par == 0) {
                            merge_ids(false);             // line 2m's half (landed at this point)
                            load_ids(u0 / LU + 1, tn);    // line 2m + 1's half, one unit later
                        }
                        if (j == 0 && uu == 1 && par == 0) merge_ids(true);
                        if (j == 0 && uu == LU - 1 && par == 1 && u0 + LU < nunit) load_ids(u0 / LU + 1, tn);
                    }
                    if (j == 0 && uu == 0 && u0 > 0) {
                        uint4* d = dst + (u0 - LU);
#pragma unroll
                        for (int k = 0; k < LU; ++k) d[k] = q[k];
                    }
                    ch.point();
                }
                __builtin_amdgcn_sched_barrier(0);
                uint32_t tid = 0;
                if constexpr (Model::kTids) {
                    const int tb = uu * U + j;  // id byte within the line (the pop fences the id)
                    if constexpr (kPair) tid = __builtin_amdgcn_ubfe(tl[tb / 4], 8 * (tb % 4) + 4 * par, 4);
                    else tid = (tl[tb / 4] >> (8 * (tb % 4))) & 0xFFu;
                }
                uint32_t hi = 0;
                uint32_t lo = md.pop(ch, ds, tid, hi);
                // the symbol is formed here (volatile fences keep their order): otherwise the
                // compiler sank every pop's symbol arithmetic to the line's store and kept its
                // operands (the table header among them) alive across 128 pops, in scratch
                if constexpr (sizeof(Sym) == 8) asm volatile("" : "+v"(lo), "+v"(hi));
                else asm volatile("" : "+v"(lo));
                unit_put<Sym>(outv, j, lo, hi);
            }
            asm volatile("" : "+v"(outv.x), "+v"(outv.y), "+v"(outv.z), "+v"(outv.w));
            q[uu] = outv;
        };
        unroll_seq(unit, std::make_integer_sequence<int, LU>{});
    }
    wait_vm();
    if (nunit > 0) {  // the last line (nunit is a multiple of 8: chunk bytes % 128 == 0)
        uint4* d = dst + (nunit - LU);
#pragma unroll
        for (int k = 0; k < LU; ++k) d[k] = q[k];
    }
    // assert_eq!(initial, m) (src/ans.rs:56, 302-310)
    ch.pull_until(kMaxMinHead);
    const int32_t remaining = (ch.P8 >> 3) + 4;  // < 0: generated
    if (remaining < 0 && gen_kind == ANS_GEN_EMPTY) atomicOr(status, 1u << ANS_E_EXHAUSTED);
    else if (ch.bad || md.dec_bad(ds) || ch.head != ini.head(c) || remaining != 0) atomicOr(status, 1u << ANS_E_MISMATCH);
}

// ====================================================================== helpers for the models
// floor(x / d) for any u64 x and 1 <= d < 2^64, from m = floor((2^64 - 1) / d): the product's
// high word is q or q - 1 (m >= 2^64/d - 1), one compare fixes it.  r = x - q d.
__device__ __forceinline__ uint64_t mulhi64(uint64_t a, uint64_t b) { return __umul64hi(a, b); }
__device__ __forceinline__ uint64_t div_magic(uint64_t x, uint64_t d, uint64_t m, uint64_t& r) {
    uint64_t q = mulhi64(x, m);
    r = x - q * d;
    if (r >= d) {
        ++q;
        r -= d;
    }
    return q;
}

// stage `bytes` (a multiple of 16) of a global image into LDS (every thread of a workgroup of nl)
__device__ __forceinline__ void stage_image(const uint4* __restrict__ g, uint32_t bytes, unsigned char* l,
                                            uint32_t nl = kLanes) {
    uint4* d = reinterpret_cast<uint4*>(l);
    for (uint32_t i = threadIdx.x; i < bytes / 16; i += nl) d[i] = g[i];
}

struct NoState {
    __device__ __forceinline__ bool bad() const { return false; }
};

// ====================================================================== Independent<Categorical>
// A set of T <= kIndMaxTables Categoricals with <= 256 symbols, all in one norm range (kNR)
// (src/codec.rs:51-92), a table per position (src/codec.rs:366-403), table ids as one byte each.
//
// Encoder image (LDS kTabE, the same bytes in global memory; r05: 24 B per row, so five 256-
// symbol tables fit the 1,024-lane layout's 32 KiB): for row i = 257 t + s (s >= nsym: zero mass)
// {p, cdf(s), w (u64)} at 16 i (one ds_read_b128: every 16-B read spans the LDS bank quads, where
// 32-B rows used half of them), rcp = 1/p (f64) at ro + 8 i, {norm_t, -0x43300000 norm_t mod 2^32}
// at no + 8 t, K_t (u64) at k_off + 8 t and, for sets with screened rows (kRare), screen (u32) at
// so + 4 i.  At most 15
// tables (16 i below 2^16).  w is the renorm word: every push starts from head in
// [Hmin, 2^64) (Hmin = min_t norm_t K_t > 2^56 - 2^31, or the chunk's initial head), where the
// bounds pK 2^8j (src/ans.rs:246-253) below Hmin always count, and with T = the first above it,
// k = k0 + [head >= T] whenever 2^8 T >= 2^64: w = T + 8 k0 (T's low byte is zero), one compare
// as in ans_renorm.hpp.  Rows where that fails (2^8 T < 2^64, or pK = 2^56), or where a push can
// start below pK and take a byte back (pK > Hmin: a symbol of probability above 1 - 2^-25), get
// a screen: hi32(head) <= screen sends the lane to the exact renorm on a voted branch (kRare;
// sets without such rows compile it out).
//
// Decoder image (LDS kDecTab): a 16-B header per table at 16 t {1/norm (f64; lean standard-range
// sets 1/(8 norm)), norm, us | (bucket 0's offset / 8) << 5 | 257 t << 19}, L = norm K (u64) at
// kIndLOff + 8 t (read only by the renorm's rare path and the unflatten), the renorm screen the
// constant 0xFFFFFF00 for every table (r05: one ds_read_b128 per pop where a 32-B header took
// two; the decoder is LDS-bound), the (cdf(s), pmf(s)) rows of every table at
// kIndRowOff + 8 (t*257 + s), then each table's icdf
// buckets of width 2^us (ans_fast.hpp kModeU's folded words): bucket j at a = j << us holds
// w1 = ((min(cdf(s0+1) - a, 2^us) - 1) << rshift) | s0 and w2 the same for cdf(s0+2) (where
// cdf(s0+3) still lies inside the bucket, cf beyond s0+2 shows as cf - cdf(s) >= pmf(s) on the
// row and takes a voted scan of the rows).  rshift = 32 - us >= 10 keeps the 9-bit symbol clear,
// so a table of norm 2^31 needs only 512 buckets.
constexpr uint32_t kIndMaxTables = 15;                  // 16 (257 t + s) < 2^16
constexpr uint32_t kIndHdrBytes = 16;                   // decoder header per table at kIndHdrBytes t
constexpr uint32_t kIndLOff = 256;                      // L_t at kIndLOff + 8 t (the renorm's rare path)
constexpr uint32_t kIndRowOff = 1024;                   // decoder rows after the headers
constexpr uint32_t kIndBktShift = 5;                    // header word: us | bucket offset / 8 << 5 | 257 t << 19
constexpr uint32_t kIndRowShift = 19;
static_assert(kIndHdrBytes * kIndMaxTables <= kIndLOff && kIndLOff + 8 * kIndMaxTables <= kIndRowOff, "header area");
static_assert(257 * (kIndMaxTables - 1) < (1u << (32 - kIndRowShift)), "row index field");
constexpr uint32_t kScreenAll = 0xFFFFFF00u;  // hi32(L) << 8 >= this for every norm < 2^32 (L > 2^56 - 2^32)
constexpr uint32_t kIndMaxShift = 22;                   // rshift = 32 - us >= 10

// kNR (ans_fast.hpp kNormStd / kNormSmall / kNormBig): every table of the set in that norm range;
// kNormSmall rows carry 1/p rounded up and the headers 1/norm rounded up (the long division).
// kTab: the LDS offset of the decoder image (DecLayout: kDecTab for 256-lane decoders, 0 for the
// 1,024-lane one; the image's bucket addresses are built for it, IndepFast::dec_wide).
// kLean (decoder): every mass and hi32(q) is below 2^24 (the update's high word by one
// v_mad_u32_u24, as ans_fast.hpp DecChain::update<kP24>), every row's p K is at least 2^32
// (kmax <= 3: the renorm's byte count needs no clamp) and, in the standard range, every norm is
// at least 2^20 (the quotient rounded to nearest with a voted fix-up, pop).
// kTabE: the LDS offset of the encoder image (EncLayout: kEncTab for 256-lane encoders, 0 for
// the 1,024-lane one).
template <bool kRare, int kNR = fast::kNormStd, uint32_t kTabD = kDecTab, bool kLean = false,
          uint32_t kTabEnc = kEncTab>
struct IndepModel {
    static constexpr bool kTids = true;
    static constexpr bool kPairIds = kNR != fast::kNormSmall;  // k_mdec's paired id halves (1,024 lanes)
    static constexpr uint32_t kTab = kTabD;
    static constexpr uint32_t kTabE = kTabEnc;
    using DecState = NoState;
    const uint4* enc_img;
    const uint4* dec_img;
    const uint32_t* nsym;  // per table, global (error classification)
    uint32_t enc_bytes, dec_bytes, k_off, ro, no, so;

    __device__ __forceinline__ void stage_enc(unsigned char* l, uint32_t nl) const { stage_image(enc_img, enc_bytes, l, nl); }
    __device__ __forceinline__ void stage_dec(unsigned char* l, uint32_t nl) const { stage_image(dec_img, dec_bytes, l, nl); }

    // blanket push (src/ans.rs:96-105) with Categorical t's row (src/codec.rs:63-64)
    // kByte: u8 symbols, below 256 already (no clamp to the sentinel row: -1 VALU per push)
    template <class E, bool kByte = false>
    __device__ __forceinline__ void push(E& e, uint32_t sym, uint32_t, uint32_t tid) const {
        const uint32_t i = __umul24(tid, 257u) + (kByte ? sym : min(sym, 256u));  // row 257 t + s
        const uint4 r = lds_ld128(kTabE + shl16<4>(i));          // {p, cdf, w}
        uint32_t ra, na;
        asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(ra) : "v"(i), "s"(ro));
        asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(na) : "v"(tid), "s"(no));
        const double rcp = __longlong_as_double(static_cast<long long>(lds_ld64(kTabE + ra)));
        const uint64_t nw = lds_ld64(kTabE + na);  // {norm, -0x43300000 norm}
        const uint32_t mass = r.x, cum = r.y, norm = lo32(nw);
        const uint64_t w = mk64(r.w, r.z);
        uint32_t k8 = (r.z & 0xFFu) + (mk64(hi32(e.head), lo32(e.head) | 0xFFu) > w ? 8u : 0u);
        if constexpr (kRare) {
            const uint32_t screen = lds_ld32(kTabE + so + 4 * i);
            if (__builtin_expect(__builtin_amdgcn_ballot_w64(hi32(e.head) <= screen) != 0, 0)) {
                if (hi32(e.head) <= screen) {  // exact renorm(pK): take back, then count (src/ans.rs:233-253)
                    const uint64_t pK = static_cast<uint64_t>(mass) * lds_ld64(kTabE + k_off + 8 * tid);
                    e.take_back_until(pK);
                    k8 = bytes_out8_exact(e.head, pK);
                }
            }
        }
        e.emit4(k8);
        // q = head / p, r = head % p (src/ans.rs:101-102): round(head/p - 1/2), exact unless head/p
        // lies within 2^-4 of an integer; such lanes (and zero-mass rows, rcp 0) take the voted
        // 64-bit remainder (ans_fast.hpp k_encode push_one)
        // (kNormSmall: on x' = (H - qh p) 2^32 + lo after the exact high step, ans_fast.hpp div_hi;
        // kNormBig: rows of mass above 2^31 always take the exact branch, ans_fast.hpp k_encode)
        uint32_t qh = 0;
        uint64_t qb;
        if constexpr (kNR == fast::kNormSmall) {
            double hd;
            asm("v_cvt_f64_u32 %0, %1" : "=v"(hd) : "v"(hi32(e.head)));
            qh = fast::div_hi(hd, rcp, -static_cast<double>(mass));
            const double xd = __builtin_fma(hd, 4294967296.0, static_cast<double>(lo32(e.head)));
            double t;
            asm("v_fma_f64 %0, %1, %2, %3" : "=v"(t) : "v"(xd), "v"(rcp), "v"(4503599627370495.5));
            qb = static_cast<uint64_t>(__double_as_longlong(t));
        } else {
            qb = fast::qest_half(e.head, rcp);
        }
        uint32_t rm = lo32(e.head) - lo32(qb) * mass;
        const bool fix = kNR == fast::kNormBig ? (rm >= mass || static_cast<int32_t>(mass) < 0) : rm >= mass;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(fix) != 0, 0)) {
            if (fix) {
                if (mass == 0) e.err |= kErrZeroMass;
                const uint64_t x = kNR == fast::kNormSmall ? mk64(hi32(e.head) - qh * mass, lo32(e.head)) : e.head;
                const int64_t r = static_cast<int64_t>(x - (qb - 0x4330000000000000ull) * mass);
                const int64_t d = r < 0 ? -1 : (kNR != fast::kNormBig || r >= static_cast<int64_t>(mass) ? 1 : 0);
                qb += static_cast<uint64_t>(d);
                rm = static_cast<uint32_t>(r - d * static_cast<int64_t>(mass));
            }
        }
        // head = norm * q + cdf(x, r) (src/ans.rs:103-104): q < 2^52, hi32(q) = the raw high word's
        // low 20 bits (+ qh); outside kNormSmall the high word is one v_mul_lo_u32 of the raw word
        // and a v_add3 with the table's -0x43300000 norm (r05: the mask and a 64-bit product took
        // four VALU with their register moves)
        const uint64_t lo64 = static_cast<uint64_t>(lo32(qb)) * norm + (cum + rm);
        if constexpr (kNR == fast::kNormSmall) {
            e.head = mk64(hi32(lo64) + ((hi32(qb) & 0xFFFFFu) + qh) * norm, lo32(lo64));
        } else {
            uint32_t h;
            asm("v_add3_u32 %0, %1, %2, %3" : "=v"(h) : "v"(hi32(qb) * norm), "v"(hi32(lo64)), "v"(hi32(nw)));
            e.head = mk64(h, lo32(lo64));
        }
    }
    // a zero-mass lane: an out-of-range symbol (src/codec.rs:63) or p == 0 (src/ans.rs:98)
    template <typename Sym>
    __device__ uint32_t classify(const Sym* s, const uint8_t* t, uint64_t len, uint32_t err) const {
        for (uint64_t k = 0; k < len; ++k)
            if (static_cast<uint32_t>(s[k]) >= nsym[t[k]]) return err | kErrSymbol;
        return err;
    }

    __device__ __forceinline__ uint64_t first_bound(const uint8_t* t) const {
        return lds_ld64(kTab + kIndLOff + 8 * t[0]);
    }
    __device__ __forceinline__ void dec_init(DecState&) const {}
    __device__ __forceinline__ bool dec_bad(const DecState&) const { return false; }
    // blanket pop (src/ans.rs:107-116) with Categorical t's icdf (src/codec.rs:65-68)
    template <class Ch>
    __device__ __forceinline__ uint32_t pop(Ch& ch, DecState&, uint32_t tid, uint32_t& hi) const {
        // (a volatile fence on the table id: the header reads of a unit's pops are not hoisted
        // ahead of the pops before them, which held every header in registers at once)
        asm volatile("" : "+v"(tid));
        const uint4 h = lds_ld128(kTab + shl16<4>(tid));
        const double rcp_norm = __longlong_as_double(static_cast<long long>(mk64(h.y, h.x)));
        const uint32_t norm = h.z, hw = h.w;  // hw: us | bkt / 8 << 5 | 257 t << 19
        const auto L = [&]() __attribute__((always_inline)) { return lds_ld64(kTab + kIndLOff + 8 * tid); };
        // the chain from the renorm to the bucket read at raised wave priority, as in the C3
        // decoder (ans_fast.hpp k_decode): decode -1.3% (profiles/r04h_ab_rejected.txt; a second
        // bracket around the row read gained nothing)
        __builtin_amdgcn_s_setprio(2);
        ch.form_window();
        ch.P8 -= ch.template renorm_up8<!kLean>(L, kScreenAll);
        ch.read_window();  // for the next pop
        __builtin_amdgcn_sched_barrier(0);
        uint64_t qq;
        uint32_t cf;
        if constexpr (kNR == fast::kNormStd && kLean) {
            // r05: q rounded to nearest in the 2^49 binade (the header holds 1/(8 norm), an exact
            // scaling): t = fma(x, 1/(8 norm), 2^49 - 1/16) has raw bits 0x43000000'00000000 +
            // round(x / norm - 1/2 + e), |e| < 2^-52 x / norm + 2^-48, which is q unless x / norm
            // lies within |e| of an integer (kLean sets have every norm >= 2^20: x / norm < 2^44,
            // |e| < 2^-8); cf = lo32(x) - lo32(q') norm is then outside [0, norm) and a voted branch
            // moves q' by one.  The raw high word's low 24 bits are hi32(q), all the kLean update
            // reads.  Replaces the estimate from below and its select-based fix-up (five VALU per
            // pop) by one compare.
            double hd;
            asm("v_cvt_f64_u32 %0, %1" : "=v"(hd) : "v"(hi32(ch.head)));
            const double xd = __builtin_fma(hd, 4294967296.0, static_cast<double>(lo32(ch.head)));
            double t;
            asm("v_fma_f64 %0, %1, %2, %3" : "=v"(t) : "v"(xd), "v"(rcp_norm), "v"(562949953421311.9375));
            qq = static_cast<uint64_t>(__double_as_longlong(t));
            cf = lo32(ch.head) - lo32(qq) * norm;
            if (__builtin_expect(__builtin_amdgcn_ballot_w64(cf >= norm) != 0, 0)) {
                if (cf >= norm) {  // q' = q +- 1: the remainder's sign in 64 bits (|r| < 2 norm)
                    const int64_t r = static_cast<int64_t>(ch.head - (qq - 0x4300000000000000ull) * norm);
                    const int64_t d = r < 0 ? -1 : 1;
                    qq += static_cast<uint64_t>(d);
                    cf = static_cast<uint32_t>(r - d * static_cast<int64_t>(norm));
                }
            }
        } else {
            fast::div_norm<kNR>(ch.head, norm, rcp_norm, qq, cf, -static_cast<double>(norm));
        }
        // the bucket at kTab + ((cf >> us) + bkt / 8) * 8 (v_lshrrev takes us from the word's low
        // five bits; v_bfe the offset; one v_add_lshl)
        uint32_t ba;
        asm("v_add_lshl_u32 %0, %1, %2, 3" : "=v"(ba) : "v"(cf >> hw), "v"(__builtin_amdgcn_ubfe(hw, kIndBktShift, kIndRowShift - kIndBktShift)));
        const uint64_t cc = lds_ld64(kTab + ba);
        __builtin_amdgcn_s_setprio(0);
        // rx = cf << (32 - us) as ({cf, 0} >> us): v_alignbit takes us from the header word's low
        // five bits as they are (no unpacking of 32 - us)
        const uint32_t rx = __builtin_amdgcn_alignbit(cf, 0u, hw);
        uint32_t sx;
        asm volatile(
            "v_cmp_gt_u32 vcc, %[rx], %[w1]\n\t"
            "s_nop 1\n\t"
            "v_addc_co_u32 %[sx], vcc, 0, %[w1], vcc\n\t"
            "v_cmp_gt_u32 vcc, %[rx], %[w2]\n\t"
            "s_nop 1\n\t"
            "v_addc_co_u32 %[sx], vcc, 0, %[sx], vcc"
            : [sx] "=&v"(sx)
            : [rx] "v"(rx), [w1] "v"(lo32(cc)), [w2] "v"(hi32(cc))
            : "vcc");
        sx &= 0x1FFu;  // the symbol (w1's threshold bits above it dropped)
        const uint32_t r257 = hw >> kIndRowShift;  // 257 t: the table's first row
        uint32_t ra;
        asm("v_add_lshl_u32 %0, %1, %2, 3" : "=v"(ra) : "v"(sx), "v"(r257));
        const uint64_t row = lds_ld64(kTab + kIndRowOff + ra);  // (cdf(s), pmf(s))
        uint32_t p = hi32(row), r = cf - lo32(row);
        // a bucket with three or more boundaries can leave cf past s0 + 2's interval: r >= pmf(s)
        // is exactly that case (the thresholds never overshoot: cf >= cdf(sx)), one compare on the
        // row the pop reads anyway (r05; the bucket's far bit and its test took five VALU), then a
        // voted scan of the rows
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(r >= p) != 0, 0)) {
            if (r >= p) {
                while (cf >= lo32(lds_ld64(kTab + kIndRowOff + 8 * (r257 + sx + 1)))) ++sx;
                const uint64_t rw = lds_ld64(kTab + kIndRowOff + 8 * (r257 + sx));
                p = hi32(rw);
                r = cf - lo32(rw);
            }
        }
        // head = pmf(s) q + cf - cdf(s) (src/ans.rs:113-114)
        if constexpr (kLean) {
            const uint64_t lo = static_cast<uint64_t>(lo32(qq)) * p + r;
            uint32_t h;
            asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(h) : "v"(hi32(qq)), "v"(p), "v"(hi32(lo)));
            ch.head = mk64(h, lo32(lo));
        } else {
            ch.head = qq * p + r;
        }
        hi = 0;
        return sx;
    }
};

// ====================================================================== IID<Uniform(size)>
// size <= MAX_SIZE = 2^46 (src/codec.rs:13-49): pmf 1, cdf(x, 0) = x.  A push is renorm(K) and
// head = size * head + x (no division); one codec, so every push starts in [L, 2^8 L) and the
// renorm is ans_renorm.hpp's one-compare word (up to 7 bytes).  A pop is renorm(L) (two rounds
// of up to four bytes when size > 2^24) and (q, x) = head divmod size: a shift for powers of
// two, else the high word of head * floor((2^64 - 1) / size) and one fix-up.
template <bool kPow2>
struct UniformModel {
    static constexpr bool kTids = false;
    static constexpr bool kPairIds = false;
    static constexpr uint32_t kTab = kDecTab;
    static constexpr uint32_t kTabE = kEncTab;
    using DecState = NoState;
    uint64_t size, K, L, w, magic;
    uint32_t log2size, hL8;

    __device__ __forceinline__ void stage_enc(unsigned char*, uint32_t) const {}
    __device__ __forceinline__ void stage_dec(unsigned char*, uint32_t) const {}
    template <class E, bool kByte = false>
    __device__ __forceinline__ void push(E& e, uint32_t lo, uint32_t hi, uint32_t) const {
        const uint64_t x = mk64(hi, lo);
        if (x >= size) e.err |= kErrSymbol;  // outside the alphabet (the reference would code garbage)
        const uint32_t k8 = (lo32(w) & 0xFFu) + (mk64(hi32(e.head), lo32(e.head) | 0xFFu) > w ? 8u : 0u);
        e.emit(k8);
        e.head = kPow2 ? ((e.head << log2size) | x) : size * e.head + x;
    }
    template <typename Sym>
    __device__ uint32_t classify(const Sym*, const uint8_t*, uint64_t, uint32_t err) const { return err; }
    __device__ __forceinline__ uint64_t first_bound(const uint8_t*) const { return L; }
    __device__ __forceinline__ void dec_init(DecState&) const {}
    __device__ __forceinline__ bool dec_bad(const DecState&) const { return false; }
    template <class Ch>
    __device__ __forceinline__ uint32_t pop(Ch& ch, DecState&, uint32_t, uint32_t& hi) const {
        ch.renorm_wide(L, hL8);
        __builtin_amdgcn_sched_barrier(0);
        uint64_t x;
        if constexpr (kPow2) {
            x = ch.head & (size - 1);
            ch.head >>= log2size;
        } else {
            ch.head = div_magic(ch.head, size, magic, x);
        }
        hi = hi32(x);
        return lo32(x);
    }
};

// ====================================================================== IID<LogUniform(E)>
// (src/codec.rs:561-611) Per element x: bits = 64 - clz(x) (0 for x = 0), a Uniform(2^(bits-1))
// push of x's bits below the top one (K = 2^(57 - bits): renorm by bit lengths, the head shifted
// up by bits - 1), then a Uniform(E + 1) push of bits (at most one byte out: its K >= 2^49.9).
// Only bits = 1 can take a byte back (Uniform(1): bound 2^56); only the bits pop can hand one
// back (MChain::renorm_up8).  The pop is the mirror: renorm(L_E) in up to two rounds,
// (head, bits) = head divmod (E + 1) by the magic reciprocal, then renorm(2^56) and the low bits.
struct LogUniformState {
    bool bad;
};
struct LogUniformModel {
    static constexpr bool kTids = false;
    static constexpr bool kPairIds = false;
    static constexpr uint32_t kTab = kDecTab;
    static constexpr uint32_t kTabE = kEncTab;
    using DecState = LogUniformState;
    uint64_t nb, KE, LE, TEm1, magic;  // TEm1 = 2^8 KE - 1 (~0 when E = 0: no byte ever)
    uint32_t hL8E;

    __device__ __forceinline__ void stage_enc(unsigned char*, uint32_t) const {}
    __device__ __forceinline__ void stage_dec(unsigned char*, uint32_t) const {}
    template <class E, bool kByte = false>
    __device__ __forceinline__ void push(E& e, uint32_t lo, uint32_t hi, uint32_t) const {
        const uint64_t x = mk64(hi, lo);
        const uint32_t bits = x ? 64u - static_cast<uint32_t>(__builtin_clzll(x)) : 0u;  // LogUniform::get_bits
        if (bits >= nb) e.err |= kErrSymbol;                                               // assert!(bits < size)
        else if (bits > 47) e.err |= kErrNormRange;  // Uniform::new(2^(bits-1)) > MAX_SIZE
        if (bits != 0) {
            // Uniform(2^(bits-1)) push of the low bits: renorm(2^s), s = 57 - bits
            if (__builtin_expect(__builtin_amdgcn_ballot_w64(bits == 1 && e.head < kMaxMinHead) != 0, 0)) {
                if (bits == 1) e.take_back_until(kMaxMinHead);
            }
            const uint32_t bl = 64u - static_cast<uint32_t>(__builtin_clzll(e.head));
            const int32_t t = static_cast<int32_t>(bl) - static_cast<int32_t>(58u - min(bits, 48u));
            e.emit(t > 0 ? 8u * (static_cast<uint32_t>(t) >> 3) : 0u);
            const uint32_t sh = min(bits, 48u) - 1u;
            e.head = (e.head << sh) | (x & ((1ull << sh) - 1ull));
        }
        // Uniform(E + 1) push of bits: one byte out iff head >= 2^8 KE
        e.emit4(e.head > TEm1 ? 8u : 0u);
        e.head = e.head * nb + bits;
    }
    template <typename Sym>
    __device__ uint32_t classify(const Sym*, const uint8_t*, uint64_t, uint32_t err) const { return err; }
    __device__ __forceinline__ uint64_t first_bound(const uint8_t*) const { return LE; }
    __device__ __forceinline__ void dec_init(DecState& s) const { s.bad = false; }
    __device__ __forceinline__ bool dec_bad(const DecState& s) const { return s.bad; }
    template <class Ch>
    __device__ __forceinline__ uint32_t pop(Ch& ch, DecState& st, uint32_t, uint32_t& hi) const {
        ch.renorm_wide(LE, hL8E);
        __builtin_amdgcn_sched_barrier(0);
        uint64_t bits64;
        ch.head = div_magic(ch.head, nb, magic, bits64);
        const uint32_t bits = lo32(bits64);
        uint64_t x = 0;
        if (bits != 0) {
            st.bad |= bits > 47;  // no valid stream holds such a count (the encoder refuses it)
            ch.form_window();
            ch.P8 -= ch.renorm_up8(kMaxMinHead, 0xFFFFFFFFu);  // renorm(2^(bits-1) * 2^(57-bits)) = 2^56
            ch.read_window();
            const uint32_t sh = min(bits, 48u) - 1u;
            x = (ch.head & ((1ull << sh) - 1ull)) | (1ull << sh);
            ch.head >>= sh;
        }
        hi = hi32(x);
        return lo32(x);
    }
};

}  // namespace mfast
}  // namespace shuffle_coding
