// ans_fast.hpp — the throughput kernels of the bulk path (included by ans_kernels.hip).
//
// One lane = one chunk = one reference Message (src/ans.rs:292 zeros, src/codec.rs:415-424 IID,
// src/ans.rs:96-116 push/pop, src/ans.rs:255-264 flatten/unflatten).  The bytes are identical
// to the generic kernels' and to the oracle's; what changes is how the work maps to gfx950
// (DESIGN.md §3 has the measurements behind each choice):
//
//  * Global memory is touched only at wave-uniform "points", one per 16-byte unit of symbols.
//    Each point starts with `s_waitcnt vmcnt(0)`, so it waits only for what earlier points
//    issued.  Every global transfer is 64 contiguous bytes per lane (symbols in groups of
//    four units, compressed streams in 64-byte pages): gfx950 HBM writes at 64-byte
//    granularity, and 16-byte per-lane stores cost 4x their bytes in HBM traffic.
//  * Each lane stages its stream in a 128-byte LDS ring (two pages) with ALIGNED dword
//    accesses only (unaligned LDS writes are ~7x slower: tools/lds_probe.hip).  The ring is
//    laid out [dword][lane], so any lane-varying index is bank-conflict free and a page is
//    16 accesses at immediate offsets from one address.
//  * Bytes move between the 64-bit head and the stream through v_alignbyte funnels.
//  * q = head / p uses an f64 estimate and one integer fix-up, exact for
//    2^16 <= norm <= 2^31.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "ans_renorm.hpp"
#include "ans_table.hpp"

namespace shuffle_coding {
namespace fast {

constexpr int kBlock = 512;      // 8 waves; 2 workgroups (16 waves) per CU
constexpr int kRingDwords = 32;  // 128-byte ring per lane = 2 pages of 64 bytes
constexpr int kGroupBytes = 64;  // symbols move in 64-byte groups (4 units)
// encode LDS rows: rcp[257], (mass, cum)[257] and the first renorm threshold
// thr[257] = p*K*2^8 - 1 (saturated at 2^64 - 1); the others follow from it (k_encode)
// LDS-row encoder tables at offset 0, three 8-B arrays indexed by 8 s: rcp at 0, {mass, cum} at
// kEncRowOffset, the renorm word at kEncThrOffset (one address per symbol for all three reads)
constexpr uint32_t kEncRowOffset = (8 * 257 + 15) & ~15u;
constexpr uint32_t kEncThrOffset = kEncRowOffset + ((8 * 257 + 15) & ~15u);
constexpr uint32_t kEncLdsBytes = kEncThrOffset + 8 * 257;
constexpr uint32_t kEncRingBytes = kRingDwords * kBlock * 4;  // 64 KiB
// encode LDS: the row tables at offset 0 (a row address is the symbol times 8, each array at an
// immediate offset), the ring after them at a multiple of 256 B (the ds_write2st64 offset unit),
// so its row addresses stay one v_and_or with the ring base in the instructions' offset field
constexpr uint32_t kEncRingBase = (kEncLdsBytes + 255) & ~255u;
constexpr uint32_t kEncSharedBytes = kEncRingBase + kEncRingBytes;
static_assert(2 * kEncSharedBytes <= 160 * 1024, "two encode workgroups per CU");
constexpr uint32_t kDecTableBytes = 28672;  // decode buckets + cdf in LDS beside the 132 KiB ring (k_decode)
// fixed decode table layout (LDS offset 0, and the same in global memory): kDecNbMax buckets as
// two arrays of 8-B halves (cdf(s0), cdf(s0+1) | cdf(s0+2), cdf(s0+3)),
// their s0 bytes at kDecS0Off (a compile-time ds offset from the bucket index), the cdf table
// (nsym + 5 <= 261 words) at kDecCumOff
constexpr uint32_t kDecNbMax = (kDecTableBytes - 4 * 261 - 16) / 17;
constexpr uint32_t kDecS0Off = 16 * kDecNbMax;
constexpr uint32_t kDecCumOff = (kDecS0Off + kDecNbMax + 15) & ~15u;
static_assert(kDecCumOff + 4 * 261 <= kDecTableBytes, "decode tables fit");
// the no-far decoder's LDS layout (staged from the same global image): the two inner
// boundaries (cdf(s0+1), cdf(s0+2)) of each bucket as one 8-B array, the s0 bytes, then one
// 8-B row (cdf(s), pmf(s)) per symbol.  (16-B entries holding s0 too, addressed by one shift
// and mask, measured 2.6% slower: their 8-B reads use half the LDS banks.)
constexpr uint32_t kDecS0OffR = 8 * kDecNbMax;
constexpr uint32_t kDecRowOff = (kDecS0OffR + kDecNbMax + 15) & ~15u;
static_assert(kDecRowOff + 8 * 257 <= kDecTableBytes, "row decode tables fit");
// the fix-up-free decoder's LDS layout (k_decode kMode = kModeU, FastTable::dec_u): the quotient
// from below (q_m in {q - 1, q}) leaves u = head - q_m * norm in [0, 2 norm), which indexes a
// virtual alphabet of 512 symbols: v < 256 is symbol v at cdf(v) (q = q_m), v >= 256 symbol
// v - 256 at norm + cdf(v - 256) (q = q_m + 1).  Buckets of u (width 2^us) as 8-B threshold
// pairs, then 512 rows (cum_row, p) with head = p * q_m + (u - cum_row).  A bucket at a = j << us
// holds, for its boundaries c = cdfv(s0+1) and cdfv(s0+2) (s0 = the virtual symbol at a), the
// word (j & 1) << 31 | ((min(c - a, 2^us) - 1) << (31 - us)) | s0: u's offset in the bucket
// shifted up to bit 30 under the bucket index's low bit; rx = u << (31 - us) (mod 2^32) holds the
// same bit 31 and exceeds the word exactly when u >= c (its low bits are zero, the word's are
// s0).  The two differ by less than 2^31, so [rx > w] is the sign bit of w - rx, and
// s = w1 + ((w1 - rx) >> 31) + ((w2 - rx) >> 31) in its low bits: two v_sub, two v_lshrrev and
// a v_add3 (r06, 14.2 issue cycles; two v_cmp / v_addc pairs took 19.1 with their vcc hazards),
// on w1 itself, with no separate s0 array (one random LDS read fewer per symbol).  The bits of
// w1 above s0 start at bit 31 - us >= 13 and leave the row address ((s << 3) mod 2^16) alone:
// us <= 18 (norm up to 3,072 * 2^17 = 402,653,184; wider tables keep the row decoder).
constexpr uint32_t kDecUNbMax = (kDecTableBytes - 8 * 512) / 8;
constexpr uint32_t kDecURowOff = 8 * kDecUNbMax;
constexpr uint32_t kDecUShiftMax = 18;
static_assert(kDecURowOff + 8 * 512 <= kDecTableBytes, "u-domain decode tables fit");
static_assert(kDecURowOff <= 65535, "ds offsets");
// decode lookup modes (k_decode kMode)
constexpr int kModeFar = 0;   // 16-B buckets, three candidates, voted scan of the staged cdf
constexpr int kModeRows = 1;  // 8-B buckets, two boundaries, then the symbol's (cdf, pmf) row
constexpr int kModeU = 2;     // kModeRows over u in [0, 2 norm): no quotient fix-up
constexpr uint64_t kMaxMinHead = 1ull << 56;
// norm ranges of the LDS-table kernels (k_encode / k_decode kNR; FastTable::nr):
//  kNormStd    2^16 <= norm <= 2^31: head / d < 2^48, one f64 estimate within one of the quotient
//  kNormSmall  norm < 2^16 (the reference's count-built dataset tables, src/benchmark.rs:552-578):
//              head / d reaches 2^64 / norm, so the quotient is a long division in two f64
//              estimates: qh = floor(H / d) - 1 exactly (H = hi32(head), from a reciprocal rounded
//              UP, truncated), then the low part of x' = (H - qh d) 2^32 + lo32(head) < 2 d 2^32
//  kNormBig    2^31 < norm < 2^32: the estimate is accurate (head / d < 2^33) but 32-bit
//              remainders over [0, 2 norm) wrap, so the remainder is checked in 64 bits
constexpr int kNormStd = 0;
constexpr int kNormSmall = 1;
constexpr int kNormBig = 2;

// Non-temporal 16-byte global load / store (streamed data that must not evict cached tables).
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_load(const uint4* p) {
    const v4u32 v = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_store(uint4* p, const uint4& v) {
    __builtin_nontemporal_store(v4u32{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u32*>(p));
}

// s_waitcnt vmcnt(0) (gfx9 encoding; expcnt/lgkmcnt left at their maxima).
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// s_waitcnt vmcnt(N): all but the N youngest vector-memory operations done (in issue order)
template <int N>
__device__ __forceinline__ void wait_vm_n() {
    static_assert(N >= 0 && N < 64, "vmcnt field");
    __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}

// x << S in 16 bits (the upper half of the result is zero on gfx950): v_lshlrev_b16 issues in
// ~2.5 cycles per wave64 instruction where v_lshlrev_b32 and its SDWA forms take ~4.4
// (tools/b16_probe.hip), so LDS addresses below 2^16 are formed with it
template <int S>
__device__ __forceinline__ uint32_t shl16(uint32_t x) {
    static_assert(S >= 0 && S < 16, "16-bit shift");
    uint32_t r;
    asm("v_lshlrev_b16 %0, %1, %2" : "=v"(r) : "I"(S), "v"(x));
    return r;
}

// f(integral_constant<int, I>) for each I in order, every call inlined: a loop unrolled by
// construction, so register arrays indexed by I stay in registers
template <typename F, int... I>
__device__ __forceinline__ void unroll_seq(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}

__device__ __forceinline__ uint32_t ab(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}
__device__ __forceinline__ uint32_t lo32(uint64_t x) { return static_cast<uint32_t>(x); }
__device__ __forceinline__ uint32_t hi32(uint64_t x) { return static_cast<uint32_t>(x >> 32); }
__device__ __forceinline__ uint64_t mk64(uint32_t hi, uint32_t lo) { return (static_cast<uint64_t>(hi) << 32) | lo; }

// ~x / d (floor or floor+1) for x / d < 2^48, rcp = fl(1/d); see ans_kernels.hip quot_estimate.
__device__ __forceinline__ uint64_t qest(uint64_t x, double rcp) {
    // v_cvt_f64_u32 of the high dword through asm: from C++ the compiler sees (double)(x >> 32)
    // and emits its generic u64 -> f64 expansion (two extra f64 ops).
    double hd;
    asm("v_cvt_f64_u32 %0, %1" : "=v"(hd) : "v"(hi32(x)));
    const double xd = __builtin_fma(hd, 4294967296.0, static_cast<double>(lo32(x)));
    const double t = __builtin_fma(xd, rcp, 4503599627370496.0);
    return static_cast<uint64_t>(__double_as_longlong(t)) - 0x4330000000000000ull;
}

// qest - 1 (floor - 1 or floor) from the magic constant 2^52 - 1, for x / d >= 1: the sum lands
// at or above 2^52, where the ulp is 1, so it still rounds to an integer.
__device__ __forceinline__ uint64_t qest_m1(uint64_t x, double rcp) {
    double hd;
    asm("v_cvt_f64_u32 %0, %1" : "=v"(hd) : "v"(hi32(x)));
    const double xd = __builtin_fma(hd, 4294967296.0, static_cast<double>(lo32(x)));
    double t;  // v_fma_f64 (from C++ the compiler copies the magic into a v_fmac accumulator)
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(t) : "v"(xd), "v"(rcp), "v"(4503599627370495.0));
    return static_cast<uint64_t>(__double_as_longlong(t));  // raw bits: qest - 1 + 0x43300000'00000000
}

// round(x / d - 1/2) from the magic constant 2^52 - 1/2 (exact in f64), for x / d >= 1: the
// estimate's error is below 2^-52 x/d + 2^-48 (<= 2^-4 for x/d < 2^48), so this is floor(x / d)
// unless x / d lies within that error of an integer, and floor - 1 or floor + 1 there.  Raw bits:
// the estimate + 0x43300000'00000000.
__device__ __forceinline__ uint64_t qest_half(uint64_t x, double rcp) {
    double hd;
    asm("v_cvt_f64_u32 %0, %1" : "=v"(hd) : "v"(hi32(x)));
    const double xd = __builtin_fma(hd, 4294967296.0, static_cast<double>(lo32(x)));
    double t;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(t) : "v"(xd), "v"(rcp), "v"(4503599627370495.5));
    return static_cast<uint64_t>(__double_as_longlong(t));
}

// v_cvt_u32_f64: truncates toward zero, negatives saturate to 0 (a C++ cast of a negative
// double to an unsigned type is undefined)
__device__ __forceinline__ uint32_t cvt_u32(double x) {
    uint32_t r;
    asm("v_cvt_u32_f64 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// kNormSmall's first division step: with rcp_up >= 1/d rounded UP (by less than
// 2^-52 relative; the host's rcp_up) and d < 2^16, trunc(fma(H, rcp_up, -1)) = floor(H / d) - 1
// for every H < 2^32: the product overshoots H / d by less than 2^-19 < 1/d - the largest
// fraction below 1 that H / d can have, and Q - 1 is representable (rounding is monotone).
// Returns qh and replaces hd (= H as f64) by rh = H - qh d in [d, 2d), exactly.
__device__ __forceinline__ uint32_t div_hi(double& hd, double rcp_up, double neg_d) {
    const double qhf = __builtin_trunc(__builtin_fma(hd, rcp_up, -1.0));
    hd = __builtin_fma(qhf, neg_d, hd);
    return cvt_u32(qhf);
}

// TailGenerator::Random (src/ans.rs:129-164): rand_pcg 0.3.1 Pcg64Mcg (MCG-128, XSL-RR-64
// output) seeded by rand_core 0.6 seed_from_u64 (PCG32 expansion), one byte per draw
// (rand 0.8.5 Standard<u8> = next_u32() as u8 = next_u64() as u8).  The same restatement as
// the host's (ans_core.hpp TailGenerator), so GPU samples equal the host's; no reference test
// pins these bytes (parity unpinned).
struct Pcg64Mcg {
    uint64_t lo, hi;
    __device__ __forceinline__ void seed_from_u64(uint64_t st) {
        uint32_t w[4];
        for (int c = 0; c < 4; ++c) {
            st = st * 6364136223846793005ull + 11634580027462260723ull;
            const uint32_t xs = static_cast<uint32_t>(((st >> 18) ^ st) >> 27);
            const uint32_t rot = static_cast<uint32_t>(st >> 59);
            w[c] = (xs >> rot) | (xs << ((32 - rot) & 31));
        }
        lo = (static_cast<uint64_t>(w[1]) << 32 | w[0]) | 3;  // Mcg128Xsl64::new: state | 3
        hi = static_cast<uint64_t>(w[3]) << 32 | w[2];
    }
    __device__ __forceinline__ uint32_t next_byte() {
        constexpr uint64_t ML = 0x4385DF649FCCF645ull, MH = 0x2360ED051FC65DA4ull;
        const uint64_t nlo = lo * ML;
        hi = __umul64hi(lo, ML) + lo * MH + hi * ML;
        lo = nlo;
        const uint32_t rot = static_cast<uint32_t>(hi >> 58);
        const uint64_t xsl = hi ^ lo;
        return static_cast<uint32_t>((xsl >> rot) | (xsl << ((64 - rot) & 63))) & 0xFFu;
    }
};

// A chunk's initial message (include/ans_capi.h ans_*_ex): Message::zeros() / empty() (head
// 2^56, src/ans.rs:292-299) or Message::random(seed + c) (head 1 then renorm_up(MAX_MIN_HEAD)
// pulls seven generator bytes, src/ans.rs:285-290).  A push never pulls (head >= norm*K >= p*K),
// so a chunk's stream holds no generated byte and decoding ends back at this head.
struct ChunkInit {
    int kind;
    uint64_t seed;
    __device__ __forceinline__ uint64_t head(uint64_t c) const {
        if (kind != ANS_GEN_RANDOM) return 1ull << 56;
        Pcg64Mcg r;
        r.seed_from_u64(seed + c);
        uint64_t h = 1;
        while (h < (1ull << 56)) h = (h << 8) | r.next_byte();
        return h;
    }
};

// Lane-private ring of 32 dwords in a [dword][lane] image.
// LDS accesses by byte offset (address space 3): keeps the address arithmetic in 32 bits
// where the compiler otherwise adds the (zero) LDS base or splits constants out of offsets.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
__device__ __forceinline__ uint32_t lds_ld32(uint32_t off) { return *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(off)); }
__device__ __forceinline__ uint64_t lds_ld64(uint32_t off) { return *reinterpret_cast<const lds_u64*>(static_cast<uintptr_t>(off)); }
typedef __attribute__((address_space(3))) v4u32 lds_v4u32;
__device__ __forceinline__ uint4 lds_ld128(uint32_t off) {
    const v4u32 v = *reinterpret_cast<const lds_v4u32*>(static_cast<uintptr_t>(off));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// at kBase (kEncRingBase for the LDS-row encoder): a row address is one v_and_or of the row bits
// and the lane's column
template <uint32_t kBase>
struct RingT {
    uint32_t col;  // 4 * lane
    __device__ __forceinline__ lds_u32& at(int32_t i) const {
        const uint32_t a = ((static_cast<uint32_t>(i) << 11) & 0xF800u) | col;
        return *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(a + kBase));
    }
};
using Ring = RingT<kEncRingBase>;

// 8 * byte b of w in one SDWA shift (an LDS row offset straight from a u8 symbol; for byte 0
// the compiler emitted a shift and a mask).  b is a compile-time constant after unrolling.
__device__ __forceinline__ uint32_t byte_x8(uint32_t w, int b) {
    uint32_t r;
    const uint32_t three = 3;
    switch (b) {
    case 0: asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(three), "v"(w)); break;
    case 1: asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(three), "v"(w)); break;
    case 2: asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(three), "v"(w)); break;
    default: asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(three), "v"(w)); break;
    }
    return r;
}

template <typename Sym>
__device__ __forceinline__ uint32_t sym_of(const uint4& v, int j) {
    constexpr int per = 4 / static_cast<int>(sizeof(Sym));
    const int wi = j / per, sh = 8 * static_cast<int>(sizeof(Sym)) * (j % per);
    const uint32_t w = wi == 0 ? v.x : wi == 1 ? v.y : wi == 2 ? v.z : v.w;
    if constexpr (sizeof(Sym) == 4) return w;
    else return (w >> sh) & ((1u << (8 * sizeof(Sym))) - 1u);
}

template <typename Sym>
__device__ __forceinline__ void put_sym(uint4& v, int j, uint32_t s) {
    constexpr int per = 4 / static_cast<int>(sizeof(Sym));
    const int wi = j / per, sh = 8 * static_cast<int>(sizeof(Sym)) * (j % per);
    uint32_t& w = wi == 0 ? v.x : wi == 1 ? v.y : wi == 2 ? v.z : v.w;
    w = (j % per) == 0 ? s : (w | (s << sh));
}

// ====================================================================== encode
// Byte funnel.  pos8 = 8 * (stream bytes so far), neg8 = -pos8; the stream's dword w = pos/4
// lives in ring row w & 31, and X holds its contents with the b = pos & 3 written bytes at the
// bottom (garbage above).  A push of the head's low k bytes (lo, little-endian = stream order,
// src/ans.rs:246-253) forms both dwords it can touch, whatever k is:
//   dword w   = X's b bytes | lo << 8b           (v_bfe_u32 + v_lshl_or_b32)
//   dword w+1 = lo >> (32 - 8b)                  (v_lshrrev_b32; for b = 0 all of lo: unused bytes)
// and stores only dword w (one ds_write_b32).  Dword w+1, when the push reached it, becomes X:
// the next push (or finish) stores it with its own bytes, before any page holding it completes.
// Bytes past the new end are garbage that the next push overwrites.
template <uint32_t kBase>
struct FunnelT {
    uint32_t X, pos8, neg8, addr, col;  // addr = ring address of dword pos/4 (row | col)

    __device__ __forceinline__ void push(uint32_t lo, uint32_t k8) {
        uint32_t xv, d0, d1;
        asm("v_bfe_u32 %0, %1, 0, %2" : "=v"(xv) : "v"(X), "v"(pos8));
        asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(d0) : "v"(lo), "v"(pos8), "v"(xv));
        asm("v_lshrrev_b32 %0, %1, %2" : "=v"(d1) : "v"(neg8), "v"(lo));
        *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(addr + kBase)) = d0;
        pos8 += k8;
        neg8 -= k8;
        const uint32_t a = (shl16<6>(pos8) & 0xF800u) | col;  // (pos8 << 6) & 0xF800 needs 16 bits
        X = a != addr ? d1 : d0;
        addr = a;
    }
    __device__ __forceinline__ uint32_t len() const { return pos8 >> 3; }
    // the partial last dword, zero-padded, into its ring row (nothing is pushed after this)
    __device__ __forceinline__ void finish() {
        uint32_t xv;
        asm("v_bfe_u32 %0, %1, 0, %2" : "=v"(xv) : "v"(X), "v"(pos8));
        *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(addr + kBase)) = xv;
    }
};
using Funnel = FunnelT<kEncRingBase>;

// Completed ring pages leave in aligned pairs, one whole 128-B line per lane: the even page
// waits in registers for its odd partner.  A lone 64-B store leaves its line half-written in L2
// until the next page, and the streaming traffic around it evicts such lines in pieces (1.2x
// the stream's bytes written, profiles/r02c_pmc_c3_summary.txt; the 128-B symbol stores of
// k_decode write exactly theirs, profiles/r02d_pmc_c3_summary.txt).
template <uint32_t kBase>
struct PageOut {
    uint4 h0, h1, h2, h3;  // page 2m, until 2m+1 completes
    __device__ __forceinline__ void page(const RingT<kBase>& ring, uint32_t p, uint8_t* dst) {
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
        // held unconditionally (an odd page's copy is dead): as an else branch the compiler
        // merged these writes with the stores above into stores through a selected pointer,
        // which put the held page in scratch
        h0 = v0;
        h1 = v1;
        h2 = v2;
        h3 = v3;
    }
    // after the last page: np pages completed in all (an odd count leaves the last one held)
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

// KMAX: most bytes one push can emit (table property); kK32: K < 2^32 (norm > 2^24).
// kGlobalRows: the rows stay in global memory (alphabets above 256 symbols, e.g. C4's 65,536:
// 1 MiB of rows, L2-resident); each unit's rows are then requested at the point BEFORE the
// unit that uses them, so their latency hides behind one unit of work.
// LDS rows: one renorm test per push whatever KMAX is (enc_thr below).
// kVar (LDS rows only): chunk c holds vlen[c] <= chunk_len symbols at the start of its stride
// (staged ragged / variable-length chunks, ans_kernels.hip launch_staged_encode); the pushes
// past vlen[c], all in its first-coded group, are skipped.
// kNR: the norm range (kNormStd / kNormSmall / kNormBig above).  kNormSmall also runs with global
// rows (more than 256 symbols below 2^16: a count-built label table, src/benchmark.rs:576-578);
// kNormBig's large alphabets take k_encode_w (norm >= kWideNormMin).
// kM24 (LDS rows, kNormStd): every mass is below 2^24, so a row's mass word carries 8 k0 in its
// top byte and its renorm word is T - 1: head >= T is then head > T - 1 on the head's own
// register pair (r05; the (head | 0xFF) > T + 8 k0 form needed a v_or and a v_mov of the high
// word into the pair beside it, two VALU per push, for one v_and of the mass)
template <typename Sym, int KMAX, bool kK32, bool kGlobalRows, bool kVar = false, int kNR = kNormStd, bool kM24 = false>
__global__ __launch_bounds__(kBlock, kGlobalRows ? 2 : 4) void k_encode(FastTable t, const Sym* __restrict__ syms,
                                                                         uint64_t chunk_len, uint64_t nfull,
                                                                         uint8_t* __restrict__ slots, uint64_t slot_cap,
                                                                         uint32_t* __restrict__ lens,
                                                                         uint32_t* __restrict__ status, ChunkInit ini,
                                                                         const uint32_t* __restrict__ vlen = nullptr) {
    static_assert(!(kVar && kGlobalRows), "staged chunks take the LDS-row kernel");
    static_assert(kNR != kNormBig || !kGlobalRows, "2^31 < norm: the large-alphabet rows take k_encode_w");
    static_assert(!kM24 || (!kGlobalRows && kNR == kNormStd), "kM24: the LDS rows of the standard range");
    extern __shared__ __align__(16) unsigned char lds[];
    // a symbol's row is three random ds_read_b64 (32-lane groups over 32 bank pairs) from 8-B
    // arrays at one address, 8 s: rcp, {mass, cum} and the renorm word.  r06: against rcp by
    // ds_read_b64 and {mass, cum, renorm word} by one ds_read_b128 (16-lane groups over 16 bank
    // quads, ~7% fewer conflict cycles), one VALU less per push (the 16-B row's address), the
    // encoder being VALU-issue bound (0.92 of the issue slots, profiles/r06g_pmc_c3.json).
    // Tables at offset 0, ring after them (kEncRingBase)
    double* rcps = reinterpret_cast<double*>(lds);
    uint2* rows = reinterpret_cast<uint2*>(lds + kEncRowOffset);
    uint2* thrs = reinterpret_cast<uint2*>(lds + kEncThrOffset);
    // u8 symbols index the rows unclamped: all 256 byte values get a row (zero mass beyond the
    // alphabet, so they fail like the sentinel row they used to be clamped to)
    constexpr bool kByteRows = sizeof(Sym) == 1;
    if (!kGlobalRows) {
        const uint32_t nrows = kByteRows ? 256u : t.enc_rows;
        for (uint32_t i = threadIdx.x; i < nrows; i += kBlock) {
            const EncRow r = i < t.enc_rows ? t.enc[i] : EncRow{0.0, 0u, 0u};
            const uint64_t w = enc_thr(static_cast<uint64_t>(r.mass) * t.K, t.L);
            if constexpr (kM24) {  // {mass | 8 k0 << 24, cum}, T - 1 (T's low byte is zero)
                const uint64_t tm1 = (w & ~0xFFull) - 1u;
                rows[i] = make_uint2(r.mass | (lo32(w) << 24), r.cum);
                thrs[i] = make_uint2(lo32(tm1), hi32(tm1));
            } else {
                rows[i] = make_uint2(r.mass, r.cum);
                thrs[i] = make_uint2(lo32(w), hi32(w));
            }
            rcps[i] = r.rcp;  // 0 for zero mass: such a push always takes the voted branch
        }
    }
    // a row in registers: the table row plus its renorm word (enc_thr)
    struct Row {
        EncRow e;
        uint64_t thr;
    };
    auto row_at = [&](uint32_t off) __attribute__((always_inline)) {  // off = 8 * symbol (tables at LDS offset 0)
        const uint64_t v = lds_ld64(off + kEncRowOffset), w = lds_ld64(off + kEncThrOffset);
        Row r;
        r.e = EncRow{__longlong_as_double(static_cast<long long>(lds_ld64(off))), lo32(v), hi32(v)};
        r.thr = w;
        return r;
    };
    const Ring ring{4 * threadIdx.x};
    PageOut<kEncRingBase> pout;
    __syncthreads();
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (c >= nfull) return;

    constexpr int U = 16 / static_cast<int>(sizeof(Sym));
    const uint4* src = reinterpret_cast<const uint4*>(syms + c * chunk_len);
    uint8_t* dst = slots + c * slot_cap;
    const uint32_t npages_cap = static_cast<uint32_t>(slot_cap / 64);
    const uint64_t norm = t.norm;
    const uint64_t K = t.K;
    const uint32_t sentinel = t.enc_rows - 1;  // zero-mass row: out-of-range symbols land here
    const uint32_t exp_norm = 0x43300000u * static_cast<uint32_t>(t.norm);  // the estimate's exponent word x norm

    uint64_t head = ini.head(c);  // Message::zeros() / random(seed + c)
    Funnel f{0, 0, 0, ring.col, ring.col};
    uint32_t fp = 0, over = 0;
    uint32_t minmass = ~0u;  // 0 after a zero-mass / out-of-range symbol (push_one's voted branch)

    auto point = [&]() __attribute__((always_inline)) {
        wait_vm();
        if ((f.pos8 >> 9) > fp) {  // at most one page completes per unit (U * KMAX <= 64 bytes)
            if (fp < npages_cap) pout.page(ring, fp, dst);
            else over = 1;
            ++fp;
        }
    };
    auto bound = [&](const EncRow& e) __attribute__((always_inline)) {
        return kK32 ? static_cast<uint64_t>(e.mass) * static_cast<uint32_t>(K) : static_cast<uint64_t>(e.mass) * K;
    };
    // renorm(p*K) (src/ans.rs:100,246-253): k = #{j >= 1 : (head >> 8j) >= p*K} bytes out
    auto bytes_out = [&](uint64_t pK) __attribute__((always_inline)) {
        uint32_t k = (head >> 8) >= pK ? 1u : 0u;
        if constexpr (KMAX >= 2) k += (head >> 16) >= pK ? 1u : 0u;
        if constexpr (KMAX >= 3) k += (head >> 24) >= pK ? 1u : 0u;
        if constexpr (KMAX >= 4) k += (head >> 32) >= pK ? 1u : 0u;
        return k;
    };
    // 8k from the row's renorm word w = T + 8 k0 (enc_thr): k = k0 + [head >= T], and with T's
    // low byte zero, head >= T iff (head | 0xFF) > w
    auto bytes_out_w8 = [&](uint64_t w) __attribute__((always_inline)) {
        const bool up = mk64(hi32(head), lo32(head) | 0xFFu) > w;
        return (lo32(w) & 0xFFu) + (up ? 8u : 0u);
    };
    // kM24: w = T - 1 and 8 k0 in the mass word's top byte
    auto bytes_out_m24 = [&](uint64_t w, uint32_t mw) __attribute__((always_inline)) {
        return (mw >> 24) + (head > w ? 8u : 0u);
    };
    // a zero-mass row (rcp 0: q_est 0, so rm = lo32(head) >= 0 = p) always takes the voted
    // branch, which records it (the reference's assert_ne!(p, 0), src/ans.rs:98)
    auto push_one = [&](const EncRow& e, uint32_t k8) __attribute__((always_inline)) {
        f.push(lo32(head), k8);
        head >>= k8;
        // q = head / p, r = head % p (src/ans.rs:101-102), then head = norm * q + cdf(x, r)
        // (src/ans.rs:103-104, src/codec.rs:64).  The estimate round(head/p - 1/2) is q except
        // where head/p lies within 2^-4 of an integer (C3: head/p < 2^37, so within 2^-15, about
        // one symbol in 2^14): r = head - q_est*p in 32 bits is then < p exactly when q_est = q,
        // and the rare lanes where it is not take the exact 64-bit remainder on a voted branch
        // (q_est = q - 1 or q + 1).  The common path is one compare and one add, where the
        // estimate from below (q_m in {q - 1, q}) needed a borrow-select on every symbol.
        // kNormSmall: the same estimate on x' = (H - qh p) 2^32 + lo32(head) in [p 2^32, 2p 2^32)
        // after the exact high step (div_hi; e.rcp is 1/p rounded up there), q = qh 2^32 + q_est
        uint32_t qh = 0;
        uint64_t qb;  // q_est + 0x43300000'00000000
        if constexpr (kNR == kNormSmall) {
            double hd;
            asm("v_cvt_f64_u32 %0, %1" : "=v"(hd) : "v"(hi32(head)));
            qh = div_hi(hd, e.rcp, -static_cast<double>(e.mass));
            const double xd = __builtin_fma(hd, 4294967296.0, static_cast<double>(lo32(head)));
            double t;
            asm("v_fma_f64 %0, %1, %2, %3" : "=v"(t) : "v"(xd), "v"(e.rcp), "v"(4503599627370495.5));
            qb = static_cast<uint64_t>(__double_as_longlong(t));
        } else {
            qb = qest_half(head, e.rcp);
        }
        uint32_t rm = lo32(head) - lo32(qb) * e.mass;
        // kNormBig: the 32-bit test cannot tell a remainder off by one estimate step from a true
        // one for masses above 2^31 (2^32 - p < p), so those rows always take the exact branch
        const bool fix = kNR == kNormBig ? (rm >= e.mass || static_cast<int32_t>(e.mass) < 0) : rm >= e.mass;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(fix) != 0, 0)) {
            if (fix) {
                minmass = min(minmass, e.mass);
                const uint64_t x = kNR == kNormSmall ? mk64(hi32(head) - qh * e.mass, lo32(head)) : head;
                const int64_t r = static_cast<int64_t>(x - (qb - 0x4330000000000000ull) * e.mass);
                // q_est is within one of q; off by one wherever the 32-bit test fired, except
                // on kNormBig's forced rows, which may be right already
                const int64_t d = r < 0 ? -1 : (kNR != kNormBig || r >= static_cast<int64_t>(e.mass) ? 1 : 0);
                qb += static_cast<uint64_t>(d);
                rm = static_cast<uint32_t>(r - d * static_cast<int64_t>(e.mass));
            }
        }
        const uint32_t a = e.cum + rm;
        // the high word as v_mul_lo_u32 + v_add3 on the raw exponent word (its 0x43300000 * norm
        // comes off as a scalar): a second v_mad_u64_u32 costs two v_mov and the exponent a v_add
        const uint64_t lo64 = static_cast<uint64_t>(lo32(qb)) * static_cast<uint32_t>(norm) + a;
        uint32_t hq;
        asm("v_mul_lo_u32 %0, %1, %2" : "=v"(hq) : "v"(hi32(qb) + qh), "s"(static_cast<uint32_t>(norm)));
        head = mk64(hi32(lo64) + hq - exp_norm, lo32(lo64));
    };
    const uint32_t nvalid = kVar ? vlen[c] : static_cast<uint32_t>(chunk_len);
    auto roff_rt = [&](const uint4& v, int j) __attribute__((always_inline)) {  // 8 * symbol j of a unit
        if constexpr (kByteRows) return byte_x8(j == 0 || j == 1 || j == 2 || j == 3 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w, j & 3);
        else return 8 * min(sym_of<Sym>(v, j), sentinel);
    };
    // rows are read TWO pushes ahead, across units (the next unit's first rows during this
    // unit's last pushes), where one ahead within a unit left the first row of each unit waiting
    // for its read: encode −0.7 to −0.8% in two same-box A/Bs (three ahead measured the same,
    // for 6 more VGPRs); the scheduling barriers keep the compiler from hoisting all the reads
    Row q1, q2;  // the rows of the next two pushes
    auto process = [&](const uint4& unit, const uint4& nextu, uint32_t upos) __attribute__((always_inline)) {
#pragma unroll
        for (int j = U - 1; j >= 0; --j) {  // IID::push: last symbol first (src/codec.rs:417)
            __builtin_amdgcn_sched_barrier(0);
            const Row e = q1;
            q1 = q2;
            q2 = row_at(j >= 2 ? roff_rt(unit, j - 2) : roff_rt(nextu, j - 2 + U));
            if (kVar && upos + j >= nvalid) continue;  // past the chunk (its first, partial group)
            // the push (the head chain) at raised wave priority, the row reads and page flushes
            // at the base one (encode -2.3% in a same-box A/B; the reads raised instead: +1.6%)
            __builtin_amdgcn_s_setprio(2);
            if constexpr (kM24) {
                const uint32_t k8 = bytes_out_m24(e.thr, e.e.mass);
                EncRow em = e.e;
                em.mass &= 0xFFFFFFu;
                push_one(em, k8);
            } else {
                push_one(e.e, bytes_out_w8(e.thr));
            }
            __builtin_amdgcn_s_setprio(0);
        }
    };
    auto request_rows = [&](const uint4& unit, EncRow* buf) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < U; ++j) buf[j] = t.enc[min(sym_of<Sym>(unit, j), sentinel)];
    };
    auto process_rows = [&](const EncRow* buf) __attribute__((always_inline)) {
#pragma unroll
        for (int j = U - 1; j >= 0; --j) push_one(buf[j], 8 * bytes_out(bound(buf[j])));
    };

    // (non-temporal symbol loads / page stores measured 28% SLOWER with rows in global memory)
    auto load_sym = [&](const uint4* p) __attribute__((always_inline)) { return *p; };
    if constexpr (kGlobalRows) {
        // groups are walked last to first; group g-1's 64 bytes are requested while g is coded
        const int ngroups = static_cast<int>(chunk_len * sizeof(Sym) / kGroupBytes);
        uint4 n0, n1, n2, n3;
        {
            const uint4* gsrc = src + 4 * (ngroups - 1);
            n0 = load_sym(gsrc + 0);
            n1 = load_sym(gsrc + 1);
            n2 = load_sym(gsrc + 2);
            n3 = load_sym(gsrc + 3);
        }
        EncRow ra[U], rb[U];
        wait_vm();
        request_rows(n3, ra);
        for (int g = ngroups - 1; g >= 0; --g) {
            point();
            const uint4 c0 = n0, c1 = n1, c2 = n2;
            if (g > 0) {  // (uniform) group 0 has no successor to fetch
                const uint4* gsrc = src + 4 * (g - 1);
                n0 = load_sym(gsrc + 0);
                n1 = load_sym(gsrc + 1);
                n2 = load_sym(gsrc + 2);
                n3 = load_sym(gsrc + 3);
            }
            request_rows(c2, rb);
            process_rows(ra);  // unit 3 of group g
            point();
            request_rows(c1, ra);
            process_rows(rb);
            point();
            request_rows(c0, rb);
            process_rows(ra);
            point();
            request_rows(n3, ra);  // unit 3 of group g-1 (landed at the previous point)
            process_rows(rb);
        }
    } else {
        // groups of 128 B (8 units: one whole L2 line per lane and fetch, profiles/r02_hbm_calib.txt)
        // walked last to first.  Group g-1 is requested once units 7..4 of group g are coded, so
        // at most 12 units of symbols are live (the pair of held pages needs those registers),
        // and stays in flight for four units; no explicit wait: the page stores need none (their
        // data leaves the registers at issue), and the compiler waits for the loads at first use.
        constexpr int GU = 8;
        constexpr int GS = 128 / static_cast<int>(sizeof(Sym));  // symbols per group
        const int ngroups = kVar ? static_cast<int>((nvalid + GS - 1) / GS) : static_cast<int>(chunk_len * sizeof(Sym) / 128);
        uint4 n[GU];
#pragma unroll
        for (int i = 0; i < GU; ++i) n[i] = make_uint4(0, 0, 0, 0);
        if (ngroups > 0) {  // (an empty staged chunk codes no symbol)
            const uint4* gsrc = src + GU * (ngroups - 1);
#pragma unroll
            for (int i = 0; i < GU; ++i) n[i] = load_sym(gsrc + i);
        }
        auto flush_ready = [&]() __attribute__((always_inline)) {
            if ((f.pos8 >> 9) > fp) {
                if (fp < npages_cap) pout.page(ring, fp, dst);
                else over = 1;
                ++fp;
            }
        };
        q1 = row_at(roff_rt(n[GU - 1], U - 1));  // the first unit's first two rows
        q2 = row_at(roff_rt(n[GU - 1], U - 2));
        for (int g = ngroups - 1; g >= 0; --g) {
            uint4 cc[GU];
#pragma unroll
            for (int i = 0; i < GU; ++i) cc[i] = n[i];
            // the eight units as eight inlined calls with compile-time indices (unroll_seq, as in
            // k_decode): a #pragma unroll was refused for the staged kmax-4 instantiations, which
            // then indexed cc[] in scratch (144 B per lane)
            auto unit = [&](auto ic) __attribute__((always_inline)) {
                constexpr int u = GU - 1 - decltype(ic)::value;  // last unit first
                flush_ready();
                if (u == GU / 2 - 1 && g > 0) {
                    const uint4* gsrc = src + GU * (g - 1);
#pragma unroll
                    for (int i = 0; i < GU; ++i) n[i] = load_sym(gsrc + i);
                }
                // the unit after this one: cc[u - 1], or the next group's last unit (its loads
                // were issued three units ago; on the last group, unused rows of valid symbols)
                process(cc[u], u > 0 ? cc[u > 0 ? u - 1 : 0] : n[GU - 1], static_cast<uint32_t>(g * GS + u * U));
            };
            unroll_seq(unit, std::make_integer_sequence<int, GU>{});
        }
    }
    point();  // the last unit's completed page: the flatten's 8 bytes may reach the ring slot it holds

    // flatten (src/ans.rs:255-260): all significant head bytes, low first (7 or 8 here,
    // since the head is >= norm*K > 2^55 after any push).
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
    lens[c] = (over || minmass == 0) ? 0u : len;  // no length past the slot reaches k_compact or a decoder
}

// ---- shared decode steps
// renorm_up (src/ans.rs:239-243) with W = the next four stream bytes (first byte on top):
// head = head << 8k | the top k bytes of W, for the least k that makes head >= L; returns k.
// With js = min(clz64(head) >> 3, 4), X = (h:W) >> (32 - 8js) is >= 2^56 >= L (or head itself
// when js = 0), and k = js - 1 suffices iff X >> 8 is >= L already.  The head is >= K >= 2^25
// after any pop in the fast range, so a zero high word means js = 4 (v_ffbh_u32(0) = ~0
// saturates through the min).  X comes from byte permutes, exact for every js in 0..4.
//
// X >> 8 >= L needs hi32(X >> 8) >= hi32(L), i.e. hi32(X) >= hL8 = hi32(L) << 8: the top
// 24 bits of X all but saturated (L > 2^56 - norm).  That is ~2^-24 per symbol, so the exact
// 64-bit test runs only when some lane of the wave passes the 32-bit screen (a uniform
// branch; the common path is js bytes with no select).  hL8 = ~0 when L = 2^56 (hi32(L) << 8
// would overflow, and X >> 8 < 2^56 = L never needs one byte less).
// kJ4 = false: no pop leaves the high word zero (kmax <= 3: p*K >= 2^32 for every symbol, and
// a pop leaves head >= p*q >= p*K), so js = clz >> 3 needs no clamp.
// Returns 8k.  The permute selector (7-js, 6-js, 5-js, 4-js) is the high word of the byte ramp
// 0x0706050403020100 shifted left by 8js: one 64-bit shift of the bit count 8js = clz & ~7,
// where the byte count took a shift, a broadcasting v_perm and a subtract.
// kScreen = false (k_decode's deferred screen): no test here; the caller takes max(hi32(head))
// over a unit and re-runs the unit exactly when it reached the screen.
template <bool kJ4 = true, bool kScreen = true>
__device__ __forceinline__ uint32_t renorm_up8(uint64_t& head, uint32_t W, uint64_t L, uint32_t hL8) {
    const uint32_t h1 = hi32(head), h0 = lo32(head);
    uint32_t fb;
    asm("v_ffbh_u32 %0, %1" : "=v"(fb) : "v"(h1));
    const uint32_t m = kJ4 ? min(fb, 32u) & 0x38u : fb & 0x18u;  // 8 js
    const uint32_t sel = hi32(0x0706050403020100ull << m);
    const uint32_t xj1 = __builtin_amdgcn_perm(h1, h0, sel), xj0 = __builtin_amdgcn_perm(h0, W, sel);
    head = mk64(xj1, xj0);
    uint32_t m8 = m;
    if (kScreen && __builtin_expect(__builtin_amdgcn_ballot_w64(xj1 >= hL8) != 0, 0)) {
        const uint32_t xm1 = xj1 >> 8, xm0 = ab(xj1, xj0, 1);
        if (m != 0 && mk64(xm1, xm0) >= L) {
            head = mk64(xm1, xm0);
            m8 = m - 8;
        }
    }
    return m8;
}
template <bool kJ4 = true>
__device__ __forceinline__ uint32_t renorm_up(uint64_t& head, uint32_t W, uint64_t L, uint32_t hL8) {
    return renorm_up8<kJ4>(head, W, L, hL8) >> 3;
}
__host__ __device__ inline uint32_t renorm_screen(uint64_t L) {
    const uint64_t h = (L >> 32) << 8;
    return h > 0xFFFFFFFFull ? 0xFFFFFFFFu : static_cast<uint32_t>(h);
}
// q = head / norm, cf = head % norm (src/ans.rs:110-111): estimate, then one fix-up
// The estimate's raw f64 bits are q' + 0x43300000'00000000; q = q' - [ii < 0] and the exponent
// come off in ONE 64-bit add of (m - 0x43300000 : m), m = ii >> 31 (0 or -1), where the compiler
// emitted the sign extension, the 64-bit add and a separate v_add for the exponent word.
// kNormSmall: rcp_norm is 1/norm rounded up; the estimate divides x' = (H - qh norm) 2^32 + lo
// after the exact high step (div_hi), and qh joins the high word of the same add.
// kNormBig: 2^31 < norm, so ii does not fit 32 signed bits: the estimate is rounded to nearest
// (within one of q: head / norm < 2^33), the remainder taken in 64 bits and, on the rare lanes
// outside [0, norm), fixed on a voted branch.
template <int kNR = kNormStd>
__device__ __forceinline__ void div_norm(uint64_t head, uint32_t norm, double rcp_norm, uint64_t& qq, uint32_t& cf,
                                         double neg_norm = 0.0) {
    double hd;
    asm("v_cvt_f64_u32 %0, %1" : "=v"(hd) : "v"(hi32(head)));
    uint32_t qh = 0;
    if constexpr (kNR == kNormSmall) qh = div_hi(hd, rcp_norm, neg_norm);
    const double xd = __builtin_fma(hd, 4294967296.0, static_cast<double>(lo32(head)));
    if constexpr (kNR == kNormBig) {
        const double t = __builtin_fma(xd, rcp_norm, 4503599627370495.5);
        const uint64_t raw = static_cast<uint64_t>(__double_as_longlong(t));
        qq = mk64(hi32(raw) & 0xFFFFFu, lo32(raw));  // q_est < 2^33
        uint64_t r = head - qq * norm;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(r >= norm) != 0, 0)) {
            if (r >= norm) {
                if (static_cast<int64_t>(r) < 0) {
                    qq -= 1;
                    r += norm;
                } else {
                    qq += 1;
                    r -= norm;
                }
            }
        }
        cf = lo32(r);
        return;
    }
    const double t = __builtin_fma(xd, rcp_norm, 4503599627370496.0);
    const uint64_t raw = static_cast<uint64_t>(__double_as_longlong(t));
    const int32_t ii = static_cast<int32_t>(lo32(head) - lo32(raw) * norm);
    const uint32_t m = static_cast<uint32_t>(ii >> 31);
    cf = static_cast<uint32_t>(ii) + (norm & m);
    const uint64_t adj = mk64(m + 0xBCD00000u + qh, m);  // -0x43300000'00000000 - [ii < 0] (+ qh 2^32)
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(qq) : "v"(raw), "v"(adj));
}

// Stream bytes below the stream start (sh > 0: another chunk's bytes in a dense container)
// read as zeros, the Zeros tail generator's bytes (src/ans.rs:160-170), exactly as below a
// slot; only a corrupt stream reaches them.  S: one 64-B page at stream position pos.
// (k_decode_g only: k_decode and k_decode_w count positions from the stream's first byte, so
// their pages never hold another stream's bytes.)
__device__ __forceinline__ uint32_t keep_from(uint32_t w, int32_t pos, int32_t sh) {
    const int32_t k = sh - pos;  // low bytes to clear
    return k <= 0 ? w : (k >= 4 ? 0u : w & (~0u << (8 * k)));
}
__device__ __forceinline__ uint4 keep4(const uint4& v, int32_t pos, int32_t sh) {
    return make_uint4(keep_from(v.x, pos, sh), keep_from(v.y, pos + 4, sh), keep_from(v.z, pos + 8, sh),
                      keep_from(v.w, pos + 12, sh));
}
// (by value: a pointer into a register array that differs between branches puts it in scratch)
__device__ __forceinline__ void clear_below(uint4& a0, uint4& a1, uint4& a2, uint4& a3, int32_t pos, int32_t sh) {
    if (__builtin_expect(pos < sh, 0)) {
        a0 = keep4(a0, pos, sh);
        a1 = keep4(a1, pos + 16, sh);
        a2 = keep4(a2, pos + 32, sh);
        a3 = keep4(a3, pos + 48, sh);
    }
}

// ====================================================================== decode
// One decode chain = one chunk, read from the end.  P is the stream position minus 4: the
// window W = stream bytes [P, P+4) (byte P+3 on top) comes from ring dwords y = P>>2 and y+1
// with one v_alignbyte.  The ring (after the tables, at kDecTableBytes) is [row][lane] with kDecRows = 33 rows:
// row 32 mirrors row 0, so y and y+1 are one ds_read2st64_b32 even across the wrap.  Pages
// (16 rows) land at points: page low+1 is free once dword y+1 lies in page low, and the page
// below `low` is always in flight in registers (S); pages below 0 are zeros (the Zeros
// generator, src/ans.rs:160-170).  A point covers at most 60 stream bytes (SPP symbols of at
// most KMAX bytes), so no read between points can reach an unlanded page.
// The decoder runs 1,024-lane workgroups, one per CU: the lanes share ONE copy of the tables,
// so the whole 160 KiB of LDS holds the 1,024 rings (132 KiB) plus 28 KiB of tables, twice the
// table room two 512-lane workgroups would leave (finer icdf buckets: C3 resolves every cf with
// three candidates and compiles no far path).
__device__ const uint4 kZeroPage[8] = {};  // 128 zero bytes: the Zeros tail generator's pages
constexpr int kDecBlock = 1024;
constexpr int kDecRows = 33;
constexpr uint32_t kDecRingBytes = kDecRows * kDecBlock * 4;
static_assert(kDecRingBytes + kDecTableBytes == 160 * 1024, "decode LDS = one CU's 160 KiB");
// decode LDS: the tables at offset 0 (bucket = cf bucket * 16, its s0 byte at the bucket index
// plus an immediate offset), the ring after them at kDecTableBytes (a multiple of 256 B, folded
// into the window read's ds_read2st64 offsets)
static_assert(kDecTableBytes % 256 == 0 && kDecTableBytes / 256 + 16 <= 255, "ring base in the st64 offsets");

struct DecChain {
    uint32_t* ring;  // &ring[0][lane]
    const uint8_t* src;
    uint4 Q[8];  // the aligned page pair (2m, 2m+1) not yet landed: one 128-B L2 line per fetch
    int32_t low, P8, sh;  // P8 = 8 P (P: the window's stream position); sh = 0 (stream-relative)
    uint32_t W;
    uint64_t head;
    // per-step values between the phases
    uint64_t qq;
    uint32_t cf, cum, nxt, sx;
    bool far;

    __device__ __forceinline__ uint32_t& row(int32_t r) const { return ring[r * kDecBlock]; }
    // page p (its half of Q) into ring slot p & 1
    // (positions count from the stream's start, so no landed page holds another stream's
    // bytes: pages below the start are the zero page; nothing to clear)
    // The sixteen rows go out as eight ds_write2st64_b32 from one base address (ring row r0):
    // rows 4 KiB apart are 16 st64 units, so rows r0..r0+15 fit the 8-bit offset fields.  As C++
    // stores the compiler formed each row's address with its own v_add (the rows lie beyond
    // the 16-bit byte offsets) and stored them one dword at a time.
    template <int R0>
    __device__ __forceinline__ uint32_t put_half(uint4 a0, uint4 a1, uint4 a2, uint4 a3) {
        const uint32_t base = col + kDecTableBytes + R0 * kDecBlock * 4;
        asm volatile(
            "ds_write2st64_b32 %0, %1, %2 offset0:0 offset1:16\n\t"
            "ds_write2st64_b32 %0, %3, %4 offset0:32 offset1:48\n\t"
            "ds_write2st64_b32 %0, %5, %6 offset0:64 offset1:80\n\t"
            "ds_write2st64_b32 %0, %7, %8 offset0:96 offset1:112\n\t"
            "ds_write2st64_b32 %0, %9, %10 offset0:128 offset1:144\n\t"
            "ds_write2st64_b32 %0, %11, %12 offset0:160 offset1:176\n\t"
            "ds_write2st64_b32 %0, %13, %14 offset0:192 offset1:208\n\t"
            "ds_write2st64_b32 %0, %15, %16 offset0:224 offset1:240"
            :
            : "v"(base), "v"(a0.x), "v"(a0.y), "v"(a0.z), "v"(a0.w), "v"(a1.x), "v"(a1.y), "v"(a1.z), "v"(a1.w),
              "v"(a2.x), "v"(a2.y), "v"(a2.z), "v"(a2.w), "v"(a3.x), "v"(a3.y), "v"(a3.z), "v"(a3.w)
            : "memory");
        return a0.x;
    }
    // two exec-masked store sets, one per parity: as one store set from selected registers the
    // compiler spent 16 v_cndmask per landing (the barrier keeps it from merging them again)
    __device__ __forceinline__ void put_page(int32_t p) {
        if (p & 1) {
            put_half<16>(Q[4], Q[5], Q[6], Q[7]);
        } else {
            row(32) = put_half<0>(Q[0], Q[1], Q[2], Q[3]);  // row 32 mirrors row 0
        }
    }
    // pages are fetched as aligned 128-B pairs (2m, 2m+1): a 64-B read leaves the other half of
    // its 128-B line to be fetched again later (profiles/r02_hbm_calib.txt: 2x the bytes).
    // Pairs below 0 come from a zero pair in global memory: the same loads, where a register
    // zero-fill cost a point's worth of v_mov on every wave with one lane at its stream start
    // (global address space: a flat load would also count in lgkmcnt and stall the LDS waits)
    // Positions count from the stream's first byte (src), at any alignment: a pair below the
    // top one lies wholly inside the stream, so its 16-B loads (unaligned in a dense container;
    // the hardware runs in unaligned mode) touch only the stream's own bytes.
    __device__ __forceinline__ void fetch_pair(int32_t m) {
        typedef __attribute__((address_space(1), aligned(1))) const v4u32 gv4;
        const uint4* g = m >= 0 ? reinterpret_cast<const uint4*>(src + 128ll * m) : kZeroPage;
        const gv4* gg = reinterpret_cast<const gv4*>(reinterpret_cast<uintptr_t>(g));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const v4u32 v = gg[k];
            Q[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
    }
    // the top pair m (once per stream) may reach past the stream's end, where a wide load could
    // cross into an unmapped page: it is read as the aligned dwords holding stream bytes (each
    // inside its 128-B line) and funnelled to the stream's byte alignment by v_alignbyte
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
    // W = bytes [P, P+4): ring rows (P>>2)&31 and the next (row 32 mirrors row 0).  With the
    // ring base in the ds offsets the row address is one v_and_or of (P << 10) and the lane's column.
    // The position is kept in bits (P8): renorm_up8 returns bit counts, and v_alignbit_b32 takes
    // the window's bit offset 8 (P & 3) = P8 & 31 as it is.
    uint32_t wx, wy, col;  // col = 4 * lane: the lane's byte column in the ring
    __device__ __forceinline__ void read_window() {
        // row (P>>2)&31: the mask first, then one v_lshl_or (a left shift by a constant issues
        // at the slow rate, profiles/r02_valu_microbench.txt, and v_and_or would need it)
        uint32_t a;
        asm("v_lshl_or_b32 %0, %1, 7, %2" : "=v"(a) : "v"(static_cast<uint32_t>(P8) & 0x3E0u), "v"(col));
        wy = lds_ld32(a + kDecTableBytes);
        wx = lds_ld32(a + kDecTableBytes + 4 * kDecBlock);
    }
    // (v_alignbit_b32 reads only the low five bits of its shift operand: P8 needs no mask)
    __device__ __forceinline__ void form_window() { W = __builtin_amdgcn_alignbit(wx, wy, static_cast<uint32_t>(P8)); }
    // the top two pages land before decoding starts; the pair below them is requested.
    // s: the stream's first byte, at any alignment (a dense container).  Positions count from s
    // itself (sh = 0), so every lane's pages start at its own stream's start: streams of similar
    // length then cross page boundaries at nearly the same symbols, in a dense container as in
    // slots, and a wave runs the landing code about once per page rather than at every point
    // (with pages at absolute 64-B boundaries the packed streams' random phases put some lane's
    // landing at nearly every point: +2.2 VALU per symbol, profiles/r03_pmc_dense_vs_slot.txt).
    __device__ __forceinline__ void start(const uint8_t* s, int32_t slen) {
        sh = 0;
        src = s;
        const int32_t len = slen;
        const int32_t top = len > 0 ? (len - 1) >> 6 : 0;
        if (len > 0) fetch_top(top >> 1, len);
        else fetch_pair(-1);
        wait_vm();
        put_page(top);
        if (top & 1) {
            put_page(top - 1);
            fetch_pair((top >> 1) - 1);  // holds top-3, top-2
        } else {
            fetch_pair((top >> 1) - 1);  // holds top-2, top-1
            wait_vm();
            put_page(top - 1);  // top-2 stays in the low half
        }
        low = top - 1;
        lim8 = 8 * (64 * low + 60);
        P8 = 8 * (len - 4);
        read_window();
        head = 0;
    }
    // renorm_up one byte at a time (unflatten and the final equality check only)
    __device__ __forceinline__ void pull_until(uint64_t bound) {
        for (int g = 0; g < 9 && head < bound; ++g) {
            form_window();
            head = (head << 8) | (W >> 24);
            P8 -= 8;
            read_window();
        }
    }
    // page low+1 is no longer read once ((P >> 2) + 1) >> 4 <= low, i.e. P < 64 low + 60
    // (floor division throughout, negative positions included): one compare per point, in bits
    int32_t lim8;  // 8 (64 low + 60)
    __device__ __forceinline__ void point() {
        if (P8 < lim8) {  // land the page below
            put_page(low - 1);
            --low;
            lim8 -= 512;
            if (!(low & 1)) fetch_pair((low >> 1) - 1);  // the next page (low-1, odd) opens a new pair
        }
    }
    // phase 1: renorm_up, q/cf, next window
    template <bool kJ4, int kNR = kNormStd>
    __device__ __forceinline__ void renorm_div(uint64_t L, uint32_t hL8, uint32_t norm, double rcp_norm,
                                               double neg_norm = 0.0) {
        form_window();
        P8 -= static_cast<int32_t>(renorm_up8<kJ4>(head, W, L, hL8));
        read_window();  // for the next step; kept ahead of this step's bucket reads
        __builtin_amdgcn_sched_barrier(0);
        div_norm<kNR>(head, norm, rcp_norm, qq, cf, neg_norm);
    }
    // phase 1 for kModeU: the quotient from below, q_m = qq's low word and hi = hi32(q_m) (no
    // fix-up: u = head - q_m * norm in [0, 2 norm) goes to the u-domain tables as it is)
    // kNormSmall: the estimate divides x' = (H - qh norm) 2^32 + lo after the exact high step
    // (div_hi, rcp_norm rounded up): x' / norm in [2^32, 2^33), so q_m - qh 2^32 is too, and u is
    // the same low-word product (x' and head agree in their low words)
    //
    // r05: the estimate lands in the binade [2^49, 2^50), whose ulp is 1/8: t = fma(x, 1/(8 norm),
    // 2^49 - 1/8) holds q_m in its 52 mantissa bits exactly as 2^52 - 1 with 1/norm did (the same
    // rounding, scaled by the exact power 2^-3), but the raw high word is 0x43000000 + hi32(q_m):
    // its low 24 bits ARE hi32(q_m), which is all that update<kP24>'s v_mad_u32_u24 reads, so the
    // v_and that cleared the exponent (0x433: bits 20-21 set) goes (kP24 only; decode -1 VALU per
    // symbol).  rcp8 = rcp_norm / 8 (exact).
    template <bool kJ4, int kNR = kNormStd, bool kP24 = false, bool kScreen = true>
    __device__ __forceinline__ void renorm_div_u(uint64_t L, uint32_t hL8, uint32_t norm, double rcp_norm, double rcp8,
                                                 double magic, double neg_norm = 0.0) {
        form_window();
        P8 -= static_cast<int32_t>(renorm_up8<kJ4, kScreen>(head, W, L, hL8));
        read_window();  // for the next step; kept ahead of this step's bucket reads
        __builtin_amdgcn_sched_barrier(0);
        // 1/(8 norm) from its SGPR pair (an asm "v" operand copied it into a VGPR pair every step)
        // and the magic 2^49 - 1/8 from a loop-invariant VGPR pair as the third operand of one
        // VOP3 v_fma_f64 (__builtin_fma became v_fmac_f64 on a v_mov_b64 copy of the magic: one
        // 64-bit move per step)
        uint32_t qh = 0;
        double tq;
        if constexpr (kNR == kNormStd) {
            // r05: no conversion.  V = 2^64 + (head >> 12) 2^12 is a double by its bits alone:
            // exponent field 0x43F and the 52-bit mantissa head >> 12, two v_alignbit where two
            // v_cvt_f64_u32 and a v_fmac_f64 formed fl(head) (-1 VALU, -4.3 issue cycles per
            // step).  magic here is (2^49 - 1/8) - 2^61 fl(1/norm) rounded once, so the fma takes
            // the 2^64 back off with the same reciprocal: t = RN(V fl(1/(8 norm)) + magic) =
            // 2^49 - 1/8 + x'/(8 norm) + e, x' in (head - 2^12, head], |e| < 2^-5 + 2^-8 (the
            // magic's rounding in its binade below 2^49, the reciprocal's), so q_m stays in
            // {q - 1, q} for every norm >= 2^16 (x' / norm is at most 2^-4 below head / norm;
            // checked with exact rounding over 2.2e5 (head, norm) pairs, heads at multiples of the
            // norm and 2^12 around them included)
            uint32_t vlo, vhi;
            asm("v_alignbit_b32 %0, %1, %2, 12" : "=v"(vlo) : "v"(hi32(head)), "v"(lo32(head)));
            asm("v_alignbit_b32 %0, %1, %2, 12" : "=v"(vhi) : "s"(0x43Fu), "v"(hi32(head)));
            const double vd = __longlong_as_double(static_cast<long long>(mk64(vhi, vlo)));
            asm("v_fma_f64 %0, %1, %2, %3" : "=v"(tq) : "v"(vd), "s"(rcp8), "v"(magic));
        } else {
            double hd;
            asm("v_cvt_f64_u32 %0, %1" : "=v"(hd) : "v"(hi32(head)));
            if constexpr (kNR == kNormSmall) qh = div_hi(hd, rcp_norm, neg_norm);
            const double xd = __builtin_fma(hd, 4294967296.0, static_cast<double>(lo32(head)));
            asm("v_fma_f64 %0, %1, %2, %3" : "=v"(tq) : "v"(xd), "s"(rcp8), "v"(magic));
        }
        const uint64_t raw = static_cast<uint64_t>(__double_as_longlong(tq));  // q_m + 0x43000000'00000000
        cf = lo32(head) - lo32(raw) * norm;            // u (src/ans.rs:110-111 before the split)
        // (kNormSmall: + qh in the high word, q_m = qh 2^32 + the estimate)
        const uint32_t hw = kNR == kNormSmall ? hi32(raw) + qh : hi32(raw);
        if constexpr (kP24) qq = mk64(hw, lo32(raw));  // (low 24 bits: hi32(q_m) < 2^24)
        else qq = mk64(hw - 0x43000000u, lo32(raw));   // q_m < 2^52 (+ qh 2^32)
    }
    // the u-domain icdf: bucket u >> shift -> threshold words (w1, w2) with s0 in w1's low bits
    // (kDecUNbMax), the virtual symbol v = s0 + [rx > w1] + [rx > w2] for rx = u << rshift
    // (rshift = 31 - shift: rx and the words agree in bit 31, so each test is a sign bit), then its
    // row (cum_row, p); only v's low 13 bits reach the row address
    __device__ __forceinline__ void lookup_u(uint32_t shift, uint32_t rshift) {
        const uint32_t bi = cf >> shift;
        const uint64_t cc = lds_ld64(shl16<3>(bi));  // bi < kDecUNbMax
        const uint32_t rx = cf << rshift;
        const uint32_t w1 = lo32(cc), w2 = hi32(cc);
        asm volatile("v_add3_u32 %0, %1, %2, %3"
                     : "=v"(sx)
                     : "v"(w1), "v"((w1 - rx) >> 31), "v"((w2 - rx) >> 31));
        const uint64_t row = lds_ld64(kDecURowOff + shl16<3>(sx));  // (sx mod 2^13) < 512
        cum = lo32(row);
        nxt = hi32(row);  // pmf(s)
        far = false;
    }
    // phase 2: icdf (src/codec.rs:65-68), the last symbol with cdf <= cf, from cf's bucket:
    // c0..c3 in one ds_read_b128 (two compares pick among three candidates; cf >= c3 is the
    // voted far case), s0 from the array after the buckets.
    __device__ __forceinline__ void lookup(uint32_t shift) {
        const uint32_t bi = cf >> shift;
        // the bucket as two 8-B halves from two arrays (c0,c1 | c2,c3): random 16-B rows cost
        // more LDS bank-conflict cycles than two random 8-B reads
        const uint64_t ca = lds_ld64(bi << 3), cb = lds_ld64((bi << 3) + 8 * kDecNbMax);
        const uint4 c = make_uint4(lo32(ca), hi32(ca), lo32(cb), hi32(cb));
        const uint32_t s0 = *reinterpret_cast<const lds_u8*>(static_cast<uintptr_t>(bi + kDecS0Off));
        // the read completes here: the compiler otherwise defers parts a select needs only on
        // some lanes into branches, adding dependent LDS round trips
        asm volatile("" ::"v"(c.x), "v"(c.y), "v"(c.z), "v"(c.w));
        const bool b1 = cf >= c.y, b2 = cf >= c.z;
        cum = b2 ? c.z : (b1 ? c.y : c.x);
        nxt = b2 ? c.w : (b1 ? c.z : c.y);
        sx = s0 + (b1 ? 1u : 0u) + (b2 ? 1u : 0u);
        far = cf >= c.w;
    }
    // no-far lookup through the symbol's row: s = s0 + [cf >= cdf(s0+1)] + [cf >= cdf(s0+2)]
    // by two v_addc on the compare masks, then (cdf(s), pmf(s)) in one ds_read_b64 of row s:
    // a second, dependent LDS read in place of six selects
    __device__ __forceinline__ void lookup_rows(uint32_t shift) {
        const uint32_t bi = cf >> shift;
        const uint64_t cc = lds_ld64(shl16<3>(bi));  // bi < kDecNbMax
        const uint32_t s0 = *reinterpret_cast<const lds_u8*>(static_cast<uintptr_t>(bi + kDecS0OffR));
        asm volatile(
            "v_cmp_ge_u32 vcc, %[cf], %[c1]\n\t"
            "s_nop 1\n\t"
            "v_addc_co_u32 %[sx], vcc, 0, %[s0], vcc\n\t"
            "v_cmp_ge_u32 vcc, %[cf], %[c2]\n\t"
            "s_nop 1\n\t"
            "v_addc_co_u32 %[sx], vcc, 0, %[sx], vcc"
            : [sx] "=&v"(sx)
            : [cf] "v"(cf), [c1] "v"(lo32(cc)), [c2] "v"(hi32(cc)), [s0] "v"(s0)
            : "vcc");
        const uint64_t row = lds_ld64(kDecRowOff + shl16<3>(sx));  // sx < 256
        cum = lo32(row);
        nxt = hi32(row);  // pmf(s)
        far = false;
    }
    __device__ __forceinline__ void lookup_far(const uint32_t* lcum) {  // 3+ boundaries in the bucket
        if (far) {
            sx += 1;
            while (cf >= lcum[sx + 1]) ++sx;
            cum = lcum[sx];
            nxt = lcum[sx + 1];
        }
    }
    // phase 3: head = p*q + r (src/ans.rs:113-114).  With every mass below 2^24 (kP24) the
    // high word's product hi32(q) * p (hi32(q) < 2^16 in the fast range) is one full-rate
    // v_mad_u32_u24 instead of a second v_mad_u64_u32.
    template <bool kP24, bool kRowP = false>
    __device__ __forceinline__ void update() {
        const uint32_t p = kRowP ? nxt : nxt - cum, a = cf - cum;
        if constexpr (kP24) {
            const uint64_t lo = static_cast<uint64_t>(lo32(qq)) * p + a;
            uint32_t hi;
            asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(hi) : "v"(hi32(qq)), "v"(p), "v"(hi32(lo)));
            head = mk64(hi, lo32(lo));
        } else {
            head = qq * p + a;
        }
    }
};

// SPP: symbols per point (U, or U/2 when U*KMAX > 60: u8 tables whose pops can take 4 bytes).
// kMode: the icdf (kModeFar: some bucket holds more than four cdf boundaries, so the voted slow
// path is compiled in; kModeRows: every bucket resolves among three candidates, then the
// symbol's row; kModeU: kModeRows over u = head - q_m * norm, no quotient fix-up).
// kP24: every mass is below 2^24 (DecChain::update).  kJ4: some pop can pull 4 bytes (kmax = 4).
// kVar: chunk c decodes vlen[c] <= chunk_len symbols into the start of its stride (staged output).
// kNR: the norm range (div_norm, renorm_div_u; kNormBig never has the u-domain tables).
template <typename Sym, int SPP, int kMode, bool kP24, bool kJ4, bool kVar = false, int kNR = kNormStd>
__global__ __launch_bounds__(kDecBlock, 4) void k_decode(FastTable t, const uint8_t* __restrict__ slots, uint64_t slot_cap,
                                                      const uint64_t* __restrict__ offsets,
                                                      const uint32_t* __restrict__ lens, uint64_t chunk_len,
                                                      uint64_t nfull, int gen_kind, Sym* __restrict__ out,
                                                      uint32_t* __restrict__ status, ChunkInit ini,
                                                      const uint32_t* __restrict__ vlen = nullptr) {
    extern __shared__ __align__(16) unsigned char lds[];
    unsigned char* tab = lds;  // tables at offset 0, ring after them
    constexpr bool kFar = kMode == kModeFar;
    constexpr bool kRows = !kFar;  // the no-far lookups read (cum, pmf) rows
    if constexpr (kMode == kModeU) {  // the u-domain image is the LDS layout itself
        const uint4* g = reinterpret_cast<const uint4*>(t.dec_u_img);
        uint4* d = reinterpret_cast<uint4*>(tab);
        for (uint32_t i = threadIdx.x; i < kDecTableBytes / 16; i += kDecBlock) d[i] = g[i];
    } else if constexpr (kRows) {
        const uint2* ga = reinterpret_cast<const uint2*>(t.dbkt);  // (cdf(s0), cdf(s0+1)) per bucket
        const uint2* gb = ga + kDecNbMax;                           // (cdf(s0+2), cdf(s0+3))
        const uint8_t* gs = reinterpret_cast<const uint8_t*>(t.dbkt) + kDecS0Off;
        uint2* pr = reinterpret_cast<uint2*>(tab);
        for (uint32_t i = threadIdx.x; i < kDecNbMax; i += kDecBlock) {
            pr[i] = make_uint2(ga[i].y, gb[i].x);
            tab[kDecS0OffR + i] = gs[i];
        }
        uint2* rows = reinterpret_cast<uint2*>(tab + kDecRowOff);
        for (uint32_t i = threadIdx.x; i < t.nsym; i += kDecBlock) rows[i] = make_uint2(t.cum[i], t.cum[i + 1] - t.cum[i]);
    } else {
        uint4* b = reinterpret_cast<uint4*>(tab);  // buckets and s0 array: dec_cum_off bytes
        const uint4* gb = reinterpret_cast<const uint4*>(t.dbkt);
        for (uint32_t i = threadIdx.x; i < t.dec_cum_off / 16; i += kDecBlock) b[i] = gb[i];
        uint32_t* cl = reinterpret_cast<uint32_t*>(tab + t.dec_cum_off);
        for (uint32_t i = threadIdx.x; i < t.nsym + 5; i += kDecBlock) cl[i] = t.cum[i];
    }
    const uint32_t* lcum = reinterpret_cast<const uint32_t*>(tab + t.dec_cum_off);
    __syncthreads();
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kDecBlock + threadIdx.x;
    if (c >= nfull) return;

    constexpr int U = 16 / static_cast<int>(sizeof(Sym));
    static_assert(U % SPP == 0, "points must split units evenly");
    const uint32_t nvalid = kVar ? vlen[c] : static_cast<uint32_t>(chunk_len);
    const int nunit = static_cast<int>((nvalid + U - 1) / U);
    const uint64_t L = t.L;
    const uint32_t hL8 = renorm_screen(L);
    static_assert(!(kNR == kNormBig && kMode == kModeU), "u spans [0, 2 norm): 32 bits only below 2^31");
    static_assert(!(kNR == kNormSmall && kJ4), "norm < 2^16: p K >= 2^40, at most two bytes per pop");
    // the deferred renorm screen (a unit re-run on the rare wave): one point per unit, u-domain
    constexpr bool kDefer = kMode == kModeU && SPP == 16 / static_cast<int>(sizeof(Sym)) && !kVar;
    const uint32_t norm = t.norm;
    const double rcp_norm = t.rcp_norm;  // (kNormSmall: rounded up)
    const double neg_norm = -static_cast<double>(norm);
    // 2^49 - 1/8 in a VGPR pair for the whole kernel (opaque, so it is not rematerialised per step)
    // (kNormStd: less 2^61 fl(1/norm), rounded once: renorm_div_u's bit-built head)
    double magic_u;
    asm("" : "=v"(magic_u) : "0"(kNR == kNormStd ? 562949953421311.875 - 2305843009213693952.0 * rcp_norm
                                                 : 562949953421311.875));
    const double rcp8 = rcp_norm * 0.125;
    const uint32_t shift = kMode == kModeU ? t.dec_u_shift : t.dec_shift;
    uint4* dst = reinterpret_cast<uint4*>(out + c * chunk_len);

    // a stream longer than its slot is foreign or corrupt: its pages would lie past the slot
    // (and no stream of a fast-path chunk reaches 2^27 bytes: positions are kept in bits)
    if ((!offsets && lens[c] > slot_cap) || lens[c] >= (1u << 27)) {
        atomicOr(status, 1u << ANS_E_LEN);
        return;
    }
    DecChain ch;
    ch.ring = reinterpret_cast<uint32_t*>(lds + kDecTableBytes) + threadIdx.x;
    ch.col = 4 * threadIdx.x;
    ch.start(slots + (offsets ? offsets[c] : c * slot_cap), static_cast<int32_t>(lens[c]));
    ch.pull_until(L);  // Message::unflatten: head 0, renorm_up pulls the flushed head

    // symbols leave in whole 128-B lines per lane (eight units): a 64-B store leaves its line
    // half-written in L2 for a block, where the streaming reads can evict it in pieces
    uint4 q[8];
    // eight units per iteration, unrolled, so each unit's symbols go straight into their q[]
    // registers (a unit index known only at run time made the compiler copy the line through
    // a branch tree of v_mov, ~20 per unit)
    for (int u0 = 0; u0 < nunit; u0 += 8) {
        // the eight units as eight inlined calls with a compile-time index (a #pragma unroll
        // over them is refused for the larger instantiations, which then index q[] in scratch)
        auto unit = [&](auto ic) __attribute__((always_inline)) {
            constexpr int uu = decltype(ic)::value;
            const int u = u0 + uu;
            if (u < nunit) {  // (uniform unless staged)
                uint32_t sv[U];
                // kDefer: the one-byte-less screen of the renorm (hi32(X) >= hL8, ~2^-24 of the
                // steps) is taken once per unit as max(hi32(head)) over its steps instead of a
                // compare per step; a wave where a lane reached it re-runs the unit from the
                // head and position saved at the unit's point with the per-step screen (the ring
                // is unchanged until the next point, and a step pulls at most KMAX bytes either
                // way, so no read leaves the landed pages)
                uint64_t h_pt = 0;
                int32_t p_pt = 0;
                uint32_t hmax = 0, hodd = 0;
                static_assert(!kDefer || U % 2 == 0, "steps in pairs");
                // (kPack4, u8 symbols: each four symbols' bytes packed into their output dword as
                // soon as they are decoded, two v_perm and a v_or, so that the unit's sixteen
                // symbols are not all live at its end beside the saved head: the deferred screen
                // otherwise spilled)
                constexpr bool kPack4 = kDefer && sizeof(Sym) == 1;
                uint32_t pw[4] = {0, 0, 0, 0};
                auto pack4 = [&](int k) __attribute__((always_inline)) {
                    const uint32_t lo = __builtin_amdgcn_perm(sv[4 * k + 1], sv[4 * k], 0x0C0C0400u);
                    const uint32_t hi = __builtin_amdgcn_perm(sv[4 * k + 3], sv[4 * k + 2], 0x04000C0Cu);
                    pw[k] = lo | hi;
                };
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    sv[j] = 0;
                    if (j % SPP == 0) {
                        wait_vm();  // point: retire what the previous point issued
                        if (j == 0 && uu == 0 && u0 > 0) {
                            uint4* d = dst + (u0 - 8);
#pragma unroll
                            for (int k = 0; k < 8; ++k) d[k] = q[k];
                        }
                        ch.point();
                        if constexpr (kDefer) {
                            h_pt = ch.head;
                            p_pt = ch.P8;
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (kVar && static_cast<uint32_t>(u * U + j) >= nvalid) continue;  // past the chunk
                    if constexpr (kMode == kModeU) {
                        // The chain's dependent part up to the bucket read at raised wave priority:
                        // the arbiter then issues it ahead of the other waves' symbol bookkeeping,
                        // so the LDS round trip starts sooner (decode -6% in a same-box A/B,
                        // DESIGN.md §3.1)
                        __builtin_amdgcn_s_setprio(2);
                        ch.template renorm_div_u<kJ4, kNR, kP24, !kDefer>(L, hL8, norm, rcp_norm, rcp8, magic_u, neg_norm);
                        if constexpr (kDefer) {  // one v_max3 per two steps
                            if (j % 2 == 0) {
                                hodd = hi32(ch.head);
                            } else {
                                asm("v_max3_u32 %0, %1, %2, %3" : "=v"(hmax) : "v"(hmax), "v"(hodd), "v"(hi32(ch.head)));
                            }
                        }
                        ch.lookup_u(shift, 31u - shift);
                        __builtin_amdgcn_s_setprio(0);
                    } else {
                        ch.template renorm_div<kJ4, kNR>(L, hL8, norm, rcp_norm, neg_norm);
                        if constexpr (kFar) {
                            ch.lookup(shift);
                            if (__builtin_expect(__any(ch.far), 0)) ch.lookup_far(lcum);
                        } else {
                            ch.lookup_rows(shift);
                        }
                    }
                    ch.template update<kP24, kRows>();
                    sv[j] = ch.sx;  // kModeU: the virtual symbol (its low byte is the symbol)
                    if constexpr (kPack4) {
                        if (j % 4 == 3) pack4(j / 4);
                    }
                }
                if constexpr (kDefer) {
                    if (__builtin_expect(__builtin_amdgcn_ballot_w64(hmax >= hL8) != 0, 0)) {
                        ch.head = h_pt;  // the unit again, with the per-step screen
                        ch.P8 = p_pt;
                        ch.read_window();
#pragma unroll
                        for (int j = 0; j < U; ++j) {
                            ch.template renorm_div_u<kJ4, kNR, kP24, true>(L, hL8, norm, rcp_norm, rcp8, magic_u, neg_norm);
                            ch.lookup_u(shift, 31u - shift);
                            ch.template update<kP24, kRows>();
                            sv[j] = ch.sx;
                            if constexpr (kPack4) {
                                if (j % 4 == 3) pack4(j / 4);
                            }
                        }
                    }
                }
                uint4 outv = make_uint4(0, 0, 0, 0);
                if constexpr (kPack4) {
                    outv = make_uint4(pw[0], pw[1], pw[2], pw[3]);
                } else if constexpr (sizeof(Sym) == 1 && kMode == kModeU) {  // the low bytes, by v_perm: two per dword and an or
                    uint32_t w[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint32_t lo = __builtin_amdgcn_perm(sv[4 * k + 1], sv[4 * k], 0x0C0C0400u);
                        const uint32_t hi = __builtin_amdgcn_perm(sv[4 * k + 3], sv[4 * k + 2], 0x04000C0Cu);
                        w[k] = lo | hi;
                    }
                    outv = make_uint4(w[0], w[1], w[2], w[3]);
                } else if constexpr (kMode == kModeU) {
#pragma unroll
                    for (int j = 0; j < U; ++j) put_sym<Sym>(outv, j, sv[j] & 0xFFu);
                } else if constexpr (sizeof(Sym) == 1) {  // three v_lshl_or per dword
                    uint32_t w[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        uint32_t x;
                        asm("v_lshl_or_b32 %0, %1, 8, %2\n\t"
                            "v_lshl_or_b32 %0, %3, 16, %0\n\t"
                            "v_lshl_or_b32 %0, %4, 24, %0"
                            : "=&v"(x) : "v"(sv[4 * k + 1]), "v"(sv[4 * k]), "v"(sv[4 * k + 2]), "v"(sv[4 * k + 3]));
                        w[k] = x;
                    }
                    outv = make_uint4(w[0], w[1], w[2], w[3]);
                } else {
#pragma unroll
                    for (int j = 0; j < U; ++j) put_sym<Sym>(outv, j, sv[j]);
                }
                q[uu] = outv;
            }
        };
        unroll_seq(unit, std::make_integer_sequence<int, 8>{});
    }
    wait_vm();
    if (nunit > 0) {  // the last (partial) line: 4 or 8 units (chunk bytes % 64 == 0; staged: all 8)
        const int rem = kVar ? 8 : ((nunit - 1) & 7) + 1;
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
    const int32_t remaining = (ch.P8 >> 3) + 4 - ch.sh;  // < 0: generated
    if (remaining < 0 && gen_kind == ANS_GEN_EMPTY) atomicOr(status, 1u << ANS_E_EXHAUSTED);
    else if (ch.head != ini.head(c) || remaining != 0) atomicOr(status, 1u << ANS_E_MISMATCH);
}

// ====================================================================== decode, large alphabets
// Alphabets above 256 symbols (C4: 65,536) keep their decode buckets in global memory
// (DecBucketG, 32 B: cdf(s0..s0+5) and s0, at most 2^16 buckets = 2 MiB, L2-resident): one load
// per symbol on the dependency chain.  gfx9 retires vector-memory operations in issue order, so
// every such load also waits for the ring's page fetches and the symbol stores issued before
// it; those are therefore batched per BLOCK (four units = 64 bytes of symbols per lane) and
// issued together at the block's point, which exposes one HBM latency per block instead of
// one per unit.  The ring has four pages (65 rows, row 64 mirrors row 0); a block pops at most
// 4U*KMAX <= 128 bytes, and up to two pages land per point, so reads never reach an unlanded
// page.
constexpr int kDecGRows = 65;
constexpr uint32_t kDecGRingBytes = kDecGRows * kBlock * 4;

struct DecChainG {
    uint32_t* ring;  // &ring[0][lane]
    const uint8_t* src;
    uint4 S0[4], S1[4];  // pages low-1 and low-2, in flight
    int32_t low, P, sh;  // sh: the stream start within its 128-B line
    uint32_t wx, wy, W;
    uint64_t head;
    uint64_t qq;
    uint32_t cf, cum, nxt, sx;
    bool far;

    __device__ __forceinline__ uint32_t& row(int32_t r) const { return ring[r * kBlock]; }
    __device__ __forceinline__ void put_page(int32_t p, uint4* S) {
        clear_below(S[0], S[1], S[2], S[3], 64 * p, sh);
        const int32_t r0 = (p & 3) * 16;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            row(r0 + 4 * k + 0) = S[k].x;
            row(r0 + 4 * k + 1) = S[k].y;
            row(r0 + 4 * k + 2) = S[k].z;
            row(r0 + 4 * k + 3) = S[k].w;
        }
        if ((p & 3) == 0) row(64) = S[0].x;
    }
    __device__ __forceinline__ void fetch_page(int32_t p, uint4* S) {
        if (p >= 0) {
            // streamed once: non-temporal, so the pages do not evict the bucket table from L2
            const uint4* g = reinterpret_cast<const uint4*>(src + 64ll * p);
#pragma unroll
            for (int k = 0; k < 4; ++k) S[k] = nt_load(g + k);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) S[k] = make_uint4(0, 0, 0, 0);
        }
    }
    __device__ __forceinline__ void read_window() {
        const uint32_t* a = ring + ((static_cast<uint32_t>(P) >> 2) & 63u) * kBlock;
        wy = a[0];
        wx = a[kBlock];
    }
    __device__ __forceinline__ void form_window() { W = ab(wx, wy, static_cast<uint32_t>(P)); }  // low 2 bits used
    // the top four pages land before decoding starts; the next two are requested
    // s: the stream's first byte, at any alignment (a dense container).  Positions count from
    // the 128-B line holding it (base = s - sh), so every fetch is whole aligned lines, read
    // only from lines that hold stream bytes; the sh bytes below the stream (another chunk's)
    // are reached only by a corrupt stream, which the final position check reports.
    __device__ __forceinline__ void start(const uint8_t* s, int32_t slen) {
        sh = static_cast<int32_t>(reinterpret_cast<uintptr_t>(s) & 127u);
        src = s - sh;
        const int32_t len = slen + sh;
        const int32_t top = len > 0 ? (len - 1) >> 6 : 0;
        fetch_page(len > 0 ? top : -1, S0);
        fetch_page(top - 1, S1);
        wait_vm();
        put_page(top, S0);
        put_page(top - 1, S1);
        fetch_page(top - 2, S0);
        fetch_page(top - 3, S1);
        wait_vm();
        put_page(top - 2, S0);
        put_page(top - 3, S1);
        low = top - 3;
        fetch_page(low - 1, S0);
        fetch_page(low - 2, S1);
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
    // at a block point, after s_waitcnt vmcnt(0): land what the read frontier allows
    __device__ __forceinline__ void point() {
        const int32_t f = ((P >> 2) + 1) >> 4;  // page of the highest dword still to be read
        const bool l1 = f <= low + 2;           // page low-1 may take page low+3's slot
        const bool l2 = f <= low + 1;           // page low-2 may take page low+2's slot
        if (l1) put_page(low - 1, S0);
        if (l2) {
            put_page(low - 2, S1);
            low -= 2;
            fetch_page(low - 1, S0);
            fetch_page(low - 2, S1);
        } else if (l1) {
            low -= 1;
#pragma unroll
            for (int k = 0; k < 4; ++k) S0[k] = S1[k];
            fetch_page(low - 2, S1);
        }
    }
    template <int kNR = kNormStd>
    __device__ __forceinline__ void renorm_div(uint64_t L, uint32_t hL8, uint32_t norm, double rcp_norm,
                                               double neg_norm = 0.0) {
        form_window();
        P -= static_cast<int32_t>(renorm_up(head, W, L, hL8));
        read_window();  // for the next step; kept ahead of this step's bucket reads
        __builtin_amdgcn_sched_barrier(0);
        div_norm<kNR>(head, norm, rcp_norm, qq, cf, neg_norm);
    }
    __device__ __forceinline__ void lookup(const DecBucketG* __restrict__ bkt, uint32_t shift) {
        const uint4* e = reinterpret_cast<const uint4*>(bkt + (cf >> shift));
        uint4 a = e[0], b = e[1];  // c0..c3 | c4, c5, s0, -
        // both loads complete here (no loads sunk into the selects' branches)
        asm volatile("" ::"v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z));
        const bool b1 = cf >= a.y, b2 = cf >= a.z, b3 = cf >= a.w, b4 = cf >= b.x;
        cum = b4 ? b.x : (b3 ? a.w : (b2 ? a.z : (b1 ? a.y : a.x)));
        nxt = b4 ? b.y : (b3 ? b.x : (b2 ? a.w : (b1 ? a.z : a.y)));
        sx = b.z + (b1 ? 1u : 0u) + (b2 ? 1u : 0u) + (b3 ? 1u : 0u) + (b4 ? 1u : 0u);
        far = cf >= b.y;
    }
    __device__ __forceinline__ void lookup_far(const uint32_t* __restrict__ gcum) {
        if (far) {
            sx += 1;
            while (cf >= gcum[sx + 1]) ++sx;
            cum = gcum[sx];
            nxt = gcum[sx + 1];
        }
    }
    __device__ __forceinline__ void update() { head = qq * (nxt - cum) + (cf - cum); }
};

// kNR: the norm range (div_norm: kNormSmall's long division, kNormBig's 64-bit remainder)
template <typename Sym, int kNR = kNormStd>
__global__ __launch_bounds__(kBlock, 2) void k_decode_g(FastTable t, const uint8_t* __restrict__ slots,
                                                        uint64_t slot_cap, const uint64_t* __restrict__ offsets,
                                                        const uint32_t* __restrict__ lens,
                                                        uint64_t chunk_len, uint64_t nfull, int gen_kind,
                                                        Sym* __restrict__ out, uint32_t* __restrict__ status,
                                                        ChunkInit ini) {
    extern __shared__ __align__(16) unsigned char lds[];
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (c >= nfull) return;  // no barrier below: lanes are independent

    constexpr int U = 16 / static_cast<int>(sizeof(Sym));
    static_assert(U * 4 * 4 <= 128, "a block pops at most two pages");
    const int nblocks = static_cast<int>(chunk_len / (4 * U));
    const uint64_t L = t.L;
    const uint32_t hL8 = renorm_screen(L);
    const uint32_t norm = t.norm;
    const double rcp_norm = t.rcp_norm;
    const uint32_t shift = t.dec_shift;
    uint4* dst = reinterpret_cast<uint4*>(out + c * chunk_len);

    if (!offsets && lens[c] > slot_cap) {  // foreign or corrupt stream: its pages would lie past the slot
        atomicOr(status, 1u << ANS_E_LEN);
        return;
    }
    DecChainG ch;
    ch.ring = reinterpret_cast<uint32_t*>(lds) + threadIdx.x;
    ch.start(slots + (offsets ? offsets[c] : c * slot_cap), static_cast<int32_t>(lens[c]));
    ch.pull_until(L);

    uint4 q[4];
    for (int b = 0; b < nblocks; ++b) {
        wait_vm();  // block point
        if (b > 0) {
            uint4* d = dst + 4 * (b - 1);
            nt_store(d + 0, q[0]);
            nt_store(d + 1, q[1]);
            nt_store(d + 2, q[2]);
            nt_store(d + 3, q[3]);
        }
        ch.point();
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            uint4 outv = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int j = 0; j < U; ++j) {
                ch.template renorm_div<kNR>(L, hL8, norm, rcp_norm, -static_cast<double>(norm));
                ch.lookup(t.dbkt_g, shift);
                if (__builtin_expect(__any(ch.far), 0)) ch.lookup_far(t.cum);
                ch.update();
                put_sym<Sym>(outv, j, ch.sx);
            }
            q[u] = outv;
        }
    }
    wait_vm();
    if (nblocks > 0) {
        uint4* d = dst + 4 * (nblocks - 1);
        d[0] = q[0];
        d[1] = q[1];
        d[2] = q[2];
        d[3] = q[3];
    }
    ch.pull_until(kMaxMinHead);
    const int32_t remaining = ch.P + 4 - ch.sh;
    if (remaining < 0 && gen_kind == ANS_GEN_EMPTY) atomicOr(status, 1u << ANS_E_EXHAUSTED);
    else if (ch.head != ini.head(c) || remaining != 0) atomicOr(status, 1u << ANS_E_MISMATCH);
}

// ====================================================================== bulk sampling
// Codec::samples (src/ans.rs:38-44) on the fast decoder's tables: chunk c = len pops from
// Message::random(seed + c) (head 1 then renorm_up from the generator, src/ans.rs:285-290),
// every renorm byte drawn from TailGenerator::Random (src/ans.rs:142-157).  The decode
// buckets and cdf sit in LDS as in k_decode (one 1,024-lane workgroup per CU shares them);
// q, cf by the f64 estimate (div_norm), the icdf by the 3-candidate bucket plus the voted
// scan, head = p*q + cf - cum.  Symbols leave in 16-B groups per lane when the chunk is
// aligned, else one by one.
template <typename Sym>
__global__ __launch_bounds__(kDecBlock, 4) void k_sample(FastTable t, uint64_t seed, uint64_t n, uint64_t chunk_len,
                                                      uint64_t nchunks, Sym* __restrict__ out) {
    extern __shared__ __align__(16) unsigned char lds[];
    {
        uint4* b = reinterpret_cast<uint4*>(lds);
        const uint4* gb = reinterpret_cast<const uint4*>(t.dbkt);
        for (uint32_t i = threadIdx.x; i < t.dec_cum_off / 16; i += kDecBlock) b[i] = gb[i];
        uint32_t* cl = reinterpret_cast<uint32_t*>(lds + t.dec_cum_off);
        for (uint32_t i = threadIdx.x; i < t.nsym + 5; i += kDecBlock) cl[i] = t.cum[i];
    }
    const uint32_t* lcum = reinterpret_cast<const uint32_t*>(lds + t.dec_cum_off);
    __syncthreads();
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kDecBlock + threadIdx.x;
    if (c >= nchunks) return;
    Pcg64Mcg rng;
    rng.seed_from_u64(seed + c);
    uint64_t head = 1;
    while (head < kMaxMinHead) head = (head << 8) | rng.next_byte();
    const uint64_t L = t.L;
    const uint32_t norm = t.norm, shift = t.dec_shift;
    const double rcp_norm = t.rcp_norm;
    auto pop = [&]() __attribute__((always_inline)) {
        while (head < L) head = (head << 8) | rng.next_byte();  // renorm (src/ans.rs:109,239-243)
        uint64_t qq;
        uint32_t cf;
        div_norm(head, norm, rcp_norm, qq, cf);
        const uint32_t bi = cf >> shift;
        const uint64_t ca = lds_ld64(bi << 3), cb = lds_ld64((bi << 3) + 8 * kDecNbMax);
        const uint32_t s0 = *reinterpret_cast<const lds_u8*>(static_cast<uintptr_t>(bi + kDecS0Off));
        const bool b1 = cf >= hi32(ca), b2 = cf >= lo32(cb);
        uint32_t cum = b2 ? lo32(cb) : (b1 ? hi32(ca) : lo32(ca));
        uint32_t nxt = b2 ? hi32(cb) : (b1 ? lo32(cb) : hi32(ca));
        uint32_t sx = s0 + (b1 ? 1u : 0u) + (b2 ? 1u : 0u);
        if (__builtin_expect(__any(cf >= hi32(cb)), 0)) {
            if (cf >= hi32(cb)) {  // 3+ boundaries in the bucket: scan the staged cdf
                sx += 1;
                while (cf >= lcum[sx + 1]) ++sx;
                cum = lcum[sx];
                nxt = lcum[sx + 1];
            }
        }
        head = qq * (nxt - cum) + (cf - cum);  // src/ans.rs:113-114
        return sx;
    };
    const uint64_t a = c * chunk_len, b = min(a + chunk_len, n);
    uint64_t k = a;
    constexpr int U = 16 / static_cast<int>(sizeof(Sym));
    if ((a * sizeof(Sym)) % 16 == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
        for (; k + U <= b; k += U) {
            uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int j = 0; j < U; ++j) put_sym<Sym>(v, j, pop());
            *reinterpret_cast<uint4*>(out + k) = v;
        }
    }
    for (; k < b; ++k) out[k] = static_cast<Sym>(pop());
}

}  // namespace fast
}  // namespace shuffle_coding
