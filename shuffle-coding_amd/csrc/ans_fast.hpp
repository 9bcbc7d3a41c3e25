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

#include "ans_table.hpp"

namespace shuffle_coding {
namespace fast {

constexpr int kBlock = 512;      // 8 waves; 2 workgroups (16 waves) per CU
constexpr int kRingDwords = 32;  // 128-byte ring per lane = 2 pages of 64 bytes
constexpr int kGroupBytes = 64;  // symbols move in 64-byte groups (4 units)
constexpr uint64_t kMaxMinHead = 1ull << 56;

// s_waitcnt vmcnt(0) (gfx9 encoding; expcnt/lgkmcnt left at their maxima).
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }

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

// Lane-private ring of 32 dwords in a [dword][lane] image.
struct Ring {
    uint32_t* base;  // &image[0][lane]
    __device__ __forceinline__ uint32_t& at(int32_t i) const {
        return base[(static_cast<uint32_t>(i) & 31u) * kBlock];
    }
};

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
// Byte funnel: (a1:a0) holds n stream bytes MSB-aligned, oldest lowest (n <= 3 between pushes).
// Pushing k bytes shifts the head's low k bytes in at the top; each completed 4 bytes are a
// little-endian stream dword and go to the ring.
struct Funnel {
    uint32_t a0, a1, n, wd;  // wd = stream dwords completed

    template <int KMAX>
    __device__ __forceinline__ void push(uint32_t lo, uint32_t k, const Ring& ring) {
        uint32_t b0 = ab(a1, a0, k), b1 = ab(lo, a1, k);
        if constexpr (KMAX >= 4) {
            b0 = k == 4 ? a1 : b0;
            b1 = k == 4 ? lo : b1;
        }
        a0 = b0;
        a1 = b1;
        n += k;
        // oldest 4 bytes; written unconditionally (a partial dword is rewritten once complete)
        ring.at(static_cast<int32_t>(wd)) = n == 4 ? a1 : ab(a1, a0, 8 - n);
        const uint32_t full = n >= 4 ? 1u : 0u;
        wd += full;
        n -= 4 * full;
    }
};

__device__ __forceinline__ void flush_page(const Ring& ring, uint32_t p, uint8_t* dst) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = ring.at(static_cast<int32_t>(16 * p + i));
    uint4* d = reinterpret_cast<uint4*>(dst + 64ull * p);
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// KMAX: most bytes one push can emit (table property); kK32: K < 2^32 (norm > 2^24).
template <typename Sym, int KMAX, bool kK32>
__global__ __launch_bounds__(kBlock, 4) void k_encode(FastTable t, const Sym* __restrict__ syms, uint64_t chunk_len,
                                                      uint64_t nfull, uint8_t* __restrict__ slots, uint64_t slot_cap,
                                                      uint32_t* __restrict__ lens, uint32_t* __restrict__ status) {
    extern __shared__ __align__(16) unsigned char lds[];
    EncRow* rows = reinterpret_cast<EncRow*>(lds);
    for (uint32_t i = threadIdx.x; i < t.enc_rows; i += kBlock) rows[i] = t.enc[i];
    const Ring ring{reinterpret_cast<uint32_t*>(lds + t.enc_lds_bytes) + threadIdx.x};
    __syncthreads();
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (c >= nfull) return;

    constexpr int U = 16 / static_cast<int>(sizeof(Sym));
    const uint4* src = reinterpret_cast<const uint4*>(syms + c * chunk_len);
    const int ngroups = static_cast<int>(chunk_len * sizeof(Sym) / kGroupBytes);
    uint8_t* dst = slots + c * slot_cap;
    const uint32_t npages_cap = static_cast<uint32_t>(slot_cap / 64);
    const uint64_t norm = t.norm;
    const uint64_t K = t.K;
    const uint32_t sentinel = t.enc_rows - 1;  // zero-mass row: out-of-range symbols land here

    uint64_t head = kMaxMinHead;  // Message::zeros()
    Funnel f{0, 0, 0, 0};
    uint32_t fp = 0, over = 0;
    uint32_t minmass = ~0u;  // 0 after a zero-mass / out-of-range symbol; accumulated by an
                             // opaque v_min so the compiler cannot sink the test to the loop end
                             // (it did, keeping every row alive and spilling)

    auto point = [&]() __attribute__((always_inline)) {
        wait_vm();
        if ((f.wd >> 4) > fp) {  // at most one page completes per unit (U * KMAX <= 64 bytes)
            if (fp < npages_cap) flush_page(ring, fp, dst);
            else over = 1;
            ++fp;
        }
    };
    auto process = [&](const uint4& unit) __attribute__((always_inline)) {
        // rows are read one symbol ahead; the scheduling barriers keep the compiler from
        // hoisting all sixteen reads (and their registers) to the top of the unit
        EncRow e_next = rows[min(sym_of<Sym>(unit, U - 1), sentinel)];
#pragma unroll
        for (int j = U - 1; j >= 0; --j) {  // IID::push: last symbol first (src/codec.rs:417)
            __builtin_amdgcn_sched_barrier(0);
            const EncRow e = e_next;
            if (j > 0) e_next = rows[min(sym_of<Sym>(unit, j - 1), sentinel)];
            asm volatile("v_min_u32 %0, %0, %1" : "+v"(minmass) : "v"(e.mass));  // kept in place
            // renorm(p*K) (src/ans.rs:100,246-253): k = #{j >= 1 : (head >> 8j) >= p*K} bytes out
            const uint64_t pK = kK32 ? static_cast<uint64_t>(e.mass) * static_cast<uint32_t>(K)
                                     : static_cast<uint64_t>(e.mass) * K;
            uint32_t k = (head >> 8) >= pK ? 1u : 0u;
            if constexpr (KMAX >= 2) k += (head >> 16) >= pK ? 1u : 0u;
            if constexpr (KMAX >= 3) k += (head >> 24) >= pK ? 1u : 0u;
            if constexpr (KMAX >= 4) k += (head >> 32) >= pK ? 1u : 0u;
            f.push<KMAX>(lo32(head), k, ring);
            head >>= 8 * k;
            // q = head / p, r = head % p (src/ans.rs:101-102)
            uint64_t q = qest(head, e.rcp);
            const int32_t rr = static_cast<int32_t>(lo32(head) - lo32(q) * e.mass);
            const uint32_t neg = rr < 0 ? 1u : 0u;
            q -= neg;
            const uint32_t r = static_cast<uint32_t>(rr) + (neg ? e.mass : 0u);
            // head = norm * q + cdf(x, r) (src/ans.rs:103-104, src/codec.rs:64)
            head = q * norm + (static_cast<uint64_t>(e.cum) + r);
        }
    };

    // groups are walked last to first; group g-1's 64 bytes are requested while g is coded
    uint4 n0, n1, n2, n3;
    {
        const uint4* gsrc = src + 4 * (ngroups - 1);
        n0 = gsrc[0];
        n1 = gsrc[1];
        n2 = gsrc[2];
        n3 = gsrc[3];
    }
    for (int g = ngroups - 1; g >= 0; --g) {
        point();
        const uint4 c0 = n0, c1 = n1, c2 = n2, c3 = n3;
        {
            const uint4* gsrc = src + 4 * (g > 0 ? g - 1 : 0);
            n0 = gsrc[0];
            n1 = gsrc[1];
            n2 = gsrc[2];
            n3 = gsrc[3];
        }
        process(c3);
        point();
        process(c2);
        point();
        process(c1);
        point();
        process(c0);
    }
    wait_vm();

    // flatten (src/ans.rs:255-260): all significant head bytes, low first (7 or 8 here,
    // since the head is >= norm*K > 2^55 after any push).
    const uint32_t nb = (71u - static_cast<uint32_t>(__builtin_clzll(head))) >> 3;
    f.push<4>(lo32(head), 4, ring);
    f.push<4>(hi32(head), nb - 4, ring);
    if (f.n) ring.at(static_cast<int32_t>(f.wd)) = f.a1 >> (8 * (4 - f.n));
    const uint32_t len = 4 * f.wd + f.n;
    for (const uint32_t last = (len + 63) / 64; fp < last; ++fp) {
        if (fp < npages_cap) flush_page(ring, fp, dst);
        else over = 1;
    }
    if (minmass == 0) {  // classify like the reference: out-of-range index (codec.rs:63) or p == 0 (ans.rs:98)
        uint32_t sym_err = 0;
        for (uint64_t k = 0; k < chunk_len; ++k)
            sym_err |= static_cast<uint32_t>(syms[c * chunk_len + k]) >= t.nsym ? 1u : 0u;
        atomicOr(status, 1u << (sym_err ? ANS_E_SYMBOL : ANS_E_ZERO_MASS));
    }
    if (over) atomicOr(status, 1u << ANS_E_LEN);
    lens[c] = len;
}

// ====================================================================== decode
template <typename Sym>
__global__ __launch_bounds__(kBlock, 4) void k_decode(FastTable t, const uint8_t* __restrict__ slots,
                                                      uint64_t slot_cap, const uint32_t* __restrict__ lens,
                                                      uint64_t chunk_len, uint64_t nfull, int gen_kind,
                                                      Sym* __restrict__ out, uint32_t* __restrict__ status) {
    extern __shared__ __align__(16) unsigned char lds[];
    {
        uint4* b = reinterpret_cast<uint4*>(lds);
        const uint4* gb = reinterpret_cast<const uint4*>(t.bucket8);
        for (uint32_t i = threadIdx.x; i < t.bucket_lds_bytes / 16; i += kBlock) b[i] = gb[i];
        DecRow* r = reinterpret_cast<DecRow*>(lds + t.bucket_lds_bytes);
        for (uint32_t i = threadIdx.x; i < t.dec_rows; i += kBlock) r[i] = t.dec[i];
    }
    const uint8_t* bucket = lds;
    const DecRow* rows = reinterpret_cast<const DecRow*>(lds + t.bucket_lds_bytes);
    const Ring ring{reinterpret_cast<uint32_t*>(lds + t.dec_lds_bytes) + threadIdx.x};
    __syncthreads();
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (c >= nfull) return;

    constexpr int U = 16 / static_cast<int>(sizeof(Sym));
    const uint8_t* src = slots + c * slot_cap;
    const int32_t len = static_cast<int32_t>(lens[c]);
    uint4* dst = reinterpret_cast<uint4*>(out + c * chunk_len);
    const int nunit = static_cast<int>(chunk_len / U);
    const uint64_t L = t.L;
    const uint32_t norm = t.norm;
    const double rcp_norm = t.rcp_norm;
    const uint32_t shift = t.shift8;

    // ---- pages: page p = stream bytes [64p, 64p+64), kept in ring half p&1
    auto put_page = [&](int32_t p, const uint4& v0, const uint4& v1, const uint4& v2, const uint4& v3)
                        __attribute__((always_inline)) {
        const uint32_t w[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                                v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
#pragma unroll
        for (int i = 0; i < 16; ++i) ring.at(16 * p + i) = w[i];
    };
    auto load_page_now = [&](int32_t p) __attribute__((always_inline)) {
        const uint4* s = reinterpret_cast<const uint4*>(src + 64ll * p);
        put_page(p, s[0], s[1], s[2], s[3]);
    };
    int32_t low = len > 0 ? (len - 1) >> 6 : 0;  // lowest page present in the ring
    if (len > 0) load_page_now(low);
    uint4 S0, S1, S2, S3;  // a page in flight between two points
    int32_t pend = -1;
    auto request = [&](int32_t p) __attribute__((always_inline)) {
        const uint4* s = reinterpret_cast<const uint4*>(src + 64ll * p);
        S0 = s[0];
        S1 = s[1];
        S2 = s[2];
        S3 = s[3];
        pend = p;
    };
    auto land = [&]() __attribute__((always_inline)) {
        put_page(pend, S0, S1, S2, S3);
        low = pend;
        pend = -1;
    };
    if (low >= 1) request(low - 1);

    // ---- window: (w1:w0) holds nW stream bytes MSB-aligned (next byte to pop on top);
    //      nd = stream dword nd_idx (the next one below the window), prefetched from the ring.
    uint32_t w1 = 0, w0 = 0, nW = 0;
    int32_t nd_idx = -1;
    if (len > 0) {
        const int32_t td = (len - 1) >> 2;
        const uint32_t c0 = static_cast<uint32_t>(len - 4 * td);
        w1 = ring.at(td) << (8 * (4 - c0));
        nW = c0;
        nd_idx = td - 1;
    }
    uint32_t nd = 0;
    auto fetch_nd = [&]() __attribute__((always_inline)) {  // serve lanes whose page has not landed
        const bool starving = nd_idx >= 0 && (nd_idx >> 4) < low;
        if (__builtin_expect(__any(starving), 0)) {
            wait_vm();
            if (starving && pend >= 0) land();
            if (nd_idx >= 0 && (nd_idx >> 4) < low) {
                load_page_now(nd_idx >> 4);
                low = nd_idx >> 4;
            }
        }
        nd = nd_idx >= 0 ? ring.at(nd_idx) : 0u;  // below the stream: TailGenerator bytes (0)
    };
    fetch_nd();
    auto refill = [&]() __attribute__((always_inline)) {  // move nd into the window when nW <= 4
        const bool take = nW <= 4;
        const uint64_t wv = mk64(w1, w0) | ((static_cast<uint64_t>(nd) << 32) >> (8 * (nW & 7)));
        w1 = take ? hi32(wv) : w1;
        w0 = take ? lo32(wv) : w0;
        nW += take ? 4u : 0u;
        nd_idx -= take ? 1 : 0;
        fetch_nd();
    };
    auto pull1 = [&](uint64_t h) __attribute__((always_inline)) -> uint64_t {
        if (nW == 0) refill();
        const uint32_t b = w1 >> 24;
        w1 = ab(w1, w0, 3);
        w0 <<= 8;
        nW -= 1;
        return (h << 8) | b;
    };

    // Message::unflatten (head = 0); the first renorm_up pulls the flushed head back in.
    uint64_t head = 0;
    for (int g = 0; g < 9 && head < L; ++g) head = pull1(head);

    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0, q2 = q0, q3 = q0, outv = q0;
    for (int u = 0; u < nunit; ++u) {
        wait_vm();  // point: retire what the previous point issued
        if (u > 0 && (u & 3) == 0) {  // 64 contiguous bytes per lane
            uint4* d = dst + (u - 4);
            d[0] = q0;
            d[1] = q1;
            d[2] = q2;
            d[3] = q3;
        }
        if (pend >= 0) land();
        if (pend < 0 && low > 0 && (nd_idx >> 4) <= low) request(low - 1);
#pragma unroll
        for (int j = 0; j < U; ++j) {
            refill();
            // renorm_up (src/ans.rs:239-243): k = min{j : top64((head:W) << 8j) >= L}.  With bl
            // the head's bit length, js = (64 - bl) >> 3 bytes reach 2^56 >= L; js - 1 may too.
            const uint32_t h1 = hi32(head), h0 = lo32(head);
            const uint32_t bl = 64u - static_cast<uint32_t>(__builtin_clzll(head | 1));
            const uint32_t js = (64u - bl) >> 3;
            const uint32_t m = js - 1;
            const uint32_t s = (4u - m) & 3u;
            const uint32_t c1 = m == 0 ? h1 : ab(h1, h0, s);
            const uint32_t c0 = m == 0 ? h0 : ab(h0, w1, s);
            const uint32_t k = js - ((js >= 1 ? 1u : 0u) & (mk64(c1, c0) >= L ? 1u : 0u));
            const uint32_t sk = (4u - k) & 3u;
            const bool nz = k != 0;
            head = nz ? mk64(ab(h1, h0, sk), ab(h0, w1, sk)) : head;
            const uint32_t x1 = ab(w1, w0, sk), x0 = ab(w0, 0u, sk);
            w1 = nz ? x1 : w1;
            w0 = nz ? x0 : w0;
            nW -= k;
            // q = head / norm, cf = head % norm (src/ans.rs:110-111)
            uint64_t q = qest(head, rcp_norm);
            const int32_t ii = static_cast<int32_t>(lo32(head) - lo32(q) * norm);
            const uint32_t neg = ii < 0 ? 1u : 0u;
            q -= neg;
            const uint32_t cf = static_cast<uint32_t>(ii) + (neg ? norm : 0u);
            // icdf (src/codec.rs:65-68), last symbol with cum <= cf: the bucket gives s0, and
            // rows s0..s0+2 settle it unless the table flags a narrow neighbourhood.
            uint32_t sx = bucket[cf >> shift];
            const DecRow r0 = rows[sx], r1 = rows[sx + 1], r2 = rows[sx + 2];
            const uint32_t b1 = cf >= r1.cum ? 1u : 0u, b2 = cf >= r2.cum ? 1u : 0u;
            uint32_t cum = b2 ? r2.cum : (b1 ? r1.cum : r0.cum);
            uint32_t mass = (b2 ? r2.mass : (b1 ? r1.mass : r0.mass)) & ~kDecMulti;
            sx += b1 + b2;
            const bool multi = (r0.mass & kDecMulti) != 0;
            if (__builtin_expect(__any(multi), 0)) {
                if (multi) {
                    while (cf >= rows[sx + 1].cum) ++sx;
                    cum = rows[sx].cum;
                    mass = rows[sx].mass & ~kDecMulti;
                }
            }
            head = q * mass + (cf - cum);  // src/ans.rs:113-114
            put_sym<Sym>(outv, j, sx);
        }
        switch (u & 3) {
        case 0: q0 = outv; break;
        case 1: q1 = outv; break;
        case 2: q2 = outv; break;
        default: q3 = outv; break;
        }
    }
    wait_vm();
    if (nunit >= 4) {
        uint4* d = dst + (nunit - 4);
        d[0] = q0;
        d[1] = q1;
        d[2] = q2;
        d[3] = q3;
    }

    // assert_eq!(initial, m) with initial = Message::zeros() (src/ans.rs:56, 302-310)
    for (int g = 0; g < 9 && head < kMaxMinHead; ++g) head = pull1(head);
    const int32_t remaining = 4 * (nd_idx + 1) + static_cast<int32_t>(nW);  // < 0: generated bytes used
    if (remaining < 0 && gen_kind == ANS_GEN_EMPTY) atomicOr(status, 1u << ANS_E_EXHAUSTED);
    else if (head != kMaxMinHead || remaining != 0) atomicOr(status, 1u << ANS_E_MISMATCH);
}

}  // namespace fast
}  // namespace shuffle_coding
