// ans_kcommon.hpp — constants, error macro and device helpers shared by the kernel
// translation units (ans_kernels.hip and the per-width launch units ans_launch_*.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ans_ctx.hpp"
#include "ans_wide.hpp"

namespace {

constexpr uint64_t kMaxMinHead = 1ull << 56;  // src/ans.rs:19
constexpr int kBlock = 256;

#define HIP_TRY(expr)                                              \
    do {                                                           \
        hipError_t e_ = (expr);                                    \
        if (e_ != hipSuccess) {                                    \
            std::fprintf(stderr, "[shuffle-coding_amd] %s failed: %s\n", #expr, hipGetErrorString(e_)); \
            return ANS_E_DEVICE;                                   \
        }                                                          \
    } while (0)

// ------------------------------------------------------------------ device helpers

// floor(x / d) or floor(x / d) + 1 for x / d < 2^48, using rcp = fl(1/d).
// Adding 2^52 rounds the f64 quotient to an integer whose bits ARE the u64 value.
// Error analysis: |fl(x)*rcp - x/d| <= (x/d) * 2^-52 < 2^-4, so rounding
// lands on floor or floor + 1; the caller fixes the +1 case from the sign of the remainder.
__device__ __forceinline__ uint64_t quot_estimate(uint64_t x, double rcp) {
    const double xd = __builtin_fma(static_cast<double>(static_cast<uint32_t>(x >> 32)), 4294967296.0,
                                    static_cast<double>(static_cast<uint32_t>(x)));
    const double t = __builtin_fma(xd, rcp, 4503599627370496.0);  // + 2^52
    return static_cast<uint64_t>(__double_as_longlong(t)) - 0x4330000000000000ull;
}

__device__ __forceinline__ void raise_status(uint32_t* status, int code) { atomicOr(status, 1u << code); }

// Stages the table (and for decode, its icdf buckets) into LDS.
template <bool kWithBuckets>
__device__ __forceinline__ void stage_table(const DevTable& t, unsigned char* lds) {
    DevSym* rows = reinterpret_cast<DevSym*>(lds);
    for (uint32_t k = threadIdx.x; k <= t.nsym; k += blockDim.x) rows[k] = t.sym[k];
    if (kWithBuckets) {
        uint16_t* b = reinterpret_cast<uint16_t*>(lds + sizeof(DevSym) * (t.nsym + 1));
        for (uint32_t k = threadIdx.x; k < t.nbucket; k += blockDim.x) b[k] = t.bucket[k];
    }
    __syncthreads();
}

// icdf (src/codec.rs:65-68): the LAST x with cum[x] <= cf.  The bucket gives that x for
// the bucket's first cf; a short forward walk finishes (the sentinel row has cum = norm).
__device__ __forceinline__ uint32_t icdf(const DevSym* rows, const uint16_t* bucket, uint32_t shift, uint32_t cf) {
    uint32_t s = bucket[cf >> shift];
    while (rows[s + 1].cum <= cf) ++s;
    return s;
}

// Per-lane stream writer: bytes in push order, written 8 at a time into the lane's slot.
struct ByteSink {
    uint8_t* out;
    uint64_t cap;
    uint64_t pos;
    uint64_t acc;
    uint32_t nacc;
    bool overflow;

    __device__ __forceinline__ void put(uint32_t byte) {
        acc |= static_cast<uint64_t>(byte) << (8 * nacc);
        if (++nacc == 8) {
            if (pos + 8 <= cap) *reinterpret_cast<uint64_t*>(out + pos) = acc;
            else overflow = true;
            pos += 8;
            acc = 0;
            nacc = 0;
        }
    }
    __device__ __forceinline__ uint64_t finish() {
        if (pos + nacc > cap) overflow = true;
        else
            for (uint32_t k = 0; k < nacc; ++k) out[pos + k] = static_cast<uint8_t>(acc >> (8 * k));
        return pos + nacc;
    }
};

// Per-lane stream reader: pops bytes from the END of the stream (Tail::pop, src/ans.rs:198-203)
// through aligned 4-byte words, one word prefetched ahead.
struct ByteSource {
    uintptr_t base;
    uint64_t pos;  // bytes still in the tail
    uintptr_t floor_wa, cur_wa;
    uint32_t cur, nxt;

    __device__ __forceinline__ void init(const uint8_t* b, uint64_t len) {
        base = reinterpret_cast<uintptr_t>(b);
        pos = len;
        floor_wa = base & ~uintptr_t(3);
        cur_wa = (base + (len ? len - 1 : 0)) & ~uintptr_t(3);
        cur = len ? *reinterpret_cast<const uint32_t*>(cur_wa) : 0u;
        nxt = (len && cur_wa > floor_wa) ? *reinterpret_cast<const uint32_t*>(cur_wa - 4) : 0u;
    }
    __device__ __forceinline__ uint32_t pop() {  // requires pos > 0
        --pos;
        const uintptr_t a = base + pos;
        const uintptr_t wa = a & ~uintptr_t(3);
        if (wa != cur_wa) {
            cur = nxt;
            cur_wa = wa;
            nxt = wa > floor_wa ? *reinterpret_cast<const uint32_t*>(wa - 4) : 0u;
        }
        return (cur >> (8 * (a & 3))) & 0xffu;
    }
};

// ------------------------------------------------------------------ launch helpers

inline hipStream_t pick(ans_gpu_table* gt, void* stream) {
    return stream ? static_cast<hipStream_t>(stream) : gt->g->stream;
}

inline unsigned grid_for(uint64_t lanes) { return static_cast<unsigned>((lanes + kBlock - 1) / kBlock); }

}  // namespace
