// ans_kernels.hip — MI355X (gfx950) rANS encode / decode of independent chunks.
//
// One lane owns one chunk = one reference Message (Message::zeros(), src/ans.rs:292)
// coded with IID<Categorical> (src/codec.rs:415-424) through the blanket
// Distribution push/pop (src/ans.rs:96-116) and flattened (src/ans.rs:255-260).
// The bytes a lane writes are exactly that message's flattened tail.
//
// Layout in HBM:
//   symbols  : the caller's array, chunk j = [j*L, min(n, (j+1)*L))
//   slots    : chunk j's stream at slots + j*slot_cap (slot_cap = worst case, 16-B multiple)
//   lens     : u32 per chunk
//   table    : DevSym[nsym+1] (+ u16 icdf buckets), staged into LDS when it fits.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "ans_fast.hpp"
#include "ans_table.hpp"

using namespace shuffle_coding;

struct ans_gpu {
    int device;
    hipStream_t stream;
};

struct ans_gpu_table {
    ans_gpu* g;
    DevTable t;
    void* d_mem;
    uint32_t lds_bytes;  // 0 = table read from global memory (L2-resident)
    FastTable ft;        // throughput path (ans_fast.hpp) when ft.usable
    void* d_fast;
};

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

// ------------------------------------------------------------------ kernels

// Encode: lane = chunk; symbols consumed last -> first (IID::push, src/codec.rs:417).
template <typename Sym, bool kLds, bool kFast>
__global__ __launch_bounds__(kBlock) void k_encode(DevTable t, const Sym* __restrict__ syms, uint64_t n,
                                                   uint64_t chunk_len, uint64_t c_first, uint64_t nchunks,
                                                   uint8_t* __restrict__ slots,
                                                   uint64_t slot_cap, uint32_t* __restrict__ lens,
                                                   uint32_t* __restrict__ status) {
    extern __shared__ __align__(16) unsigned char lds[];
    const DevSym* rows = t.sym;
    if constexpr (kLds) {
        stage_table<false>(t, lds);
        rows = reinterpret_cast<const DevSym*>(lds);
    }
    const uint64_t c = c_first + static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    const uint64_t a = c * chunk_len;
    const uint64_t b = min(a + chunk_len, n);
    ByteSink sink{slots + c * slot_cap, slot_cap, 0, 0, 0, false};
    uint64_t head = kMaxMinHead;  // Message::zeros()
    const uint64_t norm = t.norm, K = t.K;
    for (uint64_t k = b; k > a;) {
        --k;
        const uint32_t x = static_cast<uint32_t>(syms[k]);
        if (x >= t.nsym) { raise_status(status, ANS_E_SYMBOL); lens[c] = 0; return; }
        const DevSym e = rows[x];
        if (e.mass == 0) { raise_status(status, ANS_E_ZERO_MASS); lens[c] = 0; return; }
        // renorm(p * K) (src/ans.rs:100): renorm_up never fires here because the head never
        // drops below norm*K >= p*K after a push; renorm_down emits the low bytes.
        const uint64_t pK = static_cast<uint64_t>(e.mass) * K;
        while ((head >> 8) >= pK) {
            sink.put(static_cast<uint32_t>(head) & 0xffu);
            head >>= 8;
        }
        // q = head / p, r = head % p (src/ans.rs:101-102)
        uint64_t q, r;
        if constexpr (kFast) {
            q = quot_estimate(head, e.rcp);
            const int32_t rr = static_cast<int32_t>(static_cast<uint32_t>(head) - static_cast<uint32_t>(q) * e.mass);
            if (rr < 0) { q -= 1; r = static_cast<uint32_t>(rr) + e.mass; }
            else r = static_cast<uint32_t>(rr);
        } else {
            q = head / e.mass;
            r = head % e.mass;
        }
        head = q * norm + (static_cast<uint64_t>(e.cum) + r);  // src/ans.rs:103-104
    }
    // flatten (src/ans.rs:255-260): renorm_down(1), then the last head byte.
    while ((head >> 8) >= 1) {
        sink.put(static_cast<uint32_t>(head) & 0xffu);
        head >>= 8;
    }
    sink.put(static_cast<uint32_t>(head) & 0xffu);
    const uint64_t len = sink.finish();
    if (sink.overflow) raise_status(status, ANS_E_LEN);
    lens[c] = static_cast<uint32_t>(len);
}

// Decode: lane = chunk; Message::unflatten (head = 0) then len pops, symbols first -> last
// (IID::pop, src/codec.rs:423), then the reference's round-trip check (src/ans.rs:56).
template <typename Sym, bool kLds, bool kFast>
__global__ __launch_bounds__(kBlock) void k_decode(DevTable t, const uint8_t* __restrict__ in,
                                                   const uint64_t* __restrict__ offsets, uint64_t slot_cap,
                                                   const uint32_t* __restrict__ lens, uint64_t n, uint64_t chunk_len,
                                                   uint64_t c_first, uint64_t nchunks, int gen_kind, Sym* __restrict__ out,
                                                   uint32_t* __restrict__ status) {
    extern __shared__ __align__(16) unsigned char lds[];
    const DevSym* rows = t.sym;
    const uint16_t* bucket = t.bucket;
    if constexpr (kLds) {
        stage_table<true>(t, lds);
        rows = reinterpret_cast<const DevSym*>(lds);
        bucket = reinterpret_cast<const uint16_t*>(lds + sizeof(DevSym) * (t.nsym + 1));
    }
    const uint64_t c = c_first + static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    const uint64_t a = c * chunk_len;
    const uint64_t b = min(a + chunk_len, n);
    ByteSource src;
    src.init(in + (offsets ? offsets[c] : c * slot_cap), lens[c]);
    uint64_t head = 0;  // Message::unflatten
    uint32_t generated = 0;
    const uint64_t L = t.L;
    const uint32_t norm = t.norm;
    for (uint64_t k = a; k < b; ++k) {
        // renorm(norm * K) (src/ans.rs:109): renorm_up pulls tail bytes; renorm_down cannot
        // fire (after a pop head < p*256K <= 256*L).
        while (head < L) {
            uint32_t byte = 0;
            if (src.pos) byte = src.pop();
            else {
                ++generated;  // TailGenerator: Zeros -> 0, Empty -> panic (src/ans.rs:140-145)
                if (gen_kind == ANS_GEN_EMPTY) { raise_status(status, ANS_E_EXHAUSTED); return; }
            }
            head = (head << 8) | byte;
        }
        uint64_t q;
        uint32_t cf;
        if constexpr (kFast) {
            q = quot_estimate(head, t.rcp_norm);
            const int32_t ii = static_cast<int32_t>(static_cast<uint32_t>(head) - static_cast<uint32_t>(q) * norm);
            if (ii < 0) { q -= 1; cf = static_cast<uint32_t>(ii) + norm; }
            else cf = static_cast<uint32_t>(ii);
        } else {
            q = head / norm;
            cf = static_cast<uint32_t>(head % norm);
        }
        const uint32_t s = icdf(rows, bucket, t.shift, cf);  // src/codec.rs:65-68
        const DevSym e = rows[s];
        head = q * e.mass + (cf - e.cum);  // src/ans.rs:113-114
        out[k] = static_cast<Sym>(s);
    }
    // assert_eq!(initial, m) with initial = Message::zeros() (src/ans.rs:56, 302-310).
    while (head < kMaxMinHead) {
        uint32_t byte = 0;
        if (src.pos) byte = src.pop();
        else ++generated;
        head = (head << 8) | byte;
    }
    if (head != kMaxMinHead || src.pos != 0 || generated != 0) raise_status(status, ANS_E_MISMATCH);
}

// Counter-based synthetic iid symbols.
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <typename Sym, bool kLds>
__global__ __launch_bounds__(kBlock) void k_gen_iid(DevTable t, uint64_t seed, uint64_t start, uint64_t n,
                                                    Sym* __restrict__ out) {
    extern __shared__ __align__(16) unsigned char lds[];
    const DevSym* rows = t.sym;
    const uint16_t* bucket = t.bucket;
    if constexpr (kLds) {
        stage_table<true>(t, lds);
        rows = reinterpret_cast<const DevSym*>(lds);
        bucket = reinterpret_cast<const uint16_t*>(lds + sizeof(DevSym) * (t.nsym + 1));
    }
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t r = splitmix64((seed << 48) ^ (start + i));
        const uint32_t cf = static_cast<uint32_t>(__umul64hi(r, t.norm));
        out[i] = static_cast<Sym>(icdf(rows, bucket, t.shift, cf));
    }
}

// One wave per chunk copies its slot into the dense container.
__global__ __launch_bounds__(kBlock) void k_compact(const uint8_t* __restrict__ slots, uint64_t slot_cap,
                                                    const uint32_t* __restrict__ lens,
                                                    const uint64_t* __restrict__ offsets, uint64_t nchunks,
                                                    uint8_t* __restrict__ out) {
    const uint64_t c = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (c >= nchunks) return;
    const uint8_t* s = slots + c * slot_cap;
    uint8_t* d = out + offsets[c];
    for (uint32_t k = lane; k < lens[c]; k += 64) d[k] = s[k];
}

// One wave per chunk copies a dense-container stream into its slot (the inverse of k_compact).
__global__ __launch_bounds__(kBlock) void k_expand(const uint8_t* __restrict__ in, const uint64_t* __restrict__ offsets,
                                                   const uint32_t* __restrict__ lens, uint64_t nchunks,
                                                   uint8_t* __restrict__ slots, uint64_t slot_cap) {
    const uint64_t c = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (c >= nchunks) return;
    const uint8_t* s = in + offsets[c];
    uint8_t* d = slots + c * slot_cap;
    for (uint32_t k = lane; k < lens[c]; k += 64) d[k] = s[k];
}

// ------------------------------------------------------------------ launch helpers

inline hipStream_t pick(ans_gpu_table* gt, void* stream) {
    return stream ? static_cast<hipStream_t>(stream) : gt->g->stream;
}

inline unsigned grid_for(uint64_t lanes) { return static_cast<unsigned>((lanes + kBlock - 1) / kBlock); }

// Full chunks whose symbols tile into 16-byte units go to the fast kernel when the table
// allows it; everything else (ragged last chunk, odd chunk lengths, other tables) to the
// generic kernel.  Both write the same slot layout and identical bytes.
template <typename Sym>
uint64_t fast_chunks(const ans_gpu_table* gt, uint64_t n, uint64_t chunk_len, bool decode) {
    if (!gt->ft.usable || (chunk_len * sizeof(Sym)) % fast::kGroupBytes != 0) return 0;
    if (decode ? !gt->ft.dec_usable : (sizeof(Sym) == 1 && gt->ft.enc_global)) return 0;
    return n / chunk_len;
}

template <typename Sym>
int launch_encode(ans_gpu_table* gt, const void* d_syms, uint64_t n, uint64_t chunk_len, uint8_t* d_slots,
                  uint64_t slot_cap, uint32_t* d_lens, uint32_t* d_status, hipStream_t s) {
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    if (nchunks == 0) return ANS_OK;
    const DevTable& t = gt->t;
    const Sym* syms = static_cast<const Sym*>(d_syms);
    const uint64_t nfull = fast_chunks<Sym>(gt, n, chunk_len, false);
    if (nfull) {
        const FastTable& ft = gt->ft;
        const unsigned grid = static_cast<unsigned>((nfull + fast::kBlock - 1) / fast::kBlock);
        const size_t lds = ft.enc_lds_bytes + sizeof(uint32_t) * fast::kRingDwords * fast::kBlock;
        const bool k32 = ft.K < (1ull << 32);
#define ENC(KM, K32, G) fast::k_encode<Sym, KM, K32, G><<<grid, fast::kBlock, lds, s>>>(ft, syms, chunk_len, nfull, d_slots, slot_cap, d_lens, d_status)
#define ENC_KMAX(G)                                                   \
        switch (ft.kmax) {                                            \
        case 1:                                                       \
        case 2: if (k32) ENC(2, true, G); else ENC(2, false, G); break; \
        case 3: if (k32) ENC(3, true, G); else ENC(3, false, G); break; \
        default: if (k32) ENC(4, true, G); else ENC(4, false, G); break; \
        }
        if constexpr (sizeof(Sym) > 1) {
            if (ft.enc_global) {
                ENC_KMAX(true)
            } else {
                ENC_KMAX(false)
            }
        } else {
            ENC_KMAX(false)
        }
#undef ENC_KMAX
#undef ENC
        HIP_TRY(hipGetLastError());
    }
    if (nfull == nchunks) return ANS_OK;
    const unsigned grid = grid_for(nchunks - nfull);
    const size_t lds = gt->lds_bytes ? sizeof(DevSym) * (t.nsym + 1) : 0;
    if (gt->lds_bytes && t.fast)
        k_encode<Sym, true, true><<<grid, kBlock, lds, s>>>(t, syms, n, chunk_len, nfull, nchunks, d_slots, slot_cap, d_lens, d_status);
    else if (gt->lds_bytes)
        k_encode<Sym, true, false><<<grid, kBlock, lds, s>>>(t, syms, n, chunk_len, nfull, nchunks, d_slots, slot_cap, d_lens, d_status);
    else if (t.fast)
        k_encode<Sym, false, true><<<grid, kBlock, 0, s>>>(t, syms, n, chunk_len, nfull, nchunks, d_slots, slot_cap, d_lens, d_status);
    else
        k_encode<Sym, false, false><<<grid, kBlock, 0, s>>>(t, syms, n, chunk_len, nfull, nchunks, d_slots, slot_cap, d_lens, d_status);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
}

template <typename Sym>
int launch_decode(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap,
                  const uint32_t* d_lens, uint64_t n, uint64_t chunk_len, int gen_kind, void* d_syms,
                  uint32_t* d_status, hipStream_t s) {
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    if (nchunks == 0) return ANS_OK;
    const DevTable& t = gt->t;
    const FastTable& ft = gt->ft;
    Sym* out = static_cast<Sym*>(d_syms);
    // the fast kernels read the encoder's 64-byte-aligned slot layout only
    const bool slots = d_offsets == nullptr && slot_cap % 64 == 0;
    const bool lds_table = slots && fast_chunks<Sym>(gt, n, chunk_len, true) > 0;
    const bool global_table = slots && sizeof(Sym) > 1 && ft.usable && ft.dec_global &&
                              (chunk_len * sizeof(Sym)) % fast::kGroupBytes == 0;
    const uint64_t nfull = (lds_table || global_table) ? n / chunk_len : 0;
    if (nfull) {
        const unsigned grid = static_cast<unsigned>((nfull + fast::kBlock - 1) / fast::kBlock);
        constexpr int U = 16 / sizeof(Sym);
        if (global_table) {
            if constexpr (sizeof(Sym) > 1)
                fast::k_decode_g<Sym><<<grid, fast::kBlock, fast::kDecGRingBytes, s>>>(ft, d_in, slot_cap, d_lens, chunk_len, nfull, gen_kind, out, d_status);
        } else {
            const size_t lds = fast::kDecTableBytes + fast::kDecRingBytes;
#define DEC(SPP, FAR) fast::k_decode<Sym, SPP, FAR><<<grid, fast::kBlock, lds, s>>>(ft, d_in, slot_cap, d_lens, chunk_len, nfull, gen_kind, out, d_status)
            if (U * ft.kmax > 60) {
                if (ft.dec_far) DEC(U / 2, true); else DEC(U / 2, false);
            } else {
                if (ft.dec_far) DEC(U, true); else DEC(U, false);
            }
#undef DEC
        }
        HIP_TRY(hipGetLastError());
    }
    if (nfull == nchunks) return ANS_OK;
    const unsigned grid = grid_for(nchunks - nfull);
    const size_t lds = gt->lds_bytes;
    if (gt->lds_bytes && t.fast)
        k_decode<Sym, true, true><<<grid, kBlock, lds, s>>>(t, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, nfull, nchunks, gen_kind, out, d_status);
    else if (gt->lds_bytes)
        k_decode<Sym, true, false><<<grid, kBlock, lds, s>>>(t, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, nfull, nchunks, gen_kind, out, d_status);
    else if (t.fast)
        k_decode<Sym, false, true><<<grid, kBlock, 0, s>>>(t, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, nfull, nchunks, gen_kind, out, d_status);
    else
        k_decode<Sym, false, false><<<grid, kBlock, 0, s>>>(t, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, nfull, nchunks, gen_kind, out, d_status);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
}

template <typename Sym>
int launch_gen(ans_gpu_table* gt, uint64_t seed, uint64_t start, uint64_t n, void* d_syms, hipStream_t s) {
    if (n == 0) return ANS_OK;
    const uint64_t want = grid_for(n);
    const unsigned grid = static_cast<unsigned>(want < 8192 ? want : 8192);
    if (gt->lds_bytes)
        k_gen_iid<Sym, true><<<grid, kBlock, gt->lds_bytes, s>>>(gt->t, seed, start, n, static_cast<Sym*>(d_syms));
    else
        k_gen_iid<Sym, false><<<grid, kBlock, 0, s>>>(gt->t, seed, start, n, static_cast<Sym*>(d_syms));
    HIP_TRY(hipGetLastError());
    return ANS_OK;
}

bool valid_width(int w) { return w == 1 || w == 2 || w == 4; }

int lowest_status(uint32_t bits) {
    for (int k = 1; k < 32; ++k)
        if (bits & (1u << k)) return k;
    return ANS_OK;
}

// Device buffer that frees itself (host API convenience only; never in a timed path).
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 16); }
};

// Derives the fast-path tables (ans_table.hpp FastTable) when the table qualifies:
// 2^16 <= norm <= 2^31 (f64 quotient estimate) and nsym <= 65536.  Up to 256
// symbols the rows and decode buckets are staged in LDS; above, the encoder reads its rows
// from global memory and decoding uses the generic kernel.
int build_fast_table(ans_gpu_table* gt, const Categorical& cat) {
    const DevTable& t = gt->t;
    FastTable ft{};
    if (!t.fast || t.nsym > 65536) {
        gt->ft = ft;
        return ANS_OK;
    }
    using u128 = unsigned __int128;
    const uint32_t nsym = t.nsym;
    std::vector<EncRow> enc(nsym + 1);
    uint32_t kmax = 1;
    for (uint32_t s = 0; s <= nsym; ++s) {
        const uint64_t m = s < nsym ? cat.masses[s] : 0;
        enc[s] = EncRow{m ? 1.0 / static_cast<double>(m) : 0.0, static_cast<uint32_t>(m),
                        s < nsym ? static_cast<uint32_t>(cat.cummasses[s]) : t.norm};
        if (!m) continue;
        const u128 pK = static_cast<u128>(m) * t.K;
        for (uint32_t j = 1; j <= 4; ++j)  // can a push emit j bytes? (head < 2^64 <= p*K*2^8j otherwise)
            if ((pK << (8 * j)) < (static_cast<u128>(1) << 64) && j > kmax) kmax = j;
    }
    ft.enc_global = nsym > 256;
    ft.dec_usable = nsym <= 256;
    // decode buckets: the finest power-of-two width whose table fits fast::kDecTableBytes in
    // LDS (with the cdf table); for large alphabets, at most 2^16 buckets in global memory
    uint32_t shift = 0;
    const size_t cum_bytes = sizeof(uint32_t) * (nsym + 5);
    static const uint32_t g_bits = [] {  // experiment knob: global bucket table size
        const char* e = getenv("ANS_DECG_BUCKET_BITS");
        return e ? static_cast<uint32_t>(atoi(e)) : 16u;
    }();
    const uint64_t max_buckets = ft.dec_usable ? (fast::kDecTableBytes - cum_bytes) / sizeof(DecBucket) : (1ull << g_bits);
    while (((static_cast<uint64_t>(t.norm) - 1) >> shift) + 1 > max_buckets) ++shift;
    const uint32_t nb = static_cast<uint32_t>(((static_cast<uint64_t>(t.norm) - 1) >> shift) + 1);
    std::vector<uint32_t> cum(nsym + 6, t.norm);
    for (uint32_t s = 0; s < nsym; ++s) cum[s] = static_cast<uint32_t>(cat.cummasses[s]);
    std::vector<DecBucket> dec(ft.dec_usable ? nb : 0);
    std::vector<DecBucketG> decg(ft.dec_usable ? 0 : nb);
    for (uint32_t j = 0; j < nb; ++j) {
        const uint32_t s0 = static_cast<uint32_t>(cat.icdf(static_cast<uint64_t>(j) << shift).first);
        if (ft.dec_usable) {
            DecBucket& d = dec[j];
            for (int i = 0; i < 5; ++i) d.c[i] = cum[s0 + i];
            d.s0 = s0;
            // every cf of the bucket below cdf(s0 + 4)?  (the last bucket ends at norm)
            const uint64_t end = std::min<uint64_t>(t.norm, (static_cast<uint64_t>(j) + 1) << shift);
            if (d.c[4] < end) ft.dec_far = 1;
        } else {
            DecBucketG& d = decg[j];
            for (int i = 0; i < 6; ++i) d.c[i] = cum[s0 + i];
            d.s0 = s0;
            d.pad = 0;
        }
    }
    ft.dec_global = !ft.dec_usable;
    ft.nsym = nsym;
    ft.enc_rows = nsym + 1;
    ft.dec_buckets = nb;
    ft.dec_shift = shift;
    ft.norm = t.norm;
    ft.enc_lds_bytes = fast::kEncLdsBytes;  // nsym + 1 <= 257 rows, split (ans_fast.hpp)
    ft.dec_cum_off = static_cast<uint32_t>((sizeof(DecBucket) * dec.size() + 15) & ~size_t(15));
    ft.dec_lds_bytes = static_cast<uint32_t>((ft.dec_cum_off + cum_bytes + 15) & ~size_t(15));
    ft.kmax = kmax;
    ft.K = t.K;
    ft.L = t.L;
    ft.rcp_norm = t.rcp_norm;
    const size_t enc_b = sizeof(EncRow) * enc.size(), dec_b = sizeof(DecBucket) * dec.size();
    const size_t decg_b = sizeof(DecBucketG) * decg.size();
    const size_t o_dec = (enc_b + 255) & ~size_t(255), o_cum = o_dec + ((dec_b + 255) & ~size_t(255));
    const size_t o_decg = o_cum + ((sizeof(uint32_t) * cum.size() + 255) & ~size_t(255));
    HIP_TRY(hipSetDevice(gt->g->device));
    void* mem = nullptr;
    HIP_TRY(hipMalloc(&mem, o_decg + decg_b));
    gt->d_fast = mem;
    char* base = static_cast<char*>(mem);
    HIP_TRY(hipMemcpy(base, enc.data(), enc_b, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(base + o_dec, dec.data(), dec_b, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(base + o_cum, cum.data(), sizeof(uint32_t) * cum.size(), hipMemcpyHostToDevice));
    if (decg_b) HIP_TRY(hipMemcpy(base + o_decg, decg.data(), decg_b, hipMemcpyHostToDevice));
    ft.dbkt_g = reinterpret_cast<const DecBucketG*>(base + o_decg);
    ft.enc = reinterpret_cast<const EncRow*>(base);
    ft.dbkt = reinterpret_cast<const DecBucket*>(base + o_dec);
    ft.cum = reinterpret_cast<const uint32_t*>(base + o_cum);
    ft.usable = 1;
    gt->ft = ft;
    return ANS_OK;
}

}  // namespace

// ====================================================================== C ABI (GPU part)
extern "C" {

int ans_gpu_device_count(int* count) {
    if (!count) return ANS_E_ARG;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return ANS_OK;
}

int ans_gpu_create(int device, ans_gpu** out) {
    if (!out) return ANS_E_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return ANS_E_DEVICE;
    HIP_TRY(hipSetDevice(device));
    auto* g = new (std::nothrow) ans_gpu{device, nullptr};
    if (!g) return ANS_E_ALLOC;
    if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
        delete g;
        return ANS_E_DEVICE;
    }
    *out = g;
    return ANS_OK;
}

void ans_gpu_free(ans_gpu* g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    (void)hipStreamDestroy(g->stream);
    delete g;
}

int ans_gpu_table_create(ans_gpu* g, const ans_table* tab, ans_gpu_table** out) {
    if (!g || !tab || !out) return ANS_E_ARG;
    *out = nullptr;
    const Categorical& cat = tab->cat;
    const uint64_t nsym = cat.masses.size();
    if (nsym == 0 || nsym > 65536) return ANS_E_NORM_RANGE;
    if (cat.norm() == 0 || cat.norm() >= (1ull << 32)) return ANS_E_NORM_RANGE;
    DevTable t{};
    t.nsym = static_cast<uint32_t>(nsym);
    t.norm = static_cast<uint32_t>(cat.norm());
    t.K = kMaxMinHead / t.norm;
    t.L = static_cast<uint64_t>(t.norm) * t.K;
    t.rcp_norm = 1.0 / static_cast<double>(t.norm);
    t.fast = (t.norm >= (1u << 16) && t.norm <= (1u << 31)) ? 1u : 0u;
    std::vector<DevSym> rows(nsym + 1);
    uint32_t pmin = 0xffffffffu;
    for (uint64_t s = 0; s < nsym; ++s) {
        const uint32_t m = static_cast<uint32_t>(cat.masses[s]);
        rows[s] = DevSym{m, static_cast<uint32_t>(cat.cummasses[s]), m ? 1.0 / static_cast<double>(m) : 0.0};
        if (m && m < pmin) pmin = m;
    }
    rows[nsym] = DevSym{0, t.norm, 0.0};
    t.pmin = pmin;
    // icdf buckets: width 2^shift so that ceil(norm / 2^shift) <= 2^kBucketBits.
    uint32_t bits = 0;
    while (bits < 32 && (1ull << bits) < t.norm) ++bits;  // 2^bits >= norm
    t.shift = bits > kBucketBits ? bits - kBucketBits : 0;
    t.nbucket = static_cast<uint32_t>((static_cast<uint64_t>(t.norm) + (1ull << t.shift) - 1) >> t.shift);
    std::vector<uint16_t> buckets(t.nbucket);
    for (uint32_t j = 0; j < t.nbucket; ++j)
        buckets[j] = static_cast<uint16_t>(cat.icdf(static_cast<uint64_t>(j) << t.shift).first);
    const size_t rows_bytes = sizeof(DevSym) * rows.size();
    const size_t bucket_bytes = sizeof(uint16_t) * buckets.size();
    HIP_TRY(hipSetDevice(g->device));
    void* mem = nullptr;
    HIP_TRY(hipMalloc(&mem, rows_bytes + bucket_bytes + 16));
    HIP_TRY(hipMemcpy(mem, rows.data(), rows_bytes, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(static_cast<char*>(mem) + rows_bytes, buckets.data(), bucket_bytes, hipMemcpyHostToDevice));
    t.sym = static_cast<const DevSym*>(mem);
    t.bucket = reinterpret_cast<const uint16_t*>(static_cast<char*>(mem) + rows_bytes);
    auto* gt = new (std::nothrow) ans_gpu_table{g, t, mem, 0, FastTable{}, nullptr};
    if (!gt) { (void)hipFree(mem); return ANS_E_ALLOC; }
    if (rows_bytes + bucket_bytes <= kLdsTableLimit) gt->lds_bytes = static_cast<uint32_t>(rows_bytes + bucket_bytes);
    const int rc = build_fast_table(gt, cat);
    if (rc) {
        ans_gpu_table_free(gt);
        return rc;
    }
    *out = gt;
    return ANS_OK;
}

void ans_gpu_table_free(ans_gpu_table* gt) {
    if (!gt) return;
    (void)hipSetDevice(gt->g->device);
    (void)hipFree(gt->d_mem);
    if (gt->d_fast) (void)hipFree(gt->d_fast);
    delete gt;
}

int ans_gpu_slot_capacity(const ans_gpu_table* gt, uint64_t chunk_len, uint64_t* slot_cap) {
    if (!gt || !slot_cap) return ANS_E_ARG;
    // Bytes of one flattened chunk <= (sum_i log2(norm/p_i) + 1 + L*log2(1+1/K)) / 8 + 8
    // (virtual-bits argument); take every p_i = pmin, plus margin.
    const double per_sym = std::log2(static_cast<double>(gt->t.norm) / static_cast<double>(gt->t.pmin)) +
                           2.0 / static_cast<double>(gt->t.K) + 1e-6;
    const double bytes = (static_cast<double>(chunk_len) * per_sym + 2.0) / 8.0 + 9.0;
    // + one page of slack: the fast encoder writes whole 64-byte pages (ans_fast.hpp)
    const uint64_t cap = static_cast<uint64_t>(std::ceil(bytes)) + 8 + 64;
    *slot_cap = (cap + 127) & ~uint64_t(127);
    return ANS_OK;
}

int ans_dev_encode_chunks(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                          uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens, uint32_t* d_status, void* stream) {
    if (!gt || !d_status || !valid_width(sym_bytes) || chunk_len == 0 || (slot_cap & 15)) return ANS_E_ARG;
    if (n && (!d_syms || !d_slots || !d_lens)) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = pick(gt, stream);
    switch (sym_bytes) {
    case 1: return launch_encode<uint8_t>(gt, d_syms, n, chunk_len, d_slots, slot_cap, d_lens, d_status, s);
    case 2: return launch_encode<uint16_t>(gt, d_syms, n, chunk_len, d_slots, slot_cap, d_lens, d_status, s);
    default: return launch_encode<uint32_t>(gt, d_syms, n, chunk_len, d_slots, slot_cap, d_lens, d_status, s);
    }
}

int ans_dev_decode_chunks(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap,
                          const uint32_t* d_lens, uint64_t n, uint64_t chunk_len, int gen_kind, void* d_syms,
                          int sym_bytes, uint32_t* d_status, void* stream) {
    if (!gt || !d_status || !valid_width(sym_bytes) || chunk_len == 0) return ANS_E_ARG;
    if (gen_kind != ANS_GEN_ZEROS && gen_kind != ANS_GEN_EMPTY) return ANS_E_ARG;
    if (n && (!d_in || !d_lens || !d_syms)) return ANS_E_ARG;
    if (sym_bytes == 1 && gt->t.nsym > 256) return ANS_E_ARG;
    if (sym_bytes == 2 && gt->t.nsym > 65536) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = pick(gt, stream);
    switch (sym_bytes) {
    case 1: return launch_decode<uint8_t>(gt, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, gen_kind, d_syms, d_status, s);
    case 2: return launch_decode<uint16_t>(gt, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, gen_kind, d_syms, d_status, s);
    default: return launch_decode<uint32_t>(gt, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, gen_kind, d_syms, d_status, s);
    }
}

int ans_dev_gen_iid(ans_gpu_table* gt, uint64_t seed, uint64_t start, uint64_t n, void* d_syms, int sym_bytes,
                    void* stream) {
    if (!gt || !valid_width(sym_bytes) || (n && !d_syms)) return ANS_E_ARG;
    if (sym_bytes == 1 && gt->t.nsym > 256) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = pick(gt, stream);
    switch (sym_bytes) {
    case 1: return launch_gen<uint8_t>(gt, seed, start, n, d_syms, s);
    case 2: return launch_gen<uint16_t>(gt, seed, start, n, d_syms, s);
    default: return launch_gen<uint32_t>(gt, seed, start, n, d_syms, s);
    }
}

int ans_dev_compact(ans_gpu* g, const uint8_t* d_slots, uint64_t slot_cap, const uint32_t* d_lens,
                    const uint64_t* d_offsets, uint64_t nchunks, uint8_t* d_out, void* stream) {
    if (!g) return ANS_E_ARG;
    if (nchunks == 0) return ANS_OK;
    HIP_TRY(hipSetDevice(g->device));
    const hipStream_t s = stream ? static_cast<hipStream_t>(stream) : g->stream;
    k_compact<<<grid_for(nchunks * 64), kBlock, 0, s>>>(d_slots, slot_cap, d_lens, d_offsets, nchunks, d_out);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
}

int ans_dev_status(ans_gpu* g, const uint32_t* d_status, void* stream, int* status) {
    if (!g || !d_status || !status) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(g->device));
    const hipStream_t s = stream ? static_cast<hipStream_t>(stream) : g->stream;
    uint32_t bits = 0;
    HIP_TRY(hipMemcpyAsync(&bits, d_status, sizeof(bits), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *status = lowest_status(bits);
    return ANS_OK;
}

int ans_gpu_encode_chunks(ans_gpu_table* gt, const void* syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                          uint8_t* out, uint64_t out_cap, uint64_t* offsets, uint64_t* lens, uint64_t* total) {
    if (!gt || !valid_width(sym_bytes) || chunk_len == 0 || !total) return ANS_E_ARG;
    if (n && !syms) return ANS_E_ARG;
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    if (out && nchunks && (!offsets || !lens)) return ANS_E_ARG;
    uint64_t slot_cap = 0;
    ans_gpu_slot_capacity(gt, chunk_len, &slot_cap);
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = gt->g->stream;
    DevBuf d_syms, d_slots, d_lens, d_status, d_offsets, d_out;
    HIP_TRY(d_syms.alloc(n * sym_bytes));
    HIP_TRY(d_slots.alloc(nchunks * slot_cap));
    HIP_TRY(d_lens.alloc(nchunks * sizeof(uint32_t)));
    HIP_TRY(d_status.alloc(sizeof(uint32_t)));
    HIP_TRY(hipMemcpyAsync(d_syms.p, syms, n * sym_bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(d_status.p, 0, sizeof(uint32_t), s));
    int rc = ans_dev_encode_chunks(gt, d_syms.p, sym_bytes, n, chunk_len, static_cast<uint8_t*>(d_slots.p), slot_cap,
                                   static_cast<uint32_t*>(d_lens.p), static_cast<uint32_t*>(d_status.p), s);
    if (rc) return rc;
    int st = 0;
    rc = ans_dev_status(gt->g, static_cast<uint32_t*>(d_status.p), s, &st);
    if (rc) return rc;
    if (st) return st;
    std::vector<uint32_t> hl(nchunks);
    HIP_TRY(hipMemcpy(hl.data(), d_lens.p, nchunks * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::vector<uint64_t> off(nchunks);
    uint64_t acc = 0;
    for (uint64_t j = 0; j < nchunks; ++j) {
        off[j] = acc;
        acc += hl[j];
    }
    *total = acc;
    if (!out) return ANS_OK;
    if (out_cap < acc) return ANS_E_LEN;
    for (uint64_t j = 0; j < nchunks; ++j) {
        offsets[j] = off[j];
        lens[j] = hl[j];
    }
    if (nchunks == 0) return ANS_OK;
    HIP_TRY(d_offsets.alloc(nchunks * sizeof(uint64_t)));
    HIP_TRY(d_out.alloc(acc));
    HIP_TRY(hipMemcpyAsync(d_offsets.p, off.data(), nchunks * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    rc = ans_dev_compact(gt->g, static_cast<uint8_t*>(d_slots.p), slot_cap, static_cast<uint32_t*>(d_lens.p),
                         static_cast<uint64_t*>(d_offsets.p), nchunks, static_cast<uint8_t*>(d_out.p), s);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, d_out.p, acc, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return ANS_OK;
}

int ans_gpu_decode_chunks(ans_gpu_table* gt, const uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                          const uint64_t* lens, uint64_t n, uint64_t chunk_len, int gen_kind, void* out,
                          int sym_bytes) {
    if (!gt || !valid_width(sym_bytes) || chunk_len == 0) return ANS_E_ARG;
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    if (nchunks && (!in || !offsets || !lens || !out)) return ANS_E_ARG;
    std::vector<uint32_t> l32(nchunks);
    for (uint64_t j = 0; j < nchunks; ++j) {
        if (lens[j] > 0xffffffffull || offsets[j] > in_len || lens[j] > in_len - offsets[j]) return ANS_E_LEN;
        l32[j] = static_cast<uint32_t>(lens[j]);
    }
    // The container is expanded into the encoder's slot layout on the device, so full chunks
    // take the fast kernel; slots are widened if a (possibly corrupt) stream is longer than
    // the worst case of a valid one.
    uint64_t slot_cap = 0, max_len = 0;
    ans_gpu_slot_capacity(gt, chunk_len, &slot_cap);
    for (uint64_t j = 0; j < nchunks; ++j) max_len = std::max<uint64_t>(max_len, l32[j]);
    slot_cap = std::max<uint64_t>(slot_cap, (max_len + 64 + 127) & ~uint64_t(127));
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = gt->g->stream;
    DevBuf d_in, d_off, d_lens, d_status, d_out, d_slots;
    HIP_TRY(d_in.alloc(in_len + 16));
    HIP_TRY(d_off.alloc(nchunks * sizeof(uint64_t)));
    HIP_TRY(d_lens.alloc(nchunks * sizeof(uint32_t)));
    HIP_TRY(d_status.alloc(sizeof(uint32_t)));
    HIP_TRY(d_out.alloc(n * sym_bytes));
    HIP_TRY(d_slots.alloc(nchunks * slot_cap));
    if (in_len) HIP_TRY(hipMemcpyAsync(d_in.p, in, in_len, hipMemcpyHostToDevice, s));
    if (nchunks) {
        HIP_TRY(hipMemcpyAsync(d_off.p, offsets, nchunks * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_lens.p, l32.data(), nchunks * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        k_expand<<<grid_for(nchunks * 64), kBlock, 0, s>>>(static_cast<uint8_t*>(d_in.p), static_cast<uint64_t*>(d_off.p),
                                                           static_cast<uint32_t*>(d_lens.p), nchunks,
                                                           static_cast<uint8_t*>(d_slots.p), slot_cap);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipMemsetAsync(d_status.p, 0, sizeof(uint32_t), s));
    int rc = ans_dev_decode_chunks(gt, static_cast<uint8_t*>(d_slots.p), nullptr, slot_cap,
                                   static_cast<uint32_t*>(d_lens.p), n, chunk_len, gen_kind, d_out.p, sym_bytes,
                                   static_cast<uint32_t*>(d_status.p), s);
    if (rc) return rc;
    int st = 0;
    rc = ans_dev_status(gt->g, static_cast<uint32_t*>(d_status.p), s, &st);
    if (rc) return rc;
    if (st) return st;
    if (n) HIP_TRY(hipMemcpy(out, d_out.p, n * sym_bytes, hipMemcpyDeviceToHost));
    return ANS_OK;
}

}  // extern "C"
