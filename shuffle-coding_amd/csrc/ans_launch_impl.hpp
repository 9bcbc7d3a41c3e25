// ans_launch_impl.hpp — the bulk kernels' launchers (fixed, ragged and variable chunks, the
// generic one-lane-per-chunk kernels, synthetic symbols, sampling).  Included only by the
// per-width launch units ans_launch_{enc,dec}_u*.hip, which instantiate them explicitly.
#pragma once

#include "ans_kcommon.hpp"
#include "ans_launch.hpp"

namespace {

// ------------------------------------------------------------------ kernels

// Encode: lane = chunk; symbols consumed last -> first (IID::push, src/codec.rs:417).
template <typename Sym, bool kLds, bool kFast>
__global__ __launch_bounds__(kBlock) void k_encode(DevTable t, const Sym* __restrict__ syms, uint64_t n,
                                                   uint64_t chunk_len, const uint64_t* __restrict__ starts,
                                                   uint64_t c_first, uint64_t nchunks,
                                                   uint8_t* __restrict__ slots,
                                                   uint64_t slot_cap, uint32_t* __restrict__ lens,
                                                   uint32_t* __restrict__ status, fast::ChunkInit ini) {
    extern __shared__ __align__(16) unsigned char lds[];
    const DevSym* rows = t.sym;
    if constexpr (kLds) {
        stage_table<false>(t, lds);
        rows = reinterpret_cast<const DevSym*>(lds);
    }
    const uint64_t c = c_first + static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    // chunk c: fixed-length [c*L, min(n, (c+1)*L)), or [starts[c], starts[c+1]) (variable chunks)
    const uint64_t a = starts ? starts[c] : c * chunk_len;
    const uint64_t b = starts ? starts[c + 1] : min(a + chunk_len, n);
    ByteSink sink{slots + c * slot_cap, slot_cap, 0, 0, 0, false};
    uint64_t head = ini.head(c);  // Message::zeros() / random(seed + c)
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
    if (sink.overflow) {  // no length past the slot reaches k_compact or a decoder
        raise_status(status, ANS_E_LEN);
        lens[c] = 0;
        return;
    }
    lens[c] = static_cast<uint32_t>(len);
}

// Decode: lane = chunk; Message::unflatten (head = 0) then len pops, symbols first -> last
// (IID::pop, src/codec.rs:423), then the reference's round-trip check (src/ans.rs:56).
template <typename Sym, bool kLds, bool kFast>
__global__ __launch_bounds__(kBlock) void k_decode(DevTable t, const uint8_t* __restrict__ in,
                                                   const uint64_t* __restrict__ offsets, uint64_t slot_cap,
                                                   const uint32_t* __restrict__ lens, uint64_t n, uint64_t chunk_len,
                                                   const uint64_t* __restrict__ starts,
                                                   uint64_t c_first, uint64_t nchunks, int gen_kind, Sym* __restrict__ out,
                                                   uint32_t* __restrict__ status, fast::ChunkInit ini) {
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
    const uint64_t a = starts ? starts[c] : c * chunk_len;
    const uint64_t b = starts ? starts[c + 1] : min(a + chunk_len, n);
    // slot layout: a stream longer than its slot is foreign or corrupt (it would read past it)
    if (!offsets && lens[c] > slot_cap) { raise_status(status, ANS_E_LEN); return; }
    ByteSource src;
    src.init(in + (offsets ? offsets[c] : c * slot_cap), lens[c]);
    uint64_t head = 0;  // Message::unflatten
    uint32_t generated = 0;
    const uint64_t L = t.L;
    const uint32_t norm = t.norm;
    for (uint64_t k = a; k < b; ++k) {
        // renorm(norm * K) (src/ans.rs:109): renorm_up pulls tail bytes; renorm_down cannot
        // fire (after a pop head < p*256K <= 256*L).  A valid stream needs at most 8 pulls
        // (head >= 1 after any pop); more means zero bytes past an exhausted or corrupt
        // stream, where the loop would never end.
        for (int pulls = 0; head < L; ++pulls) {
            if (pulls == 8) { raise_status(status, ANS_E_MISMATCH); return; }
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
    // assert_eq!(initial, m) with initial = the chunk's initial message (src/ans.rs:56, 302-310).
    for (int pulls = 0; head < kMaxMinHead; ++pulls) {
        if (pulls == 8) { raise_status(status, ANS_E_MISMATCH); return; }
        uint32_t byte = 0;
        if (src.pos) byte = src.pop();
        else ++generated;
        head = (head << 8) | byte;
    }
    if (head != ini.head(c) || src.pos != 0 || generated != 0) raise_status(status, ANS_E_MISMATCH);
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

// Codec::samples (src/ans.rs:42-44) in bulk: chunk c (len = its symbol count) is
// IID::new(codec, len).pop(&mut Message::random(seed + c)) — decoding from a message whose
// tail is empty, so every renorm byte is drawn from the generator.
template <typename Sym, bool kLds, bool kFast>
__global__ __launch_bounds__(kBlock) void k_sample_iid(DevTable t, uint64_t seed, uint64_t n, uint64_t chunk_len,
                                                       uint64_t nchunks, Sym* __restrict__ out) {
    extern __shared__ __align__(16) unsigned char lds[];
    const DevSym* rows = t.sym;
    const uint16_t* bucket = t.bucket;
    if constexpr (kLds) {
        stage_table<true>(t, lds);
        rows = reinterpret_cast<const DevSym*>(lds);
        bucket = reinterpret_cast<const uint16_t*>(lds + sizeof(DevSym) * (t.nsym + 1));
    }
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    fast::Pcg64Mcg rng;
    rng.seed_from_u64(seed + c);
    uint64_t head = 1;  // Message::random (src/ans.rs:285-289): head 1, renorm_up(MAX_MIN_HEAD)
    while (head < kMaxMinHead) head = (head << 8) | rng.next_byte();
    const uint64_t L = t.L;
    const uint32_t norm = t.norm;
    auto pop = [&]() __attribute__((always_inline)) {
        while (head < L) head = (head << 8) | rng.next_byte();  // renorm (src/ans.rs:109,239-243)
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
        const uint32_t s = icdf(rows, bucket, t.shift, cf);
        const DevSym e = rows[s];
        head = q * e.mass + (cf - e.cum);
        return s;
    };
    const uint64_t a = c * chunk_len, b = min(a + chunk_len, n);
    uint64_t k = a;
    // whole 16-byte groups are packed in registers and stored at once (a lane's chunk is
    // contiguous, so per-symbol stores would touch 64 cache lines per wave instruction)
    constexpr int G = 16 / static_cast<int>(sizeof(Sym));
    if ((a * sizeof(Sym)) % 16 == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
        for (; k + G <= b; k += G) {
            uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < G; ++j) {
                const uint32_t sym = pop();
                constexpr int per = 4 / static_cast<int>(sizeof(Sym));
                w[j / per] |= sym << (8 * sizeof(Sym) * (j % per));
            }
            *reinterpret_cast<uint4*>(out + k) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
    for (; k < b; ++k) out[k] = static_cast<Sym>(pop());
}

// Full chunks whose symbols tile into 16-byte units go to the fast kernel when the table
// allows it; everything else (ragged last chunk, odd chunk lengths, other tables) to the
// generic kernel.  Both write the same slot layout and identical bytes.
// ---- staged chunks: ragged (chunk bytes not a multiple of the fast kernels' 128-B groups, e.g.
// C2's 1,563 u16 symbols) and variable-length chunks through the fast large-alphabet kernels.
// Chunk c's symbols are copied to the start of a stride of lpad symbols (lpad * w a multiple
// of 128), k_encode_w / k_decode_w run with kVar (their first-coded group partial), and decoded
// symbols are copied back.  One thread per 16-B unit of the staging buffer.
template <typename Sym>
struct ChunkSpan {  // chunk c = symbols [start(c), start(c) + len(c)) of the caller's array
    const uint64_t* starts;  // variable chunks (nchunks + 1 entries), or nullptr
    uint64_t chunk_len, n;   // fixed chunks (the last one may be short)
    __device__ __forceinline__ uint64_t start(uint64_t c) const { return starts ? starts[c] : c * chunk_len; }
    __device__ __forceinline__ uint64_t len(uint64_t c) const {
        return starts ? starts[c + 1] - starts[c] : min(chunk_len, n - c * chunk_len);
    }
};

template <typename Sym>
__global__ __launch_bounds__(kBlock) void k_stage(const Sym* __restrict__ src, ChunkSpan<Sym> span, uint64_t nchunks,
                                                  uint64_t lpad, Sym* __restrict__ stage, uint32_t* __restrict__ vlen) {
    constexpr uint32_t U = 16 / sizeof(Sym);
    const uint64_t upc = lpad / U;  // units per chunk
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= nchunks * upc) return;
    const uint64_t c = i / upc, k0 = (i % upc) * U;
    const uint64_t a = span.start(c), l = span.len(c);
    if (k0 == 0) vlen[c] = static_cast<uint32_t>(l);
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t j = 0; j < U; ++j) {
        const uint32_t v = k0 + j < l ? static_cast<uint32_t>(src[a + k0 + j]) : 0u;
        w[j / (4 / sizeof(Sym))] |= v << (8 * sizeof(Sym) * (j % (4 / sizeof(Sym))));
    }
    reinterpret_cast<uint4*>(stage)[i] = make_uint4(w[0], w[1], w[2], w[3]);
}

template <typename Sym>
__global__ __launch_bounds__(kBlock) void k_unstage(const Sym* __restrict__ stage, ChunkSpan<Sym> span,
                                                    uint64_t nchunks, uint64_t lpad, Sym* __restrict__ out) {
    constexpr uint32_t U = 16 / sizeof(Sym);
    const uint64_t upc = lpad / U;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= nchunks * upc) return;
    const uint64_t c = i / upc, k0 = (i % upc) * U;
    const uint64_t a = span.start(c), l = span.len(c);
    if (k0 >= l) return;
    const uint4 v = reinterpret_cast<const uint4*>(stage)[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t j = 0; j < U; ++j) {
        if (k0 + j < l) {
            const uint32_t x = w[j / (4 / sizeof(Sym))] >> (8 * sizeof(Sym) * (j % (4 / sizeof(Sym))));
            out[a + k0 + j] = static_cast<Sym>(x);
        }
    }
}

template <typename Sym>
__global__ __launch_bounds__(kBlock) void k_span_lens(ChunkSpan<Sym> span, uint64_t nchunks, uint32_t* __restrict__ vlen) {
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (c < nchunks) vlen[c] = static_cast<uint32_t>(span.len(c));
}

constexpr int kNotStaged = -2;

// dynamic LDS of k_encode_w: the shift table (kSa), the ring and the prefix image
inline size_t wide_enc_lds(const FastTable& ft) {
    if (!ft.enc_pack) return fast::kWideEncCum + 4 * (ft.enc_nl + 1);
    return (ft.enc_sa ? fast::kWideSaBytes : 0) + fast::kWideBBytes + fast::kEncRingBytes + (ft.enc_pack_bytes - ft.enc_pack_ooff);
}

// k_decode_w's dynamic LDS and its staged compact buckets (ft.dec_c_nlb): the 67.5-KiB ring plus
// the first buckets, up to the rest of the CU's 160 KiB (C4: 6,016 of 65,704), so one 512-lane
// workgroup fits per CU.  Measured against two workgroups per CU with the ring alone (four waves
// per SIMD where a grid has more workgroups than CUs): 2^31 u16 symbols (1,024 workgroups) decode
// in 8.55 ms staged vs 8.98 ms (profiles/r05_ab_c4_2e31_two_wg_per_cu_rejected.txt; a C4 shard,
// 256 workgroups, is the same either way): the L2 request rate, not the wave count, binds.
inline size_t wide_dec_lds(FastTable& ft, unsigned /*wgrid*/, int /*ncu*/) {
    const uint32_t nb = static_cast<uint32_t>(((static_cast<uint64_t>(ft.norm) - 1) >> ft.dec_cl_shift) + 1);
    ft.dec_c_nlb = std::min(nb, fast::kWideDecBktLds);
    return fast::kWideDecTab + 16ull * ft.dec_c_nlb;
}

// The staged route applies to the large-alphabet fast kernels (u16 / u32 symbols).
template <typename Sym>
bool staged_encode_ok(const ans_gpu_table* gt) {  // large-alphabet or LDS-row encoder
    return gt->ft.usable && ((sizeof(Sym) > 1 && gt->ft.enc_wide) || !gt->ft.enc_global);
}
template <typename Sym>
bool staged_decode_ok(const ans_gpu_table* gt) {  // large-alphabet or LDS-bucket decoder
    return gt->ft.usable && ((sizeof(Sym) > 1 && gt->ft.dec_wide) || gt->ft.dec_usable);
}

// go(integral_constant<int, table's norm range>) for the large-alphabet kernels' kNR
template <typename Go>
void with_norm_range(const FastTable& ft, Go&& go) {
    using std::integral_constant;
    if (ft.nr == fast::kNormSmall) go(integral_constant<int, fast::kNormSmall>{});
    else if (ft.nr == fast::kNormBig) go(integral_constant<int, fast::kNormBig>{});
    else go(integral_constant<int, fast::kNormStd>{});
}

template <typename Sym>
int launch_staged_encode(ans_gpu_table* gt, const Sym* syms, ChunkSpan<Sym> span, uint64_t nchunks, uint64_t lmax,
                         uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens, uint32_t* d_status, hipStream_t s,
                         fast::ChunkInit ini) {
    {
        if (!staged_encode_ok<Sym>(gt) || nchunks == 0) return kNotStaged;
        const FastTable& ft = gt->ft;
        constexpr uint64_t GS = 128 / sizeof(Sym);
        const uint64_t lpad = std::max<uint64_t>(GS, (lmax + GS - 1) / GS * GS);
        void* mem = nullptr;
        const size_t stage_b = nchunks * lpad * sizeof(Sym), vlen_o = (stage_b + 255) & ~size_t(255);
        if (hipMallocAsync(&mem, vlen_o + 4 * nchunks, s) != hipSuccess) {
            (void)hipGetLastError();  // no room to stage: the generic kernels need none
            return kNotStaged;
        }
        Sym* stage = static_cast<Sym*>(mem);
        uint32_t* vlen = reinterpret_cast<uint32_t*>(static_cast<char*>(mem) + vlen_o);
        const uint64_t units = nchunks * lpad / (16 / sizeof(Sym));
        k_stage<Sym><<<grid_for(units), kBlock, 0, s>>>(syms, span, nchunks, lpad, stage, vlen);
        const unsigned grid = static_cast<unsigned>((nchunks + fast::kBlock - 1) / fast::kBlock);
        const bool k32 = ft.K < (1ull << 32);
        const size_t wlds = wide_enc_lds(ft);
        // (u8 symbols never take the large-alphabet kernels: not instantiated for them)
        bool wide = false;
        if constexpr (sizeof(Sym) > 1) wide = ft.enc_wide;
        if (wide) {
            if constexpr (sizeof(Sym) > 1) {
#define ENCV2(K32, PK, SA, NR) fast::k_encode_w<Sym, K32, PK, SA, true, NR><<<grid, fast::kBlock, wlds, s>>>(ft, stage, lpad, nchunks, d_slots, slot_cap, d_lens, d_status, ini, vlen)
#define ENCV(K32, NR) if (ft.enc_sa) ENCV2(K32, true, true, NR); else if (ft.enc_pack) ENCV2(K32, true, false, NR); else ENCV2(K32, false, false, NR)
            if (ft.nr == fast::kNormBig) ENCV(true, fast::kNormBig);  // (K < 2^25)
            else if (k32) ENCV(true, fast::kNormStd);
            else ENCV(false, fast::kNormStd);
#undef ENCV
#undef ENCV2
            }
        } else {  // LDS rows (ans_fast.hpp k_encode, kVar)
#define ENCL(KM, K32, NR) fast::k_encode<Sym, KM, K32, false, true, NR><<<grid, fast::kBlock, fast::kEncSharedBytes, s>>>(ft, stage, lpad, nchunks, d_slots, slot_cap, d_lens, d_status, ini, vlen)
            if (ft.nr == fast::kNormSmall) {  // (kmax <= 2, K >= 2^40)
                ENCL(2, false, fast::kNormSmall);
            } else if (ft.nr == fast::kNormBig) {  // (K < 2^25)
                switch (ft.kmax) {
                case 1: case 2: ENCL(2, true, fast::kNormBig); break;
                case 3: ENCL(3, true, fast::kNormBig); break;
                default: ENCL(4, true, fast::kNormBig); break;
                }
            } else {
                switch (ft.kmax) {
                case 1: case 2: if (k32) ENCL(2, true, fast::kNormStd); else ENCL(2, false, fast::kNormStd); break;
                case 3: if (k32) ENCL(3, true, fast::kNormStd); else ENCL(3, false, fast::kNormStd); break;
                default: if (k32) ENCL(4, true, fast::kNormStd); else ENCL(4, false, fast::kNormStd); break;
                }
            }
#undef ENCL
        }
        const hipError_t err = hipGetLastError();  // free the staging buffer on every path
        HIP_TRY(hipFreeAsync(mem, s));
        HIP_TRY(err);
        return ANS_OK;
    }
}

// k_decode's template arguments for a <= 256-symbol table: only the combinations a table can
// select are instantiated.  u8 (U = 16) takes half-unit points exactly when kmax = 4, wider
// symbols never (U * 4 <= 60); the u-domain tables are built for u8 symbols' kernels only (the
// wider-symbol instantiations keep kModeRows: fewer kernels to compile); kNormSmall never pulls
// more than two bytes (kmax <= 2) and kNormBig runs without the 24-bit product.
// go(spp, mode, p24, j4, nr) receives each as a std::integral_constant.
template <typename Sym, typename Go>
void launch_lds_decode(const FastTable& ft, Go&& go) {
    using std::integral_constant;
    constexpr int U = 16 / sizeof(Sym);
    constexpr bool kHalf = U * 4 > 60;
    constexpr int kU = sizeof(Sym) == 1 ? fast::kModeU : fast::kModeRows;
    auto modes = [&](auto spp, auto p24, auto j4, auto nr) {
        if (ft.dec_far) {
            go(spp, integral_constant<int, fast::kModeFar>{}, p24, j4, nr);
            return;
        }
        if constexpr (decltype(nr)::value != fast::kNormBig) {
            if (ft.dec_u) {
                go(spp, integral_constant<int, kU>{}, p24, j4, nr);
                return;
            }
        }
        go(spp, integral_constant<int, fast::kModeRows>{}, p24, j4, nr);
    };
    auto points = [&](auto p24, auto nr) {
        if (kHalf && U * ft.kmax > 60) {  // (kmax = 4)
            if constexpr (kHalf && decltype(nr)::value != fast::kNormSmall)
                modes(integral_constant<int, U / 2>{}, p24, std::true_type{}, nr);
        } else if (kHalf || ft.kmax < 4 || decltype(nr)::value == fast::kNormSmall) {
            modes(integral_constant<int, U>{}, p24, std::false_type{}, nr);
        } else {
            if constexpr (!kHalf && decltype(nr)::value != fast::kNormSmall)
                modes(integral_constant<int, U>{}, p24, std::true_type{}, nr);
        }
    };
    if (ft.nr == fast::kNormSmall) {
        if (ft.p24) points(std::true_type{}, integral_constant<int, fast::kNormSmall>{});
        else points(std::false_type{}, integral_constant<int, fast::kNormSmall>{});
    } else if (ft.nr == fast::kNormBig) {
        points(std::false_type{}, integral_constant<int, fast::kNormBig>{});
    } else {
        if (ft.p24) points(std::true_type{}, integral_constant<int, fast::kNormStd>{});
        else points(std::false_type{}, integral_constant<int, fast::kNormStd>{});
    }
}

template <typename Sym>
int launch_staged_decode(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap,
                         const uint32_t* d_lens, ChunkSpan<Sym> span, uint64_t nchunks, uint64_t lmax, int gen_kind,
                         Sym* out, uint32_t* d_status, hipStream_t s, fast::ChunkInit ini) {
    {
        if (!staged_decode_ok<Sym>(gt) || nchunks == 0 || lmax > (1ull << 24)) return kNotStaged;
        const FastTable& ft = gt->ft;
        constexpr uint64_t GS = 128 / sizeof(Sym);
        const uint64_t lpad = std::max<uint64_t>(GS, (lmax + GS - 1) / GS * GS);
        void* mem = nullptr;
        const size_t stage_b = nchunks * lpad * sizeof(Sym), vlen_o = (stage_b + 255) & ~size_t(255);
        if (hipMallocAsync(&mem, vlen_o + 4 * nchunks, s) != hipSuccess) {
            (void)hipGetLastError();  // no room to stage: the generic kernels need none
            return kNotStaged;
        }
        Sym* stage = static_cast<Sym*>(mem);
        uint32_t* vlen = reinterpret_cast<uint32_t*>(static_cast<char*>(mem) + vlen_o);
        const uint64_t units = nchunks * lpad / (16 / sizeof(Sym));
        k_span_lens<Sym><<<grid_for(nchunks), kBlock, 0, s>>>(span, nchunks, vlen);
        bool wide = false;  // (u8 symbols never take the large-alphabet kernels: not instantiated for them)
        if constexpr (sizeof(Sym) > 1) wide = ft.dec_wide;
        if (wide) {
          if constexpr (sizeof(Sym) > 1) {
            const unsigned wgrid = static_cast<unsigned>((nchunks + fast::kWideDecLanes - 1) / fast::kWideDecLanes);
            with_norm_range(ft, [&](auto nr) {
                constexpr int NR = decltype(nr)::value;
                if (ft.dec_c) {
                    FastTable fw = ft;
                    const size_t wl = wide_dec_lds(fw, wgrid, gt->g->ncu);
                    fast::k_decode_w<Sym, true, false, true, false, NR><<<wgrid, fast::kWideDecLanes, wl, s>>>(fw, d_in, slot_cap, d_offsets, d_lens, lpad, nchunks, gen_kind, stage, d_status, ini, vlen);
                } else {
                    fast::k_decode_w<Sym, false, true, true, false, NR><<<wgrid, fast::kWideDecLanes, 160 * 1024, s>>>(ft, d_in, slot_cap, d_offsets, d_lens, lpad, nchunks, gen_kind, stage, d_status, ini, vlen);
                }
            });
          }
        } else {  // LDS buckets (ans_fast.hpp k_decode, kVar)
            const size_t lds = fast::kDecTableBytes + fast::kDecRingBytes;
            const unsigned dgrid = static_cast<unsigned>((nchunks + fast::kDecBlock - 1) / fast::kDecBlock);
#define DEC(SPP, MODE, P24, J4, NR) fast::k_decode<Sym, SPP, MODE, P24, J4, true, NR><<<dgrid, fast::kDecBlock, lds, s>>>(ft, d_in, slot_cap, d_offsets, d_lens, lpad, nchunks, gen_kind, stage, d_status, ini, vlen)
            launch_lds_decode<Sym>(ft, [&](auto spp, auto mode, auto p24, auto j4, auto nr) {
                DEC(decltype(spp)::value, decltype(mode)::value, decltype(p24)::value, decltype(j4)::value, decltype(nr)::value);
            });
#undef DEC
        }
        k_unstage<Sym><<<grid_for(units), kBlock, 0, s>>>(stage, span, nchunks, lpad, out);
        const hipError_t err = hipGetLastError();  // free the staging buffer on every path
        HIP_TRY(hipFreeAsync(mem, s));
        HIP_TRY(err);
        return ANS_OK;
    }
}

template <typename Sym>
uint64_t fast_chunks(const ans_gpu_table* gt, uint64_t n, uint64_t chunk_len, bool decode) {
    // the LDS-row encoder reads 128-B symbol groups; the decoders store 64-B symbol blocks
    const uint64_t group = (!decode && !gt->ft.enc_global) ? 128 : fast::kGroupBytes;
    if (!gt->ft.usable || (chunk_len * sizeof(Sym)) % group != 0) return 0;
    // k_decode keeps stream positions in bits (int32): streams stay below 2^27 bytes for chunks
    // of at most 2^24 symbols (4 bytes per push at most)
    if (decode && chunk_len > (1ull << 24)) return 0;
    if (decode ? !gt->ft.dec_usable : (sizeof(Sym) == 1 && gt->ft.enc_global)) return 0;
    // kNormBig large alphabets encode on k_encode_w alone (128-B symbol groups)
    if (!decode && gt->ft.enc_global && gt->ft.nr == fast::kNormBig && (chunk_len * sizeof(Sym)) % 128 != 0) return 0;
    return n / chunk_len;
}

}  // namespace

namespace shuffle_coding {
namespace launch {

template <typename Sym>
int launch_encode(ans_gpu_table* gt, const void* d_syms, uint64_t n, uint64_t chunk_len, uint8_t* d_slots,
                  uint64_t slot_cap, uint32_t* d_lens, uint32_t* d_status, hipStream_t s, fast::ChunkInit ini) {
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    if (nchunks == 0) return ANS_OK;
    const DevTable& t = gt->t;
    const Sym* syms = static_cast<const Sym*>(d_syms);
    // ragged chunks (C2): staged when the padded layout stays within staged_lmax's budget (short
    // chunks pad to 128 B each: chunk_len 1 would stage 128x the symbols)
    if ((chunk_len * sizeof(Sym)) % 128 != 0 && staged_encode_ok<Sym>(gt) &&
        staged_lmax(nchunks, chunk_len, n, sizeof(Sym)) != 0) {
        const int rc = launch_staged_encode<Sym>(gt, syms, ChunkSpan<Sym>{nullptr, chunk_len, n}, nchunks, chunk_len,
                                                 d_slots, slot_cap, d_lens, d_status, s, ini);
        if (rc != kNotStaged) return rc;
    }
    const uint64_t nfull = fast_chunks<Sym>(gt, n, chunk_len, false);
    if (nfull) {
        const FastTable& ft = gt->ft;
        const unsigned grid = static_cast<unsigned>((nfull + fast::kBlock - 1) / fast::kBlock);
        const size_t lds = fast::kEncSharedBytes;  // rows (LDS-row kernels) + ring
        const bool k32 = ft.K < (1ull << 32);
        const bool m24 = ft.pmax < (1u << 24);  // (k_encode kM24: the mass word's top byte is free)
#define ENC(KM, K32, G) do { if (!(G) && m24) fast::k_encode<Sym, KM, K32, false, false, fast::kNormStd, true><<<grid, fast::kBlock, lds, s>>>(ft, syms, chunk_len, nfull, d_slots, slot_cap, d_lens, d_status, ini); \
                             else fast::k_encode<Sym, KM, K32, G><<<grid, fast::kBlock, lds, s>>>(ft, syms, chunk_len, nfull, d_slots, slot_cap, d_lens, d_status, ini); } while (0)
#define ENCN(KM, K32, NR) fast::k_encode<Sym, KM, K32, false, false, NR><<<grid, fast::kBlock, lds, s>>>(ft, syms, chunk_len, nfull, d_slots, slot_cap, d_lens, d_status, ini)
#define ENC_KMAX(G)                                                   \
        if (ft.nr == fast::kNormSmall) {  /* (kmax <= 2, K >= 2^40) */ \
            fast::k_encode<Sym, 2, false, G, false, fast::kNormSmall><<<grid, fast::kBlock, lds, s>>>(ft, syms, chunk_len, nfull, d_slots, slot_cap, d_lens, d_status, ini); \
        } else if (!(G) && ft.nr == fast::kNormBig) {                 \
            switch (ft.kmax) {                                        \
            case 1: case 2: ENCN(2, true, fast::kNormBig); break;     \
            case 3: ENCN(3, true, fast::kNormBig); break;             \
            default: ENCN(4, true, fast::kNormBig); break;            \
            }                                                         \
        } else {                                                      \
        switch (ft.kmax) {                                            \
        case 1: case 2: if (k32) ENC(2, true, G); else ENC(2, false, G); break; \
        case 3: if (k32) ENC(3, true, G); else ENC(3, false, G); break; \
        default: if (k32) ENC(4, true, G); else ENC(4, false, G); break; \
        }                                                             \
        }
        if constexpr (sizeof(Sym) > 1) {
            if (ft.enc_wide && (chunk_len * sizeof(Sym)) % 128 == 0) {
                const size_t wlds = wide_enc_lds(ft);
#define ENCW2(K32, PK, SA, NR) fast::k_encode_w<Sym, K32, PK, SA, false, NR><<<grid, fast::kBlock, wlds, s>>>(ft, syms, chunk_len, nfull, d_slots, slot_cap, d_lens, d_status, ini)
#define ENCW(K32, NR) if (ft.enc_sa) ENCW2(K32, true, true, NR); else if (ft.enc_pack) ENCW2(K32, true, false, NR); else ENCW2(K32, false, false, NR)
                if (ft.nr == fast::kNormBig) ENCW(true, fast::kNormBig);  // (K < 2^25)
                else if (k32) ENCW(true, fast::kNormStd);
                else ENCW(false, fast::kNormStd);
#undef ENCW
#undef ENCW2
            } else if (ft.enc_global) {
                ENC_KMAX(true)
            } else {
                ENC_KMAX(false)
            }
        } else {
            ENC_KMAX(false)
        }
#undef ENC_KMAX
#undef ENCN
#undef ENC
        HIP_TRY(hipGetLastError());
    }
    if (nfull == nchunks) return ANS_OK;
    const unsigned grid = grid_for(nchunks - nfull);
    const size_t lds = gt->lds_bytes ? sizeof(DevSym) * (t.nsym + 1) : 0;
    if (gt->lds_bytes && t.fast)
        k_encode<Sym, true, true><<<grid, kBlock, lds, s>>>(t, syms, n, chunk_len, nullptr, nfull, nchunks, d_slots, slot_cap, d_lens, d_status, ini);
    else if (gt->lds_bytes)
        k_encode<Sym, true, false><<<grid, kBlock, lds, s>>>(t, syms, n, chunk_len, nullptr, nfull, nchunks, d_slots, slot_cap, d_lens, d_status, ini);
    else if (t.fast)
        k_encode<Sym, false, true><<<grid, kBlock, 0, s>>>(t, syms, n, chunk_len, nullptr, nfull, nchunks, d_slots, slot_cap, d_lens, d_status, ini);
    else
        k_encode<Sym, false, false><<<grid, kBlock, 0, s>>>(t, syms, n, chunk_len, nullptr, nfull, nchunks, d_slots, slot_cap, d_lens, d_status, ini);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
}

template <typename Sym>
int launch_decode(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap,
                  const uint32_t* d_lens, uint64_t n, uint64_t chunk_len, int gen_kind, void* d_syms,
                  uint32_t* d_status, hipStream_t s, fast::ChunkInit ini) {
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    if (nchunks == 0) return ANS_OK;
    const DevTable& t = gt->t;
    const FastTable& ft = gt->ft;
    Sym* out = static_cast<Sym*>(d_syms);
    if ((chunk_len * sizeof(Sym)) % 64 != 0 && staged_decode_ok<Sym>(gt) &&
        staged_lmax(nchunks, chunk_len, n, sizeof(Sym)) != 0) {  // ragged chunks (C2), within the budget
        const int rc = launch_staged_decode<Sym>(gt, d_in, d_offsets, slot_cap, d_lens, ChunkSpan<Sym>{nullptr, chunk_len, n},
                                                 nchunks, chunk_len, gen_kind, out, d_status, s, ini);
        if (rc != kNotStaged) return rc;
    }
    // the fast kernels read whole aligned 128-B lines around each stream, from the slot layout
    // or a dense container alike (fast::DecChain::start)
    const bool lds_table = fast_chunks<Sym>(gt, n, chunk_len, true) > 0;
    const bool global_table = sizeof(Sym) > 1 && ft.usable && ft.dec_global &&
                              (chunk_len * sizeof(Sym)) % fast::kGroupBytes == 0;
    const uint64_t nfull = (lds_table || global_table) ? n / chunk_len : 0;
    if (nfull) {
        const unsigned grid = static_cast<unsigned>((nfull + fast::kBlock - 1) / fast::kBlock);
        if (global_table) {
            if constexpr (sizeof(Sym) > 1) {
                const unsigned wgrid = static_cast<unsigned>((nfull + fast::kWideDecLanes - 1) / fast::kWideDecLanes);
                // compact buckets: no LDS prefix (C4 decode 2.45 -> 2.28 ms: the shard's 2 waves per
                // SIMD wait on an L2 round trip every step whatever the prefix covers, and the
                // prefix path's VALU sat on that chain); the first buckets staged in the LDS the
                // ring leaves (wide_dec_lds: one workgroup per CU)
                with_norm_range(ft, [&](auto nr) {
                    constexpr int NR = decltype(nr)::value;
                    if (ft.dec_wide && ft.dec_c && (chunk_len * sizeof(Sym)) % 64 == 0) {
                        FastTable fw = ft;
                        const size_t wl = wide_dec_lds(fw, wgrid, gt->g->ncu);
                        if constexpr (NR == fast::kNormStd) {
                            if (ft.p24)
                                fast::k_decode_w<Sym, true, false, false, true><<<wgrid, fast::kWideDecLanes, wl, s>>>(fw, d_in, slot_cap, d_offsets, d_lens, chunk_len, nfull, gen_kind, out, d_status, ini);
                            else
                                fast::k_decode_w<Sym, true, false><<<wgrid, fast::kWideDecLanes, wl, s>>>(fw, d_in, slot_cap, d_offsets, d_lens, chunk_len, nfull, gen_kind, out, d_status, ini);
                        } else {
                            fast::k_decode_w<Sym, true, false, false, false, NR><<<wgrid, fast::kWideDecLanes, wl, s>>>(fw, d_in, slot_cap, d_offsets, d_lens, chunk_len, nfull, gen_kind, out, d_status, ini);
                        }
                    } else if (ft.dec_wide && (chunk_len * sizeof(Sym)) % 64 == 0) {
                        fast::k_decode_w<Sym, false, true, false, false, NR><<<wgrid, fast::kWideDecLanes, 160 * 1024, s>>>(ft, d_in, slot_cap, d_offsets, d_lens, chunk_len, nfull, gen_kind, out, d_status, ini);
                    } else {
                        fast::k_decode_g<Sym, NR><<<grid, fast::kBlock, fast::kDecGRingBytes, s>>>(ft, d_in, slot_cap, d_offsets, d_lens, chunk_len, nfull, gen_kind, out, d_status, ini);
                    }
                });
            }
        } else {
            const size_t lds = fast::kDecTableBytes + fast::kDecRingBytes;
            const unsigned dgrid = static_cast<unsigned>((nfull + fast::kDecBlock - 1) / fast::kDecBlock);
#define DEC(SPP, MODE, P24, J4, NR) fast::k_decode<Sym, SPP, MODE, P24, J4, false, NR><<<dgrid, fast::kDecBlock, lds, s>>>(ft, d_in, slot_cap, d_offsets, d_lens, chunk_len, nfull, gen_kind, out, d_status, ini)
            launch_lds_decode<Sym>(ft, [&](auto spp, auto mode, auto p24, auto j4, auto nr) {
                DEC(decltype(spp)::value, decltype(mode)::value, decltype(p24)::value, decltype(j4)::value, decltype(nr)::value);
            });
#undef DEC
        }
        HIP_TRY(hipGetLastError());
    }
    if (nfull == nchunks) return ANS_OK;
    const unsigned grid = grid_for(nchunks - nfull);
    const size_t lds = gt->lds_bytes;
    if (gt->lds_bytes && t.fast)
        k_decode<Sym, true, true><<<grid, kBlock, lds, s>>>(t, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, nullptr, nfull, nchunks, gen_kind, out, d_status, ini);
    else if (gt->lds_bytes)
        k_decode<Sym, true, false><<<grid, kBlock, lds, s>>>(t, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, nullptr, nfull, nchunks, gen_kind, out, d_status, ini);
    else if (t.fast)
        k_decode<Sym, false, true><<<grid, kBlock, 0, s>>>(t, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, nullptr, nfull, nchunks, gen_kind, out, d_status, ini);
    else
        k_decode<Sym, false, false><<<grid, kBlock, 0, s>>>(t, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, nullptr, nfull, nchunks, gen_kind, out, d_status, ini);
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

// Variable-length chunks (chunk c = symbols [d_starts[c], d_starts[c+1])): generic kernels,
// one lane per chunk, slots of slot_cap bytes.
template <typename Sym>
int launch_encode_var(ans_gpu_table* gt, const void* d_syms, uint64_t nchunks, const uint64_t* d_starts,
                      uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens, uint32_t* d_status, hipStream_t s,
                      fast::ChunkInit ini, uint64_t lmax) {
    if (nchunks == 0) return ANS_OK;
    const DevTable& t = gt->t;
    const Sym* syms = static_cast<const Sym*>(d_syms);
    if (lmax) {  // the longest chunk known on the host: the staged fast kernels
        const int rc = launch_staged_encode<Sym>(gt, syms, ChunkSpan<Sym>{d_starts, 0, 0}, nchunks, lmax, d_slots,
                                                 slot_cap, d_lens, d_status, s, ini);
        if (rc != kNotStaged) return rc;
    }
    const unsigned grid = grid_for(nchunks);
    const size_t lds = gt->lds_bytes ? sizeof(DevSym) * (t.nsym + 1) : 0;
    if (gt->lds_bytes && t.fast)
        k_encode<Sym, true, true><<<grid, kBlock, lds, s>>>(t, syms, 0, 0, d_starts, 0, nchunks, d_slots, slot_cap, d_lens, d_status, ini);
    else if (gt->lds_bytes)
        k_encode<Sym, true, false><<<grid, kBlock, lds, s>>>(t, syms, 0, 0, d_starts, 0, nchunks, d_slots, slot_cap, d_lens, d_status, ini);
    else if (t.fast)
        k_encode<Sym, false, true><<<grid, kBlock, 0, s>>>(t, syms, 0, 0, d_starts, 0, nchunks, d_slots, slot_cap, d_lens, d_status, ini);
    else
        k_encode<Sym, false, false><<<grid, kBlock, 0, s>>>(t, syms, 0, 0, d_starts, 0, nchunks, d_slots, slot_cap, d_lens, d_status, ini);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
}

template <typename Sym>
int launch_decode_var(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap,
                      const uint32_t* d_lens, uint64_t nchunks, const uint64_t* d_starts, int gen_kind, void* d_syms,
                      uint32_t* d_status, hipStream_t s, fast::ChunkInit ini, uint64_t lmax) {
    if (nchunks == 0) return ANS_OK;
    const DevTable& t = gt->t;
    Sym* out = static_cast<Sym*>(d_syms);
    if (lmax) {
        const int rc = launch_staged_decode<Sym>(gt, d_in, d_offsets, slot_cap, d_lens, ChunkSpan<Sym>{d_starts, 0, 0},
                                                 nchunks, lmax, gen_kind, out, d_status, s, ini);
        if (rc != kNotStaged) return rc;
    }
    const unsigned grid = grid_for(nchunks);
    const size_t lds = gt->lds_bytes;
    if (gt->lds_bytes && t.fast)
        k_decode<Sym, true, true><<<grid, kBlock, lds, s>>>(t, d_in, d_offsets, slot_cap, d_lens, 0, 0, d_starts, 0, nchunks, gen_kind, out, d_status, ini);
    else if (gt->lds_bytes)
        k_decode<Sym, true, false><<<grid, kBlock, lds, s>>>(t, d_in, d_offsets, slot_cap, d_lens, 0, 0, d_starts, 0, nchunks, gen_kind, out, d_status, ini);
    else if (t.fast)
        k_decode<Sym, false, true><<<grid, kBlock, 0, s>>>(t, d_in, d_offsets, slot_cap, d_lens, 0, 0, d_starts, 0, nchunks, gen_kind, out, d_status, ini);
    else
        k_decode<Sym, false, false><<<grid, kBlock, 0, s>>>(t, d_in, d_offsets, slot_cap, d_lens, 0, 0, d_starts, 0, nchunks, gen_kind, out, d_status, ini);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
}

template <typename Sym>
int launch_sample(ans_gpu_table* gt, uint64_t seed, uint64_t n, uint64_t chunk_len, void* d_syms, hipStream_t s) {
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    if (nchunks == 0) return ANS_OK;
    Sym* out = static_cast<Sym*>(d_syms);
    if (gt->ft.usable && gt->ft.dec_usable && gt->ft.nr == fast::kNormStd) {  // the fast decoder's LDS tables (ans_fast.hpp k_sample)
        const unsigned dgrid = static_cast<unsigned>((nchunks + fast::kDecBlock - 1) / fast::kDecBlock);
        fast::k_sample<Sym><<<dgrid, fast::kDecBlock, gt->ft.dec_lds_bytes, s>>>(gt->ft, seed, n, chunk_len, nchunks, out);
        HIP_TRY(hipGetLastError());
        return ANS_OK;
    }
    const unsigned grid = grid_for(nchunks);
    if (gt->lds_bytes && gt->t.fast)
        k_sample_iid<Sym, true, true><<<grid, kBlock, gt->lds_bytes, s>>>(gt->t, seed, n, chunk_len, nchunks, out);
    else if (gt->lds_bytes)
        k_sample_iid<Sym, true, false><<<grid, kBlock, gt->lds_bytes, s>>>(gt->t, seed, n, chunk_len, nchunks, out);
    else if (gt->t.fast)
        k_sample_iid<Sym, false, true><<<grid, kBlock, 0, s>>>(gt->t, seed, n, chunk_len, nchunks, out);
    else
        k_sample_iid<Sym, false, false><<<grid, kBlock, 0, s>>>(gt->t, seed, n, chunk_len, nchunks, out);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
}

}  // namespace launch
}  // namespace shuffle_coding
