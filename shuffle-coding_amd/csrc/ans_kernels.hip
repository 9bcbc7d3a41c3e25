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

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ans_kcommon.hpp"
#include "ans_launch.hpp"

using namespace shuffle_coding::launch;

namespace {

// Self-check of the decoders' renorm step (fast::renorm_up) on caller-chosen (head, window)
// pairs, for tests: its rare exact path (X >> 8 landing in [L, 2^56)) is too rare in coded
// data to be reached reliably (~norm / 2^56 per symbol).
__global__ __launch_bounds__(256) void k_check_renorm(const uint64_t* __restrict__ heads,
                                                      const uint32_t* __restrict__ windows, uint64_t L, uint64_t n,
                                                      uint64_t* __restrict__ out_heads, uint32_t* __restrict__ out_k) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t h = heads[i];
    out_k[i] = fast::renorm_up(h, windows[i], L, fast::renorm_screen(L));
    out_heads[i] = h;
}

// One wave copies one stream: byte head until dst is dword-aligned, then aligned dword
// stores funnelled from two source dwords (v_alignbyte), then the byte tail.  Source reads
// are aligned dwords that each hold at least one byte of the stream (no over-read past the
// dword holding its last byte).
__device__ __forceinline__ void wave_copy(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint32_t len,
                                          uint32_t lane) {
    const uint32_t head = min(len, (4u - static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst) & 3)) & 3u);
    if (lane < head) dst[lane] = src[lane];
    dst += head;
    src += head;
    len -= head;
    const uint32_t nd = len / 4, sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src) & 3);
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(src) & ~uintptr_t(3));
    uint32_t* d4 = reinterpret_cast<uint32_t*>(dst);
    for (uint32_t i = lane; i < nd; i += 64) {
        const uint32_t lo = s4[i], hi = sh ? s4[i + 1] : 0u;  // sh is wave-uniform
        d4[i] = __builtin_amdgcn_alignbyte(hi, lo, sh);
    }
    if (lane < len - 4 * nd) dst[4 * nd + lane] = src[4 * nd + lane];
}

// One wave packs one stream from a 16-B-aligned source (a slot) to any destination in whole
// aligned 16-B stores: destination block j (of the 16-B-aligned line holding dst, dsh = dst & 15)
// takes stream bytes [16j - dsh, 16j - dsh + 16), i.e. source blocks j-1 and j funnelled by
// v_alignbyte at a wave-uniform dword step and byte shift.  The first and last blocks may hold
// a neighbouring stream's bytes: those are written byte by byte (no store touches a byte
// outside the stream, so neighbouring waves never race).  Only source blocks holding stream
// bytes are read, each once: block j-1 comes from the lane below (DPP wave_shr:1), and for lane
// 0 from lane 63 of the previous pass (v_readlane), where a second load per lane read every
// block twice through the L1 (the pack ran at 5.2 TB/s, profiles/r03b_kernel_stats_c3.csv).
__device__ __forceinline__ uint32_t from_lane_below(uint32_t v, uint32_t carry) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(carry), static_cast<int>(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ void wave_pack(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint32_t len,
                                          uint32_t lane) {
    if (len == 0) return;
    const uint32_t dsh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst) & 15);
    uint8_t* dbase = dst - dsh;
    const uint4* s16 = reinterpret_cast<const uint4*>(src);
    const uint32_t nblk = (dsh + len + 15) / 16;
    const uint32_t bs = (16u - dsh) & 3u;         // byte shift inside the 32-B window
    const uint32_t i0 = (16u - dsh) >> 2;         // first window dword of an output block
    uint4 carry = make_uint4(0, 0, 0, 0);         // block j0 - 1 (none before the stream)
    // passes of up to four 64-block rounds whose loads are all issued first (four 16-B loads in
    // flight per lane: one at a time left the copy latency-bound at ~5.6 TB/s)
    constexpr int kR = 4;
    for (uint32_t j0 = 0; j0 < nblk; j0 += 64 * kR) {  // (wave-uniform: every lane takes part in the DPP moves)
        uint4 bb[kR];
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            const uint32_t j = j0 + 64 * r + lane;
            bb[r] = (j < nblk && 16 * j < len) ? s16[j] : make_uint4(0, 0, 0, 0);  // only blocks holding stream bytes
        }
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            const uint32_t j = j0 + 64 * r + lane;
            if (j0 + 64 * r >= nblk) break;  // (uniform)
            const uint4 b = bb[r];
            const uint4 a = make_uint4(from_lane_below(b.x, carry.x), from_lane_below(b.y, carry.y),
                                       from_lane_below(b.z, carry.z), from_lane_below(b.w, carry.w));
            carry = make_uint4(__builtin_amdgcn_readlane(b.x, 63), __builtin_amdgcn_readlane(b.y, 63),
                               __builtin_amdgcn_readlane(b.z, 63), __builtin_amdgcn_readlane(b.w, 63));
            if (j >= nblk) continue;
            const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            uint32_t o[4];
            // i0 is wave-uniform: a scalar branch picks constant register indices
            switch (i0) {
#define PACK_CASE(I)                                                                 \
    case I:                                                                          \
        for (int k = 0; k < 4; ++k)                                                  \
            o[k] = (I + k + 1 < 8) ? __builtin_amdgcn_alignbyte(w[(I + k + 1) & 7], w[I + k], bs) : w[I + k]; \
        break;
                PACK_CASE(0)
                PACK_CASE(1)
                PACK_CASE(2)
                PACK_CASE(3)
                default:
                    for (int k = 0; k < 4; ++k) o[k] = w[4 + k];  // dsh = 0: block j itself
#undef PACK_CASE
            }
            const uint32_t lo = j == 0 ? dsh : 0u;                           // first byte of the stream here
            const uint32_t hi = min(16u, dsh + len - 16u * j);               // one past its last
            if (lo == 0 && hi == 16) {
                *reinterpret_cast<uint4*>(dbase + 16ull * j) = make_uint4(o[0], o[1], o[2], o[3]);
            } else {
#pragma unroll
                for (uint32_t t = 0; t < 16; ++t)
                    if (t >= lo && t < hi) dbase[16ull * j + t] = static_cast<uint8_t>(o[t >> 2] >> (8 * (t & 3)));
            }
        }
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
    const uint32_t len = static_cast<uint32_t>(min<uint64_t>(lens[c], slot_cap));  // never past the slot
    if ((reinterpret_cast<uintptr_t>(s) & 15) == 0) wave_pack(d, s, len, lane);
    else wave_copy(d, s, len, lane);
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
    wave_copy(d, s, lens[c], lane);
}

// ---- device-resident dense container (include/ans_capi.h ans_dev_encode_dense_ex)
// Exclusive scan of the stream lengths in tiles of 4,096 chunks (1,024 threads x 4, a
// 64-lane shuffle scan per wave, the 16 wave totals through LDS): each tile leaves its local
// offsets and its total; k_scan_tile_sums scans the totals in place (one workgroup); then
// k_compact_dense adds its tile's prefix, publishes the final offset and packs the stream.
// Lengths are clamped to the slot like k_compact's copies, so offsets and bytes agree.
constexpr uint32_t kScanTile = 4096;

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, uint32_t lane) {
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(v, d, 64);
        if (lane >= d) v += y;
    }
    return v;
}

__global__ __launch_bounds__(1024) void k_scan_tiles(const uint32_t* __restrict__ lens, uint64_t n, uint64_t slot_cap,
                                                     uint64_t* __restrict__ offs, uint64_t* __restrict__ tile_sum) {
    __shared__ uint64_t wsum[16];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t i0 = static_cast<uint64_t>(blockIdx.x) * kScanTile + 4 * threadIdx.x;
    uint64_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i0 + k < n ? min<uint64_t>(lens[i0 + k], slot_cap) : 0;
    const uint64_t t = v[0] + v[1] + v[2] + v[3];
    const uint64_t incl = wave_incl_scan(t, lane);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint64_t run = incl - t;
    for (uint32_t w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (i0 + k < n) offs[i0 + k] = run;
        run += v[k];
    }
    if (threadIdx.x == 1023) tile_sum[blockIdx.x] = run;  // the tile's total
}

__global__ __launch_bounds__(1024) void k_scan_tile_sums(uint64_t* __restrict__ tile_sum, uint64_t ntiles,
                                                         uint64_t* __restrict__ total) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) carry = 0;
    for (uint64_t b = 0; b < ntiles; b += 1024) {
        __syncthreads();  // carry written, last round's wsum reads done
        const uint64_t i = b + threadIdx.x;
        const uint64_t t = i < ntiles ? tile_sum[i] : 0;
        const uint64_t incl = wave_incl_scan(t, lane);
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint64_t pre = carry + incl - t;
        for (uint32_t w = 0; w < wave; ++w) pre += wsum[w];
        if (i < ntiles) tile_sum[i] = pre;
        __syncthreads();  // every carry read done
        if (threadIdx.x == 1023) carry = pre + t;
    }
    __syncthreads();
    if (threadIdx.x == 0) *total = carry;
}

// One wave per chunk: offset = local + tile prefix; the stream is packed unless it would end
// past out_cap (ANS_E_LEN).
__global__ __launch_bounds__(kBlock) void k_compact_dense(const uint8_t* __restrict__ slots, uint64_t slot_cap,
                                                          const uint32_t* __restrict__ lens, uint64_t* __restrict__ offs,
                                                          const uint64_t* __restrict__ tile_pre, uint64_t nchunks,
                                                          uint8_t* __restrict__ out, uint64_t out_cap,
                                                          uint32_t* __restrict__ status) {
    const uint64_t c = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (c >= nchunks) return;
    const uint32_t len = static_cast<uint32_t>(min<uint64_t>(lens[c], slot_cap));
    const uint64_t off = offs[c] + tile_pre[c / kScanTile];
    if (lane == 0) offs[c] = off;  // (every lane has read offs[c]: one load instruction)
    if (off + len > out_cap) {
        if (lane == 0) atomicOr(status, 1u << ANS_E_LEN);
        return;
    }
    const uint8_t* src = slots + c * slot_cap;
    if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) wave_pack(out + off, src, len, lane);
    else wave_copy(out + off, src, len, lane);
}

bool valid_width(int w) { return w == 1 || w == 2 || w == 4; }
bool valid_kind(int k) { return k == ANS_GEN_ZEROS || k == ANS_GEN_EMPTY || k == ANS_GEN_RANDOM; }

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

// 1/d rounded UP (fma(r, d, -1) is the exact sign of r d - 1): kNormSmall's exact high division
// step (ans_fast.hpp div_hi) needs r >= 1/d, and r - 1/d < 2^-52 / d keeps its estimates as
// tight as fl(1/d)'s
static double rcp_up(uint32_t d) {
    double r = 1.0 / static_cast<double>(d);
    while (std::fma(r, static_cast<double>(d), -1.0) < 0.0) r = std::nextafter(r, 2.0);
    return r;
}

// Derives the fast-path tables (ans_table.hpp FastTable) when the table qualifies: nsym <= 65536
// and norm < 2^32, in one of the three norm ranges (2^16 <= norm <= 2^31: one f64 quotient
// estimate; below 2^16 or above 2^31: the kNormSmall / kNormBig division of
// DESIGN.md §4b, in the LDS kernels and the large-alphabet ones alike).  Up to 256 symbols the
// rows and decode buckets are staged in LDS; above, the encoder reads its rows from global memory
// (k_encode with global rows, or k_encode_w from 2^22 on) and decodes take k_decode_w / k_decode_g.
int build_fast_table(ans_gpu_table* gt, const Categorical& cat) {
    const DevTable& t = gt->t;
    FastTable ft{};
    const uint32_t nr = t.fast ? fast::kNormStd : (t.norm < (1u << 16) ? fast::kNormSmall : fast::kNormBig);
    if (t.nsym > 65536u) {
        gt->ft = ft;
        return ANS_OK;
    }
    using u128 = unsigned __int128;
    const uint32_t nsym = t.nsym;
    std::vector<EncRow> enc(nsym + 1);
    uint32_t kmax = 1;
    std::vector<uint32_t> kmax_row(nsym + 1, 0);
    for (uint32_t s = 0; s <= nsym; ++s) {
        const uint64_t m = s < nsym ? cat.masses[s] : 0;
        const double rcp = nr == fast::kNormSmall ? rcp_up(static_cast<uint32_t>(m)) : 1.0 / static_cast<double>(m);
        enc[s] = EncRow{m ? rcp : 0.0, static_cast<uint32_t>(m),
                        s < nsym ? static_cast<uint32_t>(cat.cummasses[s]) : t.norm};
        if (!m) continue;
        const u128 pK = static_cast<u128>(m) * t.K;
        for (uint32_t j = 1; j <= 4; ++j)  // can a push emit j bytes? (head < 2^64 <= p*K*2^8j otherwise)
            if ((pK << (8 * j)) < (static_cast<u128>(1) << 64)) kmax_row[s] = j;
        kmax = std::max(kmax, kmax_row[s]);
    }
    // a symbol holding all of a power-of-two norm (L = 2^56) is the one row fast::enc_thr cannot
    // express (its renorm test must never hold, and every head up to 2^64 - 1 is possible)
    for (uint32_t s = 0; s < nsym; ++s)
        if (cat.masses[s] == t.norm && t.L == (1ull << 56)) {
            gt->ft = ft;
            return ANS_OK;
        }
    ft.enc_global = nsym > 256;
    ft.dec_usable = nsym <= 256;
    // decode buckets: the finest power-of-two width whose table fits fast::kDecTableBytes in
    // LDS (with the cdf table); for large alphabets, at most 2^16 buckets in global memory
    uint32_t shift = 0;
    const size_t cum_bytes = sizeof(uint32_t) * (nsym + 5);
    const uint64_t max_buckets = ft.dec_usable ? fast::kDecNbMax : (1ull << 16);
    while (((static_cast<uint64_t>(t.norm) - 1) >> shift) + 1 > max_buckets) ++shift;
    const uint32_t nb = static_cast<uint32_t>(((static_cast<uint64_t>(t.norm) - 1) >> shift) + 1);
    std::vector<uint32_t> cum(nsym + 6, t.norm);
    for (uint32_t s = 0; s < nsym; ++s) cum[s] = static_cast<uint32_t>(cat.cummasses[s]);
    std::vector<DecBucket> dec(ft.dec_usable ? nb : 0);
    std::vector<uint8_t> dec_s0(ft.dec_usable ? nb : 0);  // nsym <= 256: one byte each
    std::vector<DecBucketG> decg(ft.dec_usable ? 0 : nb);
    for (uint32_t j = 0; j < nb; ++j) {
        const uint32_t s0 = static_cast<uint32_t>(cat.icdf(static_cast<uint64_t>(j) << shift).first);
        if (ft.dec_usable) {
            DecBucket& d = dec[j];
            for (int i = 0; i < 4; ++i) d.c[i] = cum[s0 + i];
            dec_s0[j] = static_cast<uint8_t>(s0);
            // every cf of the bucket below cdf(s0 + 3)?  (the last bucket ends at norm)
            const uint64_t end = std::min<uint64_t>(t.norm, (static_cast<uint64_t>(j) + 1) << shift);
            if (d.c[3] < end) ft.dec_far = 1;
        } else {
            DecBucketG& d = decg[j];
            for (int i = 0; i < 6; ++i) d.c[i] = cum[s0 + i];
            d.s0 = s0;
            d.pad = 0;
        }
    }
    // the fix-up-free decoder's tables (ans_fast.hpp kModeU): the virtual alphabet over
    // u in [0, 2 norm) (v < 256: symbol v at cdf(v); v >= 256: symbol v - 256 at norm + cdf),
    // at the finest bucket width that fits; kept only if every bucket resolves among three
    // candidates (a table with fewer than 256 symbols can leave a bucket straddling u = norm
    // with the zero-mass gap between the halves: those keep the kModeRows tables)
    std::vector<uint8_t> uimg;
    if (ft.dec_usable && !ft.dec_far && t.norm < (1u << 31)) {
        const uint64_t n2 = 2ull * t.norm;
        auto cdfv = [&](uint32_t v) -> uint64_t {
            if (v >= 512) return n2;
            const uint32_t sv = v & 255u;
            const uint64_t c = cum[std::min(sv, nsym)];
            return v < 256 ? c : t.norm + c;
        };
        auto icdfv = [&](uint64_t x) {  // the last v in [0, 512) with cdfv(v) <= x
            uint32_t lo = 0, hi = 511;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) / 2;
                if (cdfv(mid) <= x) lo = mid;
                else hi = mid - 1;
            }
            return lo;
        };
        uint32_t us = 1;  // (rx = u << (31 - us) must stay a 32-bit shift)
        while (((n2 - 1) >> us) + 1 > fast::kDecUNbMax) ++us;
        const uint32_t nbu = static_cast<uint32_t>(((n2 - 1) >> us) + 1);
        uimg.assign(fast::kDecTableBytes, 0);
        bool ok = us <= fast::kDecUShiftMax;  // (norm <= 3072 * 2^17: s0 below the threshold bits)
        // threshold word of boundary c in the bucket at a, with s0 in its low bits (ans_fast.hpp
        // kDecUNbMax): u >= c  <=>  u << (31 - us) > this word (mod 2^32), for u in the bucket:
        // the shifted u keeps the bucket index's low bit at bit 31, and so does the word, so the
        // two differ by less than 2^31 and the kernel takes the comparison as the sign of their
        // difference
        auto word = [&](uint64_t a, uint64_t c, uint32_t s0) {
            const uint64_t rel = std::min<uint64_t>(c - a, 1ull << us);  // >= 1: c > a
            return static_cast<uint32_t>((((a >> us) & 1u) << 31) | ((rel - 1) << (31 - us)) | s0);
        };
        for (uint32_t j = 0; j < nbu && ok; ++j) {
            const uint64_t a = static_cast<uint64_t>(j) << us, end = std::min<uint64_t>(n2, a + (1ull << us));
            const uint32_t s0 = icdfv(a);
            if (cdfv(s0 + 3) < end) ok = false;
            const uint32_t w12[2] = {word(a, cdfv(s0 + 1), s0), word(a, cdfv(s0 + 2), s0)};
            std::memcpy(uimg.data() + 8 * j, w12, 8);
        }
        for (uint32_t v = 0; v < 512 && ok; ++v) {
            const uint32_t sv = v & 255u;
            const uint32_t m = sv < nsym ? static_cast<uint32_t>(cat.masses[sv]) : 0u;
            const uint32_t c = cum[std::min(sv, nsym)];
            // head = p * q_m + (u - cum_row): lower half q = q_m, cf = u; upper q = q_m + 1, cf = u - norm
            const uint32_t row[2] = {v < 256 ? c : t.norm + c - m, m};
            std::memcpy(uimg.data() + fast::kDecURowOff + 8 * v, row, 8);
        }
        if (ok) {
            ft.dec_u = 1;
            ft.dec_u_shift = us;
        } else {
            uimg.clear();
        }
    }
    ft.dec_global = !ft.dec_usable;
    // compact 16-B buckets for k_decode_w: the finest width with at most 2^17 buckets (2 MiB),
    // if every bucket's five candidate offsets fit u16
    std::vector<DecBucketC> decc, decl;
    if (ft.dec_global) {
        uint32_t cs = 0;
        while (((static_cast<uint64_t>(t.norm) - 1) >> cs) + 1 > (1ull << 17)) ++cs;
        const uint32_t ncb = static_cast<uint32_t>(((static_cast<uint64_t>(t.norm) - 1) >> cs) + 1);
        decc.resize(ncb);
        bool fits = true;
        for (uint32_t j = 0; j < ncb && fits; ++j) {
            const uint32_t s0 = static_cast<uint32_t>(cat.icdf(static_cast<uint64_t>(j) << cs).first);
            DecBucketC& d = decc[j];
            d.c0 = cum[s0];
            d.s0 = static_cast<uint16_t>(s0);
            for (int k = 0; k < 5; ++k) {
                const uint32_t off = cum[s0 + 1 + k] - cum[s0];
                if (off > 0xFFFFu) fits = false;
                d.d[k] = static_cast<uint16_t>(off);
            }
        }
        if (fits) {
            ft.dec_c = 1;
            ft.dec_c_shift = cs;
            ft.dec_cl_shift = cs;
        } else {
            decc.clear();
        }
        // the LDS beside k_decode_w's ring holds kWideDecBktLds buckets; a table with more stages
        // its first ones at twice the width, which doubles the share of lookups the LDS serves
        // (C4: 9.2% -> 18.3%), if they resolve among their five candidates for all but 1/256 of
        // the cf they cover (C4: 0.23%; the rest re-fetch their global bucket, ans_wide.hpp)
        if (ft.dec_c && ncb > fast::kWideDecBktLds) {
            const uint32_t ls = cs + 1;
            const uint32_t nl = static_cast<uint32_t>(std::min<uint64_t>(((static_cast<uint64_t>(t.norm) - 1) >> ls) + 1,
                                                                         fast::kWideDecBktLds));
            decl.resize(nl);
            bool lfits = true;
            uint64_t far = 0, covered = 0;
            for (uint32_t j = 0; j < nl && lfits; ++j) {
                const uint64_t b0 = static_cast<uint64_t>(j) << ls;
                const uint64_t b1 = std::min<uint64_t>(b0 + (1ull << ls), t.norm);
                const uint32_t s0 = static_cast<uint32_t>(cat.icdf(b0).first);
                DecBucketC& d = decl[j];
                d.c0 = cum[s0];
                d.s0 = static_cast<uint16_t>(s0);
                for (int k = 0; k < 5; ++k) {
                    const uint32_t off = cum[s0 + 1 + k] - cum[s0];
                    if (off > 0xFFFFu) lfits = false;
                    d.d[k] = static_cast<uint16_t>(off);
                }
                const uint64_t c5 = std::max<uint64_t>(cum[s0 + 5], b0);
                far += b1 > c5 ? b1 - c5 : 0;
                covered += b1 - b0;
            }
            if (lfits && far * 256 <= covered) ft.dec_cl_shift = ls;
            else decl.clear();
        }
    }
    ft.enc_wide = ft.enc_global && t.norm >= fast::kWideNormMin;
    ft.enc_nl = std::min<uint32_t>(nsym, fast::kWideEncCumMax - 1);
    // the packed prefix (ans_table.hpp enc_pack): the longest multiple of 16 symbols whose image
    // fits the same LDS and whose in-block offsets fit u16; used when it is longer
    std::vector<uint32_t> pack_img;
    uint32_t pmax = 0;
    for (uint32_t s = 0; s < nsym; ++s) pmax = std::max<uint32_t>(pmax, static_cast<uint32_t>(cat.masses[s]));
    // k_encode_w<kSa> (ans_wide.hpp): a renorm shift byte per mass 0..pmax at LDS offset 0, when
    // every mass has one (ans_renorm.hpp enc_sa); it takes kWideSaBytes from the prefix
    std::vector<uint8_t> sa_img;
    if (ft.enc_wide && pmax <= fast::kWideSaMax) {
        sa_img.assign(fast::kWideSaBytes, 8);
        for (uint32_t p = 0; p <= pmax && !sa_img.empty(); ++p) {
            const uint32_t sa = fast::enc_sa(static_cast<uint64_t>(p) * t.K, t.L);
            if (sa == 0) sa_img.clear();
            else sa_img[p] = static_cast<uint8_t>(sa);
        }
    }
    if (ft.enc_wide && pmax <= 0xFFFFu) {  // (pmf from two low halves: every mass below 2^16)
        const uint32_t nl_max = fast::wide_pack_nl_max(!sa_img.empty());  // (the LDS regions, ans_wide.hpp)
        auto img_bytes = [](uint32_t nl) {
            const uint32_t ooff = 4 * ((nl >> 4) + 2);
            return (ooff + 2 * (nl + 2) + 3) & ~3u;
        };
        uint32_t nlp = 0;
        while (nlp + 16 <= nsym && nlp + 16 <= nl_max) {
            bool fits = true;
            for (uint32_t k = nlp; k < nlp + 16 && fits; ++k) fits = cum[k + 1] - cum[nlp] <= 0xFFFFu || ((k + 1) & 15) == 0;
            if (!fits) break;
            nlp += 16;
        }
        if (nlp > ft.enc_nl) {
            const uint32_t ooff = 4 * ((nlp >> 4) + 2);
            pack_img.assign(img_bytes(nlp) / 4, 0);
            for (uint32_t k = 0; k < (nlp >> 4) + 2; ++k) pack_img[k] = cum[std::min<uint32_t>(16 * k, nsym + 5)];
            auto* o16 = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(pack_img.data()) + ooff);
            for (uint32_t k = 0; k < nlp + 2; ++k) o16[k] = static_cast<uint16_t>(cum[std::min<uint32_t>(k, nsym + 5)]);
            ft.enc_pack = 1;
            ft.enc_nl = nlp;
            ft.enc_pack_ooff = ooff;
            ft.enc_pack_bytes = img_bytes(nlp);
            ft.enc_sa = sa_img.empty() ? 0 : 1;
        }
    }
    if (!ft.enc_sa) sa_img.clear();
    // the packed encoder's global rows (ans_table.hpp enc_grow): (cdf(s), O(s) | O(s+1) << 16)
    // k_encode_w reads the global row of every symbol, the prefix's lanes at row nl - 1 (zero), and
    // every symbol's LDS row at min(s, nl), which for s >= nl is row C = (cdf(nl), O(nl) | O(nl+1)
    // << 16); it XORs the two, so the global rows from nl on are stored XORed with C
    std::vector<uint32_t> grow;
    if (ft.enc_pack) {
        const uint32_t nl = ft.enc_nl;
        grow.resize(2 * (static_cast<size_t>(nsym) + 1));
        const uint32_t c0 = cum[nl], c1 = (cum[nl] & 0xFFFFu) | (cum[nl + 1] << 16);
        for (uint32_t k = 0; k <= nsym; ++k) {
            grow[2 * k] = k >= nl ? cum[k] ^ c0 : 0u;
            grow[2 * k + 1] = k >= nl ? ((cum[k] & 0xFFFFu) | (cum[k + 1] << 16)) ^ c1 : 0u;
        }
    }
    // k_decode_w's LDS prefix: for each bucket width 2^shp, the longest prefix of symbols whose
    // bucket starts (u16) and cdf fit beside the ring; keep the width whose prefix covers the most
    // probability among those whose cf needs a fifth candidate at most 0.1% of the time
    std::vector<uint16_t> wide_s0;
    if (ft.dec_global && nsym <= 65536) {
        const uint32_t budget = fast::kWideDecTabBytes;
        uint32_t best_shp = 0, best_nlp = 0;
        uint64_t best_cov = 0;
        double best_far = 2.0;
        for (uint32_t shp = 0; shp <= 24; ++shp) {
            auto bytes = [&](uint32_t nlp) {
                const uint64_t nbp = nlp ? ((static_cast<uint64_t>(cum[nlp]) + (1ull << shp) - 1) >> shp) : 0;
                return ((2 * nbp + 15) & ~uint64_t(15)) + 4ull * (nlp + 6);
            };
            uint32_t lo = 0, hi = nsym;  // largest nlp with bytes(nlp) <= budget (bytes grows with nlp)
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) / 2;
                if (bytes(mid) <= budget) lo = mid;
                else hi = mid - 1;
            }
            const uint32_t nlp = lo;
            if (nlp == 0 || cum[nlp] == 0) continue;
            const uint64_t cpre = cum[nlp], nbp = (cpre + (1ull << shp) - 1) >> shp;
            uint64_t far = 0;  // cf values of the prefix past their bucket's fifth candidate
            for (uint64_t b = 0; b < nbp; ++b) {
                const uint64_t a = b << shp, e = std::min<uint64_t>(cpre, (b + 1) << shp);
                const uint64_t s0 = cat.icdf(a).first;
                const uint64_t c4 = s0 + 4 <= nsym ? cum[s0 + 4] : t.norm;
                if (c4 < e) far += e - std::max<uint64_t>(a, c4);
            }
            const double far_frac = static_cast<double>(far) / static_cast<double>(cpre);
            const bool ok = far_frac <= 1e-3, best_ok = best_far <= 1e-3;
            if ((ok && (!best_ok || cpre > best_cov)) || (!ok && !best_ok && far_frac < best_far)) {
                best_shp = shp;
                best_nlp = nlp;
                best_cov = cpre;
                best_far = far_frac;
            }
        }
        if (best_nlp > 0) {
            ft.dec_wide = 1;
            ft.dec_w_shp = best_shp;
            ft.dec_w_nlp = best_nlp;
            ft.dec_w_cpre = cum[best_nlp];
            ft.dec_w_nbp = static_cast<uint32_t>((static_cast<uint64_t>(ft.dec_w_cpre) + (1ull << best_shp) - 1) >> best_shp);
            ft.dec_w_cum_off = (2 * ft.dec_w_nbp + 15) & ~15u;
            wide_s0.resize(ft.dec_w_nbp + 2, 0);
            for (uint32_t b = 0; b < ft.dec_w_nbp; ++b)
                wide_s0[b] = static_cast<uint16_t>(cat.icdf(static_cast<uint64_t>(b) << best_shp).first);
        }
    }
    ft.nsym = nsym;
    ft.enc_rows = nsym + 1;
    ft.dec_buckets = nb;
    ft.dec_shift = shift;
    ft.norm = t.norm;
    ft.enc_lds_bytes = fast::kEncLdsBytes;  // nsym + 1 <= 257 rows, split (ans_fast.hpp)
    ft.dec_s0_off = fast::kDecS0Off;  // fixed layout (ans_fast.hpp)
    ft.dec_cum_off = fast::kDecCumOff;
    ft.dec_lds_bytes = static_cast<uint32_t>((ft.dec_cum_off + cum_bytes + 15) & ~size_t(15));
    ft.kmax = kmax;
    ft.pmax = pmax;
    ft.nr = nr;
    // k_decode's 24-bit high-word product needs hi32(q) < 2^24 too: q < 2^64 / norm
    ft.p24 = pmax < (1u << 24) && t.norm > 256 ? 1u : 0u;
    ft.K = t.K;
    ft.L = t.L;
    ft.rcp_norm = nr == fast::kNormSmall ? rcp_up(t.norm) : t.rcp_norm;
    const size_t enc_b = sizeof(EncRow) * enc.size(), dec_b = ft.dec_cum_off;  // buckets + s0 array
    const size_t decg_b = sizeof(DecBucketG) * decg.size();
    const size_t o_dec = (enc_b + 255) & ~size_t(255), o_cum = o_dec + ((dec_b + 255) & ~size_t(255));
    const size_t o_decg = o_cum + ((sizeof(uint32_t) * cum.size() + 255) & ~size_t(255));
    const size_t o_ws0 = o_decg + ((decg_b + 255) & ~size_t(255));
    const size_t ws0_b = sizeof(uint16_t) * wide_s0.size();
    const size_t o_decc = o_ws0 + ((ws0_b + 255) & ~size_t(255));
    const size_t decc_b = sizeof(DecBucketC) * decc.size();
    const size_t o_decl = o_decc + ((decc_b + 255) & ~size_t(255));
    const size_t decl_b = sizeof(DecBucketC) * decl.size();
    const size_t o_pack = o_decl + ((decl_b + 255) & ~size_t(255));
    const size_t pack_b = sizeof(uint32_t) * pack_img.size();
    const size_t o_sa = o_pack + ((pack_b + 255) & ~size_t(255));
    const size_t o_grow = o_sa + ((sa_img.size() + 255) & ~size_t(255));
    const size_t o_uimg = o_grow + ((4 * grow.size() + 255) & ~size_t(255));
    HIP_TRY(hipSetDevice(gt->g->device));
    void* mem = nullptr;
    HIP_TRY(hipMalloc(&mem, o_uimg + uimg.size() + 16));
    gt->d_fast = mem;
    char* base = static_cast<char*>(mem);
    HIP_TRY(hipMemcpy(base, enc.data(), enc_b, hipMemcpyHostToDevice));
    if (!dec.empty()) {  // buckets at 0, s0 bytes at kDecS0Off (staged into LDS as one block)
        std::vector<uint8_t> img(ft.dec_cum_off, 0);
        for (size_t j = 0; j < dec.size(); ++j) {  // halves (c0,c1) at 8j, (c2,c3) at 8 (kDecNbMax + j)
            std::memcpy(img.data() + 8 * j, &dec[j].c[0], 8);
            std::memcpy(img.data() + 8 * (fast::kDecNbMax + j), &dec[j].c[2], 8);
        }
        std::memcpy(img.data() + ft.dec_s0_off, dec_s0.data(), dec_s0.size());
        HIP_TRY(hipMemcpy(base + o_dec, img.data(), img.size(), hipMemcpyHostToDevice));
    }
    HIP_TRY(hipMemcpy(base + o_cum, cum.data(), sizeof(uint32_t) * cum.size(), hipMemcpyHostToDevice));
    if (decg_b) HIP_TRY(hipMemcpy(base + o_decg, decg.data(), decg_b, hipMemcpyHostToDevice));
    if (ws0_b) HIP_TRY(hipMemcpy(base + o_ws0, wide_s0.data(), ws0_b, hipMemcpyHostToDevice));
    if (decc_b) HIP_TRY(hipMemcpy(base + o_decc, decc.data(), decc_b, hipMemcpyHostToDevice));
    ft.dbkt_c = reinterpret_cast<const DecBucketC*>(base + o_decc);
    if (decl_b) HIP_TRY(hipMemcpy(base + o_decl, decl.data(), decl_b, hipMemcpyHostToDevice));
    ft.dbkt_cl = decl_b ? reinterpret_cast<const DecBucketC*>(base + o_decl) : ft.dbkt_c;
    if (pack_b) HIP_TRY(hipMemcpy(base + o_pack, pack_img.data(), pack_b, hipMemcpyHostToDevice));
    ft.enc_pack_img = reinterpret_cast<const uint32_t*>(base + o_pack);
    if (!sa_img.empty()) HIP_TRY(hipMemcpy(base + o_sa, sa_img.data(), sa_img.size(), hipMemcpyHostToDevice));
    ft.enc_sa_img = reinterpret_cast<const uint32_t*>(base + o_sa);
    if (!grow.empty()) HIP_TRY(hipMemcpy(base + o_grow, grow.data(), 4 * grow.size(), hipMemcpyHostToDevice));
    ft.enc_grow = reinterpret_cast<const uint32_t*>(base + o_grow);
    if (!uimg.empty()) HIP_TRY(hipMemcpy(base + o_uimg, uimg.data(), uimg.size(), hipMemcpyHostToDevice));
    ft.dec_u_img = reinterpret_cast<const uint32_t*>(base + o_uimg);
    ft.dec_w_s0 = reinterpret_cast<const uint16_t*>(base + o_ws0);
    ft.dbkt_g = reinterpret_cast<const DecBucketG*>(base + o_decg);
    ft.enc = reinterpret_cast<const EncRow*>(base);
    ft.dbkt = reinterpret_cast<const DecBucket*>(base + o_dec);
    ft.cum = reinterpret_cast<const uint32_t*>(base + o_cum);
    ft.usable = 1;
    gt->ft = ft;
    return ANS_OK;
}

// ------------------------------------------------------------------ host-buffer pipeline

constexpr int kPipeScattered = -1;

// Exclusive scan of a batch's stream lengths: offs[j] = sum of lens[0..j), offs[n] = total.
// One workgroup (n <= a few 10^5 per batch): each thread sums a contiguous segment, the
// segment sums are scanned in LDS, then each thread writes its segment's offsets.
__global__ __launch_bounds__(1024) void k_scan_lens(const uint32_t* __restrict__ lens, uint64_t n,
                                                    uint64_t* __restrict__ offs) {
    __shared__ uint64_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint64_t per = (n + 1023) / 1024, b = t * per, e = b + per < n ? b + per : n;
    uint64_t sum = 0;
    for (uint64_t i = b; i < e; ++i) sum += lens[i];
    part[t] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - sum;
    for (uint64_t i = b; i < e; ++i) {
        offs[i] = run;
        run += lens[i];
    }
    if (t == 1023) offs[n] = part[1023];
}

// the workspace slots in use
struct SlotRange {
    PipeSlot* a;
    PipeSlot* b;
    PipeSlot* begin() const { return a; }
    PipeSlot* end() const { return b; }
};
inline SlotRange slots_of(HostPipe* p) { return {p->slot, p->slot + p->depth}; }

void pipe_release(HostPipe* p) {
    for (PipeSlot& s : slots_of(p)) {
        (void)hipFree(s.d_syms);
        (void)hipFree(s.d_slots);
        (void)hipFree(s.d_dense);
        (void)hipFree(s.d_lens);
        (void)hipFree(s.d_offs);
        (void)hipHostFree(s.h_lens);
        (void)hipHostFree(s.h_offs);
        s.d_syms = s.d_slots = s.d_dense = nullptr;
        s.d_syms = nullptr;
        s.d_lens = nullptr;
        s.d_offs = nullptr;
        s.h_lens = nullptr;
        s.h_offs = nullptr;
        s.used = false;
    }
    p->cap_syms = p->cap_slots = p->cap_dense = p->cap_chunks = 0;
}

void pipe_free(ans_gpu* g) {
    HostPipe* p = g->pipe;
    if (!p) return;
    (void)hipDeviceSynchronize();
    pipe_release(p);
    for (PipeSlot& s : slots_of(p)) {
        (void)hipEventDestroy(s.ev_in);
        (void)hipEventDestroy(s.ev_comp);
        (void)hipEventDestroy(s.ev_meta);
        (void)hipEventDestroy(s.ev_out);
    }
    (void)hipFree(p->d_status);
    (void)hipFree(p->d_acc);
    if (p->h_meta) (void)hipHostFree(p->h_meta);
    if (p->ev_scan) (void)hipEventDestroy(p->ev_scan);
    (void)hipStreamDestroy(p->s_in);
    (void)hipStreamDestroy(p->s_out);
    (void)hipStreamDestroy(p->s_comp2);
    delete p;
    g->pipe = nullptr;
}

// A stream on a hardware queue of its own, its kernels restricted to the CUs of `pattern`
// (repeated over the mask words): a CU-masked queue is never shared.  The runtime moves
// device-to-host bytes with blit kernels on the copy stream's queue; with GPU_MAX_HW_QUEUES = 4
// and five streams in the process that queue was shared with the second compute stream, whose
// decode kernels then waited for every blit (tools/host_timeline.py), and a blit spread over
// all CUs leaves none free for a decode workgroup (which fills a CU's VGPRs and LDS).
hipError_t own_queue_stream(hipStream_t* s, uint32_t pattern) {
    int dev = 0, ncu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess || ncu <= 0) return e != hipSuccess ? e : hipErrorInvalidDevice;
    std::vector<uint32_t> mask((ncu + 31) / 32, pattern);
    if (ncu % 32) mask.back() &= (1u << (ncu % 32)) - 1u;
    return hipExtStreamCreateWithCUMask(s, static_cast<uint32_t>(mask.size()), mask.data());
}

// The context's pipeline with per-slot room for `syms` symbol bytes, `slots` slot bytes,
// `dense` dense bytes and `chunks` chunks (reallocated, after draining, when it must grow).
int pipe_get(ans_gpu* g, size_t syms, size_t slots, size_t dense, size_t chunks, HostPipe** out) {
    if (!g->pipe) {
        auto* p = new (std::nothrow) HostPipe{};
        if (!p) return ANS_E_ALLOC;
        g->pipe = p;
        if (const char* e = getenv("ANS_PIPE_DEPTH")) p->depth = std::min(kPipeDepthMax, std::max(2, atoi(e)));
        HIP_TRY(own_queue_stream(&p->s_in, ~0u));
        HIP_TRY(own_queue_stream(&p->s_out, 0x11111111u));  // device-to-host blits on a quarter of the CUs
        HIP_TRY(own_queue_stream(&p->s_comp2, ~0u));
        for (PipeSlot& s : slots_of(p)) {
            HIP_TRY(hipEventCreateWithFlags(&s.ev_in, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&s.ev_comp, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&s.ev_meta, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&s.ev_out, hipEventDisableTiming));
        }
        HIP_TRY(hipMalloc(&p->d_status, sizeof(uint32_t)));
    }
    HostPipe* p = g->pipe;
    if (syms > p->cap_syms || slots > p->cap_slots || dense > p->cap_dense || chunks > p->cap_chunks) {
        HIP_TRY(hipDeviceSynchronize());
        syms = std::max(syms, p->cap_syms);
        slots = std::max(slots, p->cap_slots);
        dense = std::max(dense, p->cap_dense);
        chunks = std::max(chunks, p->cap_chunks);
        pipe_release(p);
        for (PipeSlot& s : slots_of(p)) {
            HIP_TRY(hipMalloc(&s.d_syms, syms + 16));
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_slots), slots + 16));
            // + 256: k_decode_g (the non-wide large-alphabet decoder, norm < 2^22) reads whole
            // aligned 128-B lines around each stream, so the last stream of a batch may touch the
            // line past its span (k_decode and k_decode_w read only the stream's own bytes)
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_dense), dense + 256));
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_lens), sizeof(uint32_t) * chunks + 16));
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_offs), sizeof(uint64_t) * (chunks + 1) + 16));
            HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.h_lens), sizeof(uint32_t) * chunks + 16));
            HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.h_offs), sizeof(uint64_t) * (chunks + 1) + 16));
        }
        p->cap_syms = syms;
        p->cap_slots = slots;
        p->cap_dense = dense;
        p->cap_chunks = chunks;
    }
    for (PipeSlot& s : slots_of(p)) s.used = false;
    *out = p;
    return ANS_OK;
}

// Chunks per batch: about batch_bytes (default 128 MiB) of symbols.  A batch's kernels take
// about one chain latency (~1 ms) whatever its size until it fills the GPU, so batches must
// be large; 128 MiB batches through six workspace slots measured best for the round trip
// (tools/gpu_pipe_sweep.sh), with the workspace of three 256-MiB slots.
constexpr uint64_t kPipeBatchBytes = 128ull << 20;
uint64_t pipe_batch_chunks(const ans_gpu* g, uint64_t nchunks, uint64_t chunk_bytes) {
    const uint64_t target = g->batch_bytes ? g->batch_bytes : kPipeBatchBytes;
    uint64_t b = target / (chunk_bytes ? chunk_bytes : 1);
    if (b < 1) b = 1;
    return b < nchunks ? b : nchunks;
}

// Batch boundaries (chunk indices, first 0, last nchunks): batches of B chunks.  (Batches
// ramping up and down in size at the ends were measured too: with enough workspace slots
// they gained nothing over equal 128-MiB batches)
std::vector<uint64_t> pipe_cuts(uint64_t nchunks, uint64_t B) {
    std::vector<uint64_t> cuts{0};
    for (uint64_t c = B; c < nchunks; c += B) cuts.push_back(c);
    cuts.push_back(nchunks);
    return cuts;
}

// Encode from host symbols into a host dense container.  Batch b: H2D (s_in) -> encode,
// length scan, compaction, lengths D2H (compute stream b & 1); the host waits for batch
// b-1's lengths only after batch b is queued, then queues b-1's dense D2H (s_out) at its
// running offset.  With out == NULL (size query) nothing but the lengths comes back.
template <typename Sym>
int pipe_encode(ans_gpu_table* gt, const void* syms, uint64_t n, uint64_t chunk_len, uint8_t* out, uint64_t out_cap,
                uint64_t* offsets, uint64_t* lens, uint64_t* total, fast::ChunkInit ini) {
    constexpr uint64_t w = sizeof(Sym);
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    uint64_t slot_cap = 0;
    ans_gpu_slot_capacity(gt, chunk_len, &slot_cap);
    const uint64_t B = pipe_batch_chunks(gt->g, nchunks, chunk_len * w);
    HostPipe* p = nullptr;
    int rc = pipe_get(gt->g, B * chunk_len * w, B * slot_cap, out ? B * slot_cap : 0, B, &p);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(p->d_status, 0, sizeof(uint32_t), gt->g->stream));
    HIP_TRY(hipStreamSynchronize(gt->g->stream));
    const std::vector<uint64_t> cuts = pipe_cuts(nchunks, B);
    const uint64_t nbatch = cuts.size() - 1;
    const auto* src = static_cast<const uint8_t*>(syms);
    bool copy = out != nullptr;
    int len_err = ANS_OK;
    uint64_t acc = 0;
    auto enqueue = [&](uint64_t b) -> int {
        PipeSlot& s = p->slot[b % p->depth];
        const hipStream_t sc = (b & 1) ? p->s_comp2 : gt->g->stream;
        const uint64_t c0 = cuts[b], nc = cuts[b + 1] - c0, n0 = c0 * chunk_len;
        const uint64_t nb = std::min(n - n0, nc * chunk_len);
        if (s.used) HIP_TRY(hipStreamWaitEvent(p->s_in, s.ev_comp, 0));  // symbols of batch b - depth consumed
        HIP_TRY(hipMemcpyAsync(s.d_syms, src + n0 * w, nb * w, hipMemcpyHostToDevice, p->s_in));
        HIP_TRY(hipEventRecord(s.ev_in, p->s_in));
        HIP_TRY(hipStreamWaitEvent(sc, s.ev_in, 0));
        if (s.used) HIP_TRY(hipStreamWaitEvent(sc, s.ev_out, 0));  // dense bytes of batch b - depth copied out
        int r = launch_encode<Sym>(gt, s.d_syms, nb, chunk_len, s.d_slots, slot_cap, s.d_lens, p->d_status, sc,
                                   fast::ChunkInit{ini.kind, ini.seed + c0});
        if (r) return r;
        k_scan_lens<<<1, 1024, 0, sc>>>(s.d_lens, nc, s.d_offs);
        HIP_TRY(hipGetLastError());
        if (copy) {
            k_compact<<<grid_for(nc * 64), kBlock, 0, sc>>>(s.d_slots, slot_cap, s.d_lens, s.d_offs, nc, s.d_dense);
            HIP_TRY(hipGetLastError());
        }
        HIP_TRY(hipEventRecord(s.ev_comp, sc));
        HIP_TRY(hipMemcpyAsync(s.h_lens, s.d_lens, sizeof(uint32_t) * nc, hipMemcpyDeviceToHost, sc));
        HIP_TRY(hipMemcpyAsync(s.h_offs, s.d_offs + nc, sizeof(uint64_t), hipMemcpyDeviceToHost, sc));
        HIP_TRY(hipEventRecord(s.ev_meta, sc));
        s.used = true;
        return ANS_OK;
    };
    auto finish = [&](uint64_t b) -> int {
        PipeSlot& s = p->slot[b % p->depth];
        const uint64_t c0 = cuts[b], nc = cuts[b + 1] - c0;
        HIP_TRY(hipEventSynchronize(s.ev_meta));
        const uint64_t bt = s.h_offs[0];
        if (copy && acc + bt > out_cap) {
            copy = false;  // keep coding to report the exact total
            len_err = ANS_E_LEN;
        }
        if (copy && bt) HIP_TRY(hipMemcpyAsync(out + acc, s.d_dense, bt, hipMemcpyDeviceToHost, p->s_out));
        HIP_TRY(hipEventRecord(s.ev_out, p->s_out));
        uint64_t o = acc;
        for (uint64_t j = 0; j < nc; ++j) {
            if (out) {
                offsets[c0 + j] = o;
                lens[c0 + j] = s.h_lens[j];
            }
            o += s.h_lens[j];
        }
        acc = o;
        return ANS_OK;
    };
    for (uint64_t b = 0; b < nbatch; ++b) {
        if ((rc = enqueue(b))) return rc;
        if (b > 0 && (rc = finish(b - 1))) return rc;
    }
    if (nbatch && (rc = finish(nbatch - 1))) return rc;
    HIP_TRY(hipStreamSynchronize(p->s_out));
    HIP_TRY(hipStreamSynchronize(p->s_comp2));
    int st = 0;
    if ((rc = ans_dev_status(gt->g, p->d_status, gt->g->stream, &st))) return rc;
    if (st) return st;
    *total = acc;
    return len_err;
}

// Decode a host dense container into host symbols.  Batch b: its byte span and rebased
// offsets/lengths H2D (s_in) -> decode of the span in place (compute stream b & 1; the
// decoders read a dense container at any alignment, fast::DecChain::start) -> symbols D2H
// (s_out).  No host synchronisation inside the loop beyond staging reuse.
// Returns kPipeScattered when some batch's streams spread over more than twice its slot bytes
// (a container that is not dense); the caller then takes the whole-buffer path.
template <typename Sym>
int pipe_decode(ans_gpu_table* gt, const uint8_t* in, const uint64_t* offsets, const uint32_t* l32, uint64_t slot_cap,
                uint64_t n, uint64_t chunk_len, int gen_kind, void* out, fast::ChunkInit ini) {
    constexpr uint64_t w = sizeof(Sym);
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    const uint64_t B = pipe_batch_chunks(gt->g, nchunks, chunk_len * w);
    const std::vector<uint64_t> cuts = pipe_cuts(nchunks, B);
    const uint64_t nbatch = cuts.size() - 1;
    std::vector<uint64_t> lo(nbatch), span(nbatch);
    uint64_t max_span = 0;
    for (uint64_t b = 0; b < nbatch; ++b) {
        const uint64_t c0 = cuts[b], c1 = cuts[b + 1];
        uint64_t l = ~0ull, h = 0;
        for (uint64_t j = c0; j < c1; ++j) {
            l = std::min(l, offsets[j]);
            h = std::max(h, offsets[j] + l32[j]);
        }
        lo[b] = l;
        span[b] = h - l;
        max_span = std::max(max_span, span[b]);
    }
    if (max_span > 2 * B * slot_cap) return kPipeScattered;
    HostPipe* p = nullptr;
    int rc = pipe_get(gt->g, B * chunk_len * w, B * slot_cap, max_span, B, &p);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(p->d_status, 0, sizeof(uint32_t), gt->g->stream));
    HIP_TRY(hipStreamSynchronize(gt->g->stream));
    auto* dst = static_cast<uint8_t*>(out);
    for (uint64_t b = 0; b < nbatch; ++b) {
        PipeSlot& s = p->slot[b % p->depth];
        const hipStream_t sc = (b & 1) ? p->s_comp2 : gt->g->stream;
        const uint64_t c0 = cuts[b], nc = cuts[b + 1] - c0, n0 = c0 * chunk_len;
        const uint64_t nb = std::min(n - n0, nc * chunk_len);
        if (s.used) {
            HIP_TRY(hipEventSynchronize(s.ev_in));  // staging of batch b - depth uploaded
            HIP_TRY(hipStreamWaitEvent(p->s_in, s.ev_out, 0));  // its buffers drained
        }
        std::memcpy(s.h_lens, l32 + c0, sizeof(uint32_t) * nc);
        for (uint64_t j = 0; j < nc; ++j) s.h_offs[j] = offsets[c0 + j] - lo[b];  // into the batch's span
        if (span[b]) HIP_TRY(hipMemcpyAsync(s.d_dense, in + lo[b], span[b], hipMemcpyHostToDevice, p->s_in));
        HIP_TRY(hipMemcpyAsync(s.d_lens, s.h_lens, sizeof(uint32_t) * nc, hipMemcpyHostToDevice, p->s_in));
        HIP_TRY(hipMemcpyAsync(s.d_offs, s.h_offs, sizeof(uint64_t) * nc, hipMemcpyHostToDevice, p->s_in));
        HIP_TRY(hipEventRecord(s.ev_in, p->s_in));
        HIP_TRY(hipStreamWaitEvent(sc, s.ev_in, 0));
        if ((rc = launch_decode<Sym>(gt, s.d_dense, s.d_offs, slot_cap, s.d_lens, nb, chunk_len, gen_kind, s.d_syms,
                                     p->d_status, sc, fast::ChunkInit{ini.kind, ini.seed + c0})))
            return rc;
        HIP_TRY(hipEventRecord(s.ev_comp, sc));
        HIP_TRY(hipStreamWaitEvent(p->s_out, s.ev_comp, 0));
        HIP_TRY(hipMemcpyAsync(dst + n0 * w, s.d_syms, nb * w, hipMemcpyDeviceToHost, p->s_out));
        HIP_TRY(hipEventRecord(s.ev_out, p->s_out));
        s.used = true;
    }
    HIP_TRY(hipStreamSynchronize(p->s_out));
    HIP_TRY(hipStreamSynchronize(p->s_comp2));
    int st = 0;
    if ((rc = ans_dev_status(gt->g, p->d_status, gt->g->stream, &st))) return rc;
    return st;
}

// ---- page-locked host buffers: the GPU moves the bytes itself (no runtime copy calls)
//
// Page-locked host memory is mapped into the GPU's address space, so copy kernels can read
// and write it across PCIe directly (tools/pinned_probe.hip: ~41 GB/s each way with both
// directions in flight, ~55 GB/s alone).  The per-batch work then needs no host
// synchronisation at all: batch offsets are scanned and carried on the device, and the
// copy-out kernel reads its destination offset and size from device memory.

// Copy engine for page-locked buffers: the runtime's copies (default: measured faster,
// DESIGN.md §8) or these kernels (ANS_PIPE_COPY=kernel, the A/B switch behind that table).
bool pipe_kernel_copies() {
    const char* e = getenv("ANS_PIPE_COPY");  // read per call (tests switch it)
    return e && std::strcmp(e, "kernel") == 0;
}

// Device-visible address of a page-locked host pointer (nullptr for pageable memory).
uint8_t* mapped_ptr(const void* p) {
    if (!p) return nullptr;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
    return static_cast<uint8_t*>(a.devicePointer);
}

constexpr unsigned kXferGrid = 128;  // workgroups per copy kernel (probe: 64-256 saturate PCIe)

// dst[0..bytes) = src[0..bytes) between device memory and mapped host memory; 16-byte
// accesses when dst and src agree mod 16 (the pipeline arranges that), bytes otherwise.
__device__ __forceinline__ void xfer_bytes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t bytes) {
    const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t nth = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    if (((reinterpret_cast<uintptr_t>(dst) ^ reinterpret_cast<uintptr_t>(src)) & 15) == 0) {
        const uint64_t head = std::min<uint64_t>(bytes, (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15);
        if (tid < head) dst[tid] = src[tid];
        const uint64_t n16 = (bytes - head) / 16;
        uint4* d = reinterpret_cast<uint4*>(dst + head);
        const uint4* s = reinterpret_cast<const uint4*>(src + head);
        for (uint64_t i = tid; i < n16; i += nth) d[i] = s[i];
        const uint64_t done = head + 16 * n16;
        if (tid < bytes - done) dst[done + tid] = src[done + tid];
    } else {
        for (uint64_t i = tid; i < bytes; i += nth) dst[i] = src[i];
    }
}

__global__ __launch_bounds__(256) void k_xfer(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t bytes) {
    xfer_bytes(dst, src, bytes);
}

// Batch scan for the mapped encoder: like k_scan_lens, plus the running container offset.
// base = *acc (the bytes of all earlier batches), *acc += total; offs[n] = total,
// offs[n+1] = base; each chunk's absolute offset and length go to the host arrays.
__global__ __launch_bounds__(1024) void k_scan_carry(const uint32_t* __restrict__ lens, uint64_t n,
                                                     uint64_t* __restrict__ offs, uint64_t* __restrict__ acc,
                                                     uint64_t* __restrict__ h_offs, uint64_t* __restrict__ h_lens) {
    __shared__ uint64_t part[1024];
    __shared__ uint64_t base;
    const uint32_t t = threadIdx.x;
    if (t == 0) base = *acc;
    const uint64_t per = (n + 1023) / 1024, b = t * per, e = b + per < n ? b + per : n;
    uint64_t sum = 0;
    for (uint64_t i = b; i < e; ++i) sum += lens[i];
    part[t] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - sum;
    for (uint64_t i = b; i < e; ++i) {
        offs[i] = run;
        run += lens[i];
    }
    if (t == 1023) {
        offs[n] = part[1023];
        offs[n + 1] = base;
        *acc = base + part[1023];
    }
    __syncthreads();
    for (uint64_t i = t; i < n; i += 1024) {  // coalesced writes across PCIe
        h_offs[i] = base + offs[i];
        h_lens[i] = lens[i];
    }
}

// Slots -> dense bytes at dense + sh + offs[c], sh = (out + base) & 15 so that the copy-out
// kernel's source and destination agree mod 16.
__global__ __launch_bounds__(kBlock) void k_compact_at(const uint8_t* __restrict__ slots, uint64_t slot_cap,
                                                       const uint32_t* __restrict__ lens,
                                                       const uint64_t* __restrict__ offs, uint64_t nchunks,
                                                       uintptr_t out_addr, uint8_t* __restrict__ dense) {
    const uint64_t c = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (c >= nchunks) return;
    const uint64_t sh = (out_addr + offs[nchunks + 1]) & 15;
    const uint8_t* s = slots + c * slot_cap;
    uint8_t* d = dense + sh + offs[c];
    wave_copy(d, s, static_cast<uint32_t>(min<uint64_t>(lens[c], slot_cap)), lane);
}

// Copy-out of one encoded batch to out + base (size and base from the scan); a batch that
// would overrun out_cap is not copied and flags ANS_E_LEN (coding continues, so the exact
// total is still known).
__global__ __launch_bounds__(256) void k_xfer_out(uint8_t* __restrict__ out, uint64_t out_cap,
                                                  const uint8_t* __restrict__ dense, const uint64_t* __restrict__ offs,
                                                  uint64_t nchunks, uint32_t* __restrict__ status) {
    const uint64_t total = offs[nchunks], base = offs[nchunks + 1];
    if (base + total > out_cap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(status, 1u << ANS_E_LEN);
        return;
    }
    const uint64_t sh = (reinterpret_cast<uintptr_t>(out) + base) & 15;
    xfer_bytes(out + base, dense + sh, total);
}

// Dense batch bytes (at dense + sh, sh = (in + lo) & 15) -> slots; the chunk offsets and
// lengths are read from the mapped host staging, lengths also land in d_lens for the decoder.
__global__ __launch_bounds__(kBlock) void k_expand_mapped(const uint8_t* __restrict__ dense, uint64_t sh, uint64_t lo,
                                                          const uint64_t* __restrict__ h_offs,
                                                          const uint64_t* __restrict__ h_lens, uint64_t nchunks,
                                                          uint32_t* __restrict__ d_lens, uint8_t* __restrict__ slots,
                                                          uint64_t slot_cap) {
    const uint64_t c = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (c >= nchunks) return;
    const uint64_t off = h_offs[c];
    const uint32_t len = static_cast<uint32_t>(h_lens[c]);
    if (lane == 0) d_lens[c] = len;
    const uint8_t* s = dense + sh + (off - lo);
    uint8_t* d = slots + c * slot_cap;
    wave_copy(d, s, len, lane);
}

// Host staging (mapped) for 2 x u64 per chunk of a whole call, and the device carry word.
int pipe_meta(HostPipe* p, uint64_t nchunks) {
    if (!p->d_acc) HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p->d_acc), 16));
    if (!p->ev_scan) HIP_TRY(hipEventCreateWithFlags(&p->ev_scan, hipEventDisableTiming));
    if (nchunks > p->cap_meta) {
        HIP_TRY(hipDeviceSynchronize());
        if (p->h_meta) (void)hipHostFree(p->h_meta);
        p->h_meta = nullptr;
        p->cap_meta = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&p->h_meta), 2 * sizeof(uint64_t) * nchunks + 16));
        p->cap_meta = nchunks;
    }
    return ANS_OK;
}

// Encode with page-locked symbols and container.  Batch b: symbols in (k_xfer on s_in) ->
// encode, carried scan, compaction (compute stream b & 1) -> container bytes out
// (k_xfer_out on s_out).  The host only waits at the end.
template <typename Sym>
int pipe_encode_mapped(ans_gpu_table* gt, const uint8_t* syms_dev, uint64_t n, uint64_t chunk_len, uint8_t* out_dev,
                       uint64_t out_cap, uint64_t* offsets, uint64_t* lens, uint64_t* total, fast::ChunkInit ini) {
    constexpr uint64_t w = sizeof(Sym);
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    uint64_t slot_cap = 0;
    ans_gpu_slot_capacity(gt, chunk_len, &slot_cap);
    const uint64_t B = pipe_batch_chunks(gt->g, nchunks, chunk_len * w);
    HostPipe* p = nullptr;
    int rc = pipe_get(gt->g, B * chunk_len * w, B * slot_cap, out_dev ? B * slot_cap + 16 : 0, B + 1, &p);
    if (rc || (rc = pipe_meta(p, nchunks))) return rc;
    uint64_t* h_offs = p->h_meta;
    uint64_t* h_lens = p->h_meta + nchunks;
    const hipStream_t s0 = gt->g->stream;
    HIP_TRY(hipMemsetAsync(p->d_status, 0, sizeof(uint32_t), s0));
    HIP_TRY(hipMemsetAsync(p->d_acc, 0, sizeof(uint64_t), s0));
    HIP_TRY(hipStreamSynchronize(s0));
    const uint64_t nbatch = (nchunks + B - 1) / B;
    for (uint64_t b = 0; b < nbatch; ++b) {
        PipeSlot& s = p->slot[b % p->depth];
        const hipStream_t sc = (b & 1) ? p->s_comp2 : s0;
        const uint64_t c0 = b * B, nc = std::min(B, nchunks - c0), n0 = c0 * chunk_len;
        const uint64_t nb = std::min(n - n0, nc * chunk_len);
        if (s.used) HIP_TRY(hipStreamWaitEvent(p->s_in, s.ev_comp, 0));  // symbols of batch b - depth consumed
        k_xfer<<<kXferGrid, 256, 0, p->s_in>>>(static_cast<uint8_t*>(s.d_syms), syms_dev + n0 * w, nb * w);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(s.ev_in, p->s_in));
        HIP_TRY(hipStreamWaitEvent(sc, s.ev_in, 0));
        if (s.used) HIP_TRY(hipStreamWaitEvent(sc, s.ev_out, 0));  // dense bytes of batch b - depth copied out
        if ((rc = launch_encode<Sym>(gt, s.d_syms, nb, chunk_len, s.d_slots, slot_cap, s.d_lens, p->d_status, sc,
                                     fast::ChunkInit{ini.kind, ini.seed + c0})))
            return rc;
        if (b > 0) HIP_TRY(hipStreamWaitEvent(sc, p->ev_scan, 0));  // the carry runs in batch order
        k_scan_carry<<<1, 1024, 0, sc>>>(s.d_lens, nc, s.d_offs, p->d_acc, h_offs + c0, h_lens + c0);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(p->ev_scan, sc));
        if (out_dev) {
            k_compact_at<<<grid_for(nc * 64), kBlock, 0, sc>>>(s.d_slots, slot_cap, s.d_lens, s.d_offs, nc,
                                                               reinterpret_cast<uintptr_t>(out_dev), s.d_dense);
            HIP_TRY(hipGetLastError());
        }
        HIP_TRY(hipEventRecord(s.ev_comp, sc));
        HIP_TRY(hipStreamWaitEvent(p->s_out, s.ev_comp, 0));
        if (out_dev) {
            k_xfer_out<<<kXferGrid, 256, 0, p->s_out>>>(out_dev, out_cap, s.d_dense, s.d_offs, nc, p->d_status);
            HIP_TRY(hipGetLastError());
        }
        HIP_TRY(hipEventRecord(s.ev_out, p->s_out));
        s.used = true;
    }
    HIP_TRY(hipStreamSynchronize(p->s_out));
    HIP_TRY(hipStreamSynchronize(p->s_comp2));
    HIP_TRY(hipStreamSynchronize(s0));
    uint32_t bits = 0;
    uint64_t acc = 0;
    HIP_TRY(hipMemcpy(&bits, p->d_status, sizeof(bits), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&acc, p->d_acc, sizeof(acc), hipMemcpyDeviceToHost));
    const int st = lowest_status(bits & ~(1u << ANS_E_LEN));
    if (st) return st;
    *total = acc;
    if (!out_dev) return ANS_OK;
    std::memcpy(offsets, h_offs, sizeof(uint64_t) * nchunks);
    std::memcpy(lens, h_lens, sizeof(uint64_t) * nchunks);
    return (bits & (1u << ANS_E_LEN)) ? ANS_E_LEN : ANS_OK;
}

// Decode from a page-locked container into page-locked symbols.  Batch b: its byte span in
// (k_xfer on s_in) -> expansion (offsets and lengths read from the mapped staging) and
// decode (compute stream b & 1) -> symbols out (k_xfer on s_out).  No host waits in the loop.
template <typename Sym>
int pipe_decode_mapped(ans_gpu_table* gt, const uint8_t* in_dev, const uint64_t* offsets, const uint32_t* l32,
                       uint64_t slot_cap, uint64_t n, uint64_t chunk_len, int gen_kind, uint8_t* out_dev,
                       fast::ChunkInit ini) {
    constexpr uint64_t w = sizeof(Sym);
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    const uint64_t B = pipe_batch_chunks(gt->g, nchunks, chunk_len * w);
    const uint64_t nbatch = (nchunks + B - 1) / B;
    std::vector<uint64_t> lo(nbatch), span(nbatch);
    uint64_t max_span = 0;
    for (uint64_t b = 0; b < nbatch; ++b) {
        const uint64_t c0 = b * B, c1 = std::min(nchunks, c0 + B);
        uint64_t l = ~0ull, h = 0;
        for (uint64_t j = c0; j < c1; ++j) {
            l = std::min(l, offsets[j]);
            h = std::max(h, offsets[j] + l32[j]);
        }
        lo[b] = l;
        span[b] = h - l;
        max_span = std::max(max_span, span[b]);
    }
    if (max_span > 2 * B * slot_cap) return kPipeScattered;
    HostPipe* p = nullptr;
    int rc = pipe_get(gt->g, B * chunk_len * w, B * slot_cap, max_span + 16, B + 1, &p);
    if (rc || (rc = pipe_meta(p, nchunks))) return rc;
    uint64_t* h_offs = p->h_meta;
    uint64_t* h_lens = p->h_meta + nchunks;
    std::memcpy(h_offs, offsets, sizeof(uint64_t) * nchunks);
    for (uint64_t j = 0; j < nchunks; ++j) h_lens[j] = l32[j];
    const hipStream_t s0 = gt->g->stream;
    HIP_TRY(hipMemsetAsync(p->d_status, 0, sizeof(uint32_t), s0));
    HIP_TRY(hipStreamSynchronize(s0));
    for (uint64_t b = 0; b < nbatch; ++b) {
        PipeSlot& s = p->slot[b % p->depth];
        const hipStream_t sc = (b & 1) ? p->s_comp2 : s0;
        const uint64_t c0 = b * B, nc = std::min(B, nchunks - c0), n0 = c0 * chunk_len;
        const uint64_t nb = std::min(n - n0, nc * chunk_len);
        const uint64_t sh = reinterpret_cast<uintptr_t>(in_dev + lo[b]) & 15;
        if (s.used) HIP_TRY(hipStreamWaitEvent(p->s_in, s.ev_out, 0));  // batch b - depth drained
        k_xfer<<<kXferGrid, 256, 0, p->s_in>>>(s.d_dense + sh, in_dev + lo[b], span[b]);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(s.ev_in, p->s_in));
        HIP_TRY(hipStreamWaitEvent(sc, s.ev_in, 0));
        k_expand_mapped<<<grid_for(nc * 64), kBlock, 0, sc>>>(s.d_dense, sh, lo[b], h_offs + c0, h_lens + c0, nc,
                                                              s.d_lens, s.d_slots, slot_cap);
        HIP_TRY(hipGetLastError());
        if ((rc = launch_decode<Sym>(gt, s.d_slots, nullptr, slot_cap, s.d_lens, nb, chunk_len, gen_kind, s.d_syms,
                                     p->d_status, sc, fast::ChunkInit{ini.kind, ini.seed + c0})))
            return rc;
        HIP_TRY(hipEventRecord(s.ev_comp, sc));
        HIP_TRY(hipStreamWaitEvent(p->s_out, s.ev_comp, 0));
        k_xfer<<<kXferGrid, 256, 0, p->s_out>>>(out_dev + n0 * w, static_cast<const uint8_t*>(s.d_syms), nb * w);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(s.ev_out, p->s_out));
        s.used = true;
    }
    HIP_TRY(hipStreamSynchronize(p->s_out));
    HIP_TRY(hipStreamSynchronize(p->s_comp2));
    int st = 0;
    if ((rc = ans_dev_status(gt->g, p->d_status, s0, &st))) return rc;
    return st;
}

}  // namespace

// Variable-chunk encode of symbols already on the device (ans_ctx.hpp): the body of
// ans_gpu_encode_var_chunks, also used by the graph dataset coder (ans_graph.hip).
int ans_encode_var_from_device(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t nchunks,
                               const uint64_t* starts, uint8_t* out, uint64_t out_cap, uint64_t* offsets,
                               uint64_t* lens, uint64_t* total, int gen_kind, uint64_t seed) {
    if (out && nchunks && (!offsets || !lens)) return ANS_E_ARG;
    *total = 0;
    if (nchunks == 0) return ANS_OK;
    uint64_t maxlen = 0;
    for (uint64_t c = 0; c < nchunks; ++c) maxlen = std::max(maxlen, starts[c + 1] - starts[c]);
    uint64_t slot_cap = 0;
    ans_gpu_slot_capacity(gt, maxlen, &slot_cap);
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = gt->g->stream;
    DevBuf d_starts, d_slots, d_lens, d_status, d_offs, d_out;
    HIP_TRY(d_starts.alloc(8 * (nchunks + 1)));
    HIP_TRY(d_slots.alloc(nchunks * slot_cap));
    HIP_TRY(d_lens.alloc(4 * nchunks));
    HIP_TRY(d_status.alloc(4));
    HIP_TRY(hipMemcpyAsync(d_starts.p, starts, 8 * (nchunks + 1), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(d_status.p, 0, 4, s));
    int rc = dev_encode_var(gt, d_syms, sym_bytes, nchunks, static_cast<uint64_t*>(d_starts.p), gen_kind, seed,
                            static_cast<uint8_t*>(d_slots.p), slot_cap, static_cast<uint32_t*>(d_lens.p),
                            static_cast<uint32_t*>(d_status.p), s,
                            staged_lmax(nchunks, maxlen, starts[nchunks] - starts[0], sym_bytes));
    if (rc) return rc;
    int st = 0;
    if ((rc = ans_dev_status(gt->g, static_cast<uint32_t*>(d_status.p), s, &st))) return rc;
    if (st) return st;
    std::vector<uint32_t> hl(nchunks);
    HIP_TRY(hipMemcpy(hl.data(), d_lens.p, 4 * nchunks, hipMemcpyDeviceToHost));
    std::vector<uint64_t> off(nchunks);
    uint64_t acc = 0;
    for (uint64_t c = 0; c < nchunks; ++c) {
        off[c] = acc;
        acc += hl[c];
    }
    *total = acc;
    if (!out) return ANS_OK;
    if (out_cap < acc) return ANS_E_LEN;
    for (uint64_t c = 0; c < nchunks; ++c) {
        offsets[c] = off[c];
        lens[c] = hl[c];
    }
    if (!acc) return ANS_OK;
    HIP_TRY(d_offs.alloc(8 * nchunks));
    HIP_TRY(d_out.alloc(acc));
    HIP_TRY(hipMemcpyAsync(d_offs.p, off.data(), 8 * nchunks, hipMemcpyHostToDevice, s));
    if ((rc = ans_dev_compact(gt->g, static_cast<uint8_t*>(d_slots.p), slot_cap, static_cast<uint32_t*>(d_lens.p),
                              static_cast<uint64_t*>(d_offs.p), nchunks, static_cast<uint8_t*>(d_out.p), s)))
        return rc;
    HIP_TRY(hipMemcpyAsync(out, d_out.p, acc, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return ANS_OK;
}

// ====================================================================== C ABI (GPU part)
extern "C" {

int ans_gpu_device_count(int* count) try {
    if (!count) return ANS_E_ARG;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return ANS_OK;
} ANS_CATCH

int ans_gpu_create(int device, ans_gpu** out) try {
    if (!out) return ANS_E_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return ANS_E_DEVICE;
    HIP_TRY(hipSetDevice(device));
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0) ncu = 256;
    auto* g = new (std::nothrow) ans_gpu{device, ncu, nullptr, nullptr, 0, nullptr, 0};
    if (!g) return ANS_E_ALLOC;
    if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
        delete g;
        return ANS_E_DEVICE;
    }
    *out = g;
    return ANS_OK;
} ANS_CATCH

int ans_host_alloc(size_t bytes, void** out) try {
    if (!out) return ANS_E_ARG;
    *out = nullptr;
    if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return ANS_E_ALLOC;
    }
    return ANS_OK;
} ANS_CATCH

void ans_host_free(void* p) try {
    if (p) (void)hipHostFree(p);
} ANS_CATCH_VOID

int ans_gpu_set_batch_bytes(ans_gpu* g, uint64_t batch_bytes) try {
    if (!g) return ANS_E_ARG;
    g->batch_bytes = batch_bytes;
    return ANS_OK;
} ANS_CATCH

int ans_gpu_pipe_depth(const ans_gpu* g, int* depth) try {
    if (!g || !depth) return ANS_E_ARG;
    *depth = g->pipe ? g->pipe->depth : 0;
    return ANS_OK;
} ANS_CATCH

void ans_gpu_free(ans_gpu* g) try {
    if (!g) return;
    (void)hipSetDevice(g->device);
    pipe_free(g);
    if (g->d_scratch) (void)hipFree(g->d_scratch);
    (void)hipStreamDestroy(g->stream);
    delete g;
} ANS_CATCH_VOID

int ans_gpu_table_create(ans_gpu* g, const ans_table* tab, ans_gpu_table** out) try {
    if (!g || !tab || !out) return ANS_E_ARG;
    *out = nullptr;
    const Categorical& cat = tab->cat;
    const uint64_t nsym = cat.masses.size();
    if (nsym == 0 || cat.norm() == 0 || cat.norm() > kMaxMinHead) return ANS_E_NORM_RANGE;
    if (nsym > 65536 || cat.norm() >= (1ull << 32)) {  // the exact 64-bit kernels (ans_codecs.hip)
        const Categorical* one = &cat;
        ans_gpu_tableset* ts = nullptr;
        const int rc = ans_tableset_build(g, &one, 1, &ts);
        if (rc) return rc;
        DevTable t{};
        t.nsym = nsym > 0xFFFFFFFFull ? 0xFFFFFFFFu : static_cast<uint32_t>(nsym);
        auto* gt = new (std::nothrow) ans_gpu_table{g, g->device, t, nullptr, 0, FastTable{}, nullptr, ts};
        if (!gt) {
            ans_tableset_destroy(ts);
            return ANS_E_ALLOC;
        }
        *out = gt;
        return ANS_OK;
    }
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
    auto* gt = new (std::nothrow) ans_gpu_table{g, g->device, t, mem, 0, FastTable{}, nullptr, nullptr};
    if (!gt) { (void)hipFree(mem); return ANS_E_ALLOC; }
    if (rows_bytes + bucket_bytes <= kLdsTableLimit) gt->lds_bytes = static_cast<uint32_t>(rows_bytes + bucket_bytes);
    const int rc = build_fast_table(gt, cat);
    if (rc) {
        ans_gpu_table_free(gt);
        return rc;
    }
    *out = gt;
    return ANS_OK;
} ANS_CATCH

void ans_gpu_table_free(ans_gpu_table* gt) try {
    if (!gt) return;
    (void)hipSetDevice(gt->device);  // (not gt->g: a table may be freed after its context)
    if (gt->ts64) ans_tableset_destroy(gt->ts64);
    if (gt->d_mem) (void)hipFree(gt->d_mem);
    if (gt->d_fast) (void)hipFree(gt->d_fast);
    delete gt;
} ANS_CATCH_VOID

int ans_gpu_table_paths(const ans_gpu_table* gt, uint32_t* paths) try {
    if (!gt || !paths) return ANS_E_ARG;
    const FastTable& ft = gt->ft;
    uint32_t p = 0;
    if (ft.usable) p |= ft.enc_global ? ANS_PATH_ENC_GLOBAL : ANS_PATH_ENC_LDS;
    if (ft.usable && ft.dec_usable) p |= ANS_PATH_DEC_LDS;
    if (ft.usable && ft.dec_global) p |= ANS_PATH_DEC_GLOBAL;
    if (ft.usable && ft.enc_wide) p |= ANS_PATH_ENC_WIDE;
    if (ft.usable && ft.dec_wide) p |= ANS_PATH_DEC_WIDE;
    if (ft.usable && ft.dec_wide && ft.dec_c) p |= ANS_PATH_DEC_COMPACT;
    if (ft.usable && ft.enc_wide && ft.enc_pack) p |= ANS_PATH_ENC_PACKED;
    if (ft.usable && ft.enc_wide && ft.enc_sa) p |= ANS_PATH_ENC_SHIFT;
    if (ft.usable && ft.dec_usable && !ft.dec_far && ft.dec_u) p |= ANS_PATH_DEC_U;
    *paths = p;
    return ANS_OK;
} ANS_CATCH

int ans_gpu_slot_capacity(const ans_gpu_table* gt, uint64_t chunk_len, uint64_t* slot_cap) try {
    if (!gt || !slot_cap) return ANS_E_ARG;
    if (gt->ts64) {
        *slot_cap = ans_tableset_slot_bytes(gt->ts64, chunk_len);
        return ANS_OK;
    }
    // Bytes of one flattened chunk <= (sum_i log2(norm/p_i) + 1 + L*log2(1+1/K)) / 8 + 8
    // (virtual-bits argument); take every p_i = pmin, plus margin.
    const double per_sym = std::log2(static_cast<double>(gt->t.norm) / static_cast<double>(gt->t.pmin)) +
                           2.0 / static_cast<double>(gt->t.K) + 1e-6;
    const double bytes = (static_cast<double>(chunk_len) * per_sym + 2.0) / 8.0 + 9.0;
    // + one page of slack: the fast encoder writes whole 64-byte pages (ans_fast.hpp)
    const uint64_t cap = static_cast<uint64_t>(std::ceil(bytes)) + 8 + 64;
    *slot_cap = (cap + 127) & ~uint64_t(127);
    return ANS_OK;
} ANS_CATCH

int ans_dev_encode_chunks_ex(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                             int gen_kind, uint64_t seed, uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens,
                             uint32_t* d_status, void* stream) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !d_status || !valid_width(sym_bytes) || chunk_len == 0 || (slot_cap & 15) || !valid_kind(gen_kind))
        return ANS_E_ARG;
    if (n && (!d_syms || !d_slots || !d_lens)) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = pick(gt, stream);
    if (gt->ts64)
        return ans_tableset_dev_encode(gt->ts64, d_syms, sym_bytes, nullptr, n, chunk_len, (n + chunk_len - 1) / chunk_len,
                                       d_slots, slot_cap, d_lens, d_status, gen_kind, seed, s);
    const fast::ChunkInit ini{gen_kind, seed};
    switch (sym_bytes) {
    case 1: return launch_encode<uint8_t>(gt, d_syms, n, chunk_len, d_slots, slot_cap, d_lens, d_status, s, ini);
    case 2: return launch_encode<uint16_t>(gt, d_syms, n, chunk_len, d_slots, slot_cap, d_lens, d_status, s, ini);
    default: return launch_encode<uint32_t>(gt, d_syms, n, chunk_len, d_slots, slot_cap, d_lens, d_status, s, ini);
    }
} ANS_CATCH

int ans_dev_encode_chunks(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                          uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens, uint32_t* d_status, void* stream) try {
    return ans_dev_encode_chunks_ex(gt, d_syms, sym_bytes, n, chunk_len, ANS_GEN_ZEROS, 0, d_slots, slot_cap, d_lens,
                                    d_status, stream);
} ANS_CATCH

int ans_dev_decode_chunks_ex(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap,
                             const uint32_t* d_lens, uint64_t n, uint64_t chunk_len, int gen_kind, uint64_t seed,
                             void* d_syms, int sym_bytes, uint32_t* d_status, void* stream) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !d_status || !valid_width(sym_bytes) || chunk_len == 0 || !valid_kind(gen_kind)) return ANS_E_ARG;
    if (n && (!d_in || !d_lens || !d_syms)) return ANS_E_ARG;
    if (sym_bytes == 1 && gt->t.nsym > 256) return ANS_E_ARG;
    if (sym_bytes == 2 && gt->t.nsym > 65536) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = pick(gt, stream);
    if (gt->ts64)
        return ans_tableset_dev_decode(gt->ts64, d_in, d_offsets, slot_cap, d_lens, nullptr, n, chunk_len,
                                       (n + chunk_len - 1) / chunk_len, gen_kind, seed, d_syms, sym_bytes, d_status, s);
    const fast::ChunkInit ini{gen_kind, seed};
    switch (sym_bytes) {
    case 1: return launch_decode<uint8_t>(gt, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, gen_kind, d_syms, d_status, s, ini);
    case 2: return launch_decode<uint16_t>(gt, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, gen_kind, d_syms, d_status, s, ini);
    default: return launch_decode<uint32_t>(gt, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, gen_kind, d_syms, d_status, s, ini);
    }
} ANS_CATCH

int ans_dev_decode_chunks(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap,
                          const uint32_t* d_lens, uint64_t n, uint64_t chunk_len, int gen_kind, void* d_syms,
                          int sym_bytes, uint32_t* d_status, void* stream) try {
    if (gen_kind != ANS_GEN_ZEROS && gen_kind != ANS_GEN_EMPTY) return ANS_E_ARG;  // RANDOM needs a seed: _ex
    return ans_dev_decode_chunks_ex(gt, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, gen_kind, 0, d_syms, sym_bytes,
                                    d_status, stream);
} ANS_CATCH

int ans_dev_gen_iid(ans_gpu_table* gt, uint64_t seed, uint64_t start, uint64_t n, void* d_syms, int sym_bytes,
                    void* stream) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !valid_width(sym_bytes) || (n && !d_syms)) return ANS_E_ARG;
    if (gt->ts64) return ANS_E_NORM_RANGE;  // the synthetic generator reads u32 tables
    if (sym_bytes == 1 && gt->t.nsym > 256) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = pick(gt, stream);
    switch (sym_bytes) {
    case 1: return launch_gen<uint8_t>(gt, seed, start, n, d_syms, s);
    case 2: return launch_gen<uint16_t>(gt, seed, start, n, d_syms, s);
    default: return launch_gen<uint32_t>(gt, seed, start, n, d_syms, s);
    }
} ANS_CATCH

int ans_dev_check_renorm(ans_gpu* g, const uint64_t* d_heads, const uint32_t* d_windows, uint64_t L, uint64_t n,
                         uint64_t* d_out_heads, uint32_t* d_out_k, void* stream) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!g || (n && (!d_heads || !d_windows || !d_out_heads || !d_out_k))) return ANS_E_ARG;
    if (n == 0) return ANS_OK;
    HIP_TRY(hipSetDevice(g->device));
    const hipStream_t s = stream ? static_cast<hipStream_t>(stream) : g->stream;
    k_check_renorm<<<static_cast<unsigned>((n + 255) / 256), 256, 0, s>>>(d_heads, d_windows, L, n, d_out_heads, d_out_k);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
} ANS_CATCH

int ans_dev_sample_iid(ans_gpu_table* gt, uint64_t seed, uint64_t n, uint64_t chunk_len, void* d_syms, int sym_bytes,
                       void* stream) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !valid_width(sym_bytes) || chunk_len == 0 || (n && !d_syms)) return ANS_E_ARG;
    if (gt->ts64) return ANS_E_NORM_RANGE;  // the sampler reads u32 tables
    if (sym_bytes == 1 && gt->t.nsym > 256) return ANS_E_ARG;
    if (sym_bytes == 2 && gt->t.nsym > 65536) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = pick(gt, stream);
    switch (sym_bytes) {
    case 1: return launch_sample<uint8_t>(gt, seed, n, chunk_len, d_syms, s);
    case 2: return launch_sample<uint16_t>(gt, seed, n, chunk_len, d_syms, s);
    default: return launch_sample<uint32_t>(gt, seed, n, chunk_len, d_syms, s);
    }
} ANS_CATCH

int ans_gpu_sample_iid(ans_gpu_table* gt, uint64_t seed, uint64_t n, uint64_t chunk_len, void* out, int sym_bytes) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !valid_width(sym_bytes) || chunk_len == 0 || (n && !out)) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    DevBuf d;
    HIP_TRY(d.alloc(n * sym_bytes));
    const int rc = ans_dev_sample_iid(gt, seed, n, chunk_len, d.p, sym_bytes, nullptr);
    if (rc) return rc;
    if (n) HIP_TRY(hipMemcpyAsync(out, d.p, n * sym_bytes, hipMemcpyDeviceToHost, gt->g->stream));
    HIP_TRY(hipStreamSynchronize(gt->g->stream));
    return ANS_OK;
} ANS_CATCH

// The longest variable chunk and the total of device-resident starts (one workgroup: a strided
// max per lane, a wave shfl_xor reduction, the 16 wave maxima through LDS) -> out[0], out[1].
__global__ __launch_bounds__(1024) void k_span_stats(const uint64_t* __restrict__ starts, uint64_t nchunks,
                                                    uint64_t* __restrict__ out) {
    __shared__ uint64_t part[16];
    uint64_t m = 0;
    for (uint64_t c = threadIdx.x; c < nchunks; c += 1024) {
        const uint64_t a = starts[c], b = starts[c + 1];
        m = max(m, b >= a ? b - a : ~0ull);  // decreasing starts: no staging (the kernels report them)
    }
    for (int d = 32; d >= 1; d >>= 1) m = max(m, static_cast<uint64_t>(__shfl_xor(m, d)));
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) m = max(m, part[w]);
        out[0] = m;
        out[1] = starts[nchunks] - starts[0];
    }
}

// staged_lmax for device-resident starts: k_span_stats, one 16-B copy back and a stream
// synchronisation (the device API's variable chunks then take the staged fast kernels, as the
// host API's do); 0 (the generic kernels) when the staged layout would exceed the budget
static int device_lmax(const uint64_t* d_starts, uint64_t nchunks, int sym_bytes, hipStream_t s, uint64_t* lmax) {
    *lmax = 0;
    if (nchunks == 0) return ANS_OK;
    void* mem = nullptr;
    if (hipMallocAsync(&mem, 16, s) != hipSuccess) {
        (void)hipGetLastError();
        return ANS_OK;  // the generic kernels
    }
    uint64_t h[2] = {0, 0};
    k_span_stats<<<1, 1024, 0, s>>>(d_starts, nchunks, static_cast<uint64_t*>(mem));
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(h, mem, 16, hipMemcpyDeviceToHost, s);
    const hipError_t f = hipFreeAsync(mem, s);
    if (e == hipSuccess) e = f;
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    HIP_TRY(e);
    *lmax = (h[0] >> 32) ? 0 : staged_lmax(nchunks, h[0], h[1], sym_bytes);
    return ANS_OK;
}

// lmax > 0 (the longest chunk): the staged fast kernels where the table has them
// (launch_staged_encode); the device API finds it with device_lmax
int dev_encode_var(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t nchunks,
                          const uint64_t* d_starts, int gen_kind, uint64_t seed, uint8_t* d_slots, uint64_t slot_cap,
                          uint32_t* d_lens, uint32_t* d_status, void* stream, uint64_t lmax) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !d_status || !valid_width(sym_bytes) || (slot_cap & 15) || !valid_kind(gen_kind)) return ANS_E_ARG;
    if (nchunks && (!d_syms || !d_starts || !d_slots || !d_lens)) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = pick(gt, stream);
    if (gt->ts64)
        return ans_tableset_dev_encode(gt->ts64, d_syms, sym_bytes, d_starts, 0, 0, nchunks, d_slots, slot_cap, d_lens,
                                       d_status, gen_kind, seed, s);
    const fast::ChunkInit ini{gen_kind, seed};
    switch (sym_bytes) {
    case 1: return launch_encode_var<uint8_t>(gt, d_syms, nchunks, d_starts, d_slots, slot_cap, d_lens, d_status, s, ini, lmax);
    case 2: return launch_encode_var<uint16_t>(gt, d_syms, nchunks, d_starts, d_slots, slot_cap, d_lens, d_status, s, ini, lmax);
    default: return launch_encode_var<uint32_t>(gt, d_syms, nchunks, d_starts, d_slots, slot_cap, d_lens, d_status, s, ini, lmax);
    }
} ANS_CATCH

int ans_dev_encode_var_chunks_ex(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t nchunks,
                                 const uint64_t* d_starts, int gen_kind, uint64_t seed, uint8_t* d_slots,
                                 uint64_t slot_cap, uint32_t* d_lens, uint32_t* d_status, void* stream) try {
    (void)hipGetLastError();
    if (!gt || !valid_width(sym_bytes)) return ANS_E_ARG;
    if (nchunks && !d_starts) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    uint64_t lmax = 0;
    if (!gt->ts64) {
        const int rc = device_lmax(d_starts, nchunks, sym_bytes, pick(gt, stream), &lmax);
        if (rc) return rc;
    }
    return dev_encode_var(gt, d_syms, sym_bytes, nchunks, d_starts, gen_kind, seed, d_slots, slot_cap, d_lens, d_status,
                          stream, lmax);
} ANS_CATCH

int ans_dev_encode_var_chunks(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t nchunks,
                              const uint64_t* d_starts, uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens,
                              uint32_t* d_status, void* stream) try {
    return ans_dev_encode_var_chunks_ex(gt, d_syms, sym_bytes, nchunks, d_starts, ANS_GEN_ZEROS, 0, d_slots, slot_cap,
                                        d_lens, d_status, stream);
} ANS_CATCH

int dev_decode_var(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap,
                          const uint32_t* d_lens, uint64_t nchunks, const uint64_t* d_starts, int gen_kind,
                          uint64_t seed, void* d_syms, int sym_bytes, uint32_t* d_status, void* stream, uint64_t lmax) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !d_status || !valid_width(sym_bytes) || !valid_kind(gen_kind)) return ANS_E_ARG;
    if (nchunks && (!d_in || !d_lens || !d_starts || !d_syms)) return ANS_E_ARG;
    if ((sym_bytes == 1 && gt->t.nsym > 256) || (sym_bytes == 2 && gt->t.nsym > 65536)) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = pick(gt, stream);
    if (gt->ts64)
        return ans_tableset_dev_decode(gt->ts64, d_in, d_offsets, slot_cap, d_lens, d_starts, 0, 0, nchunks, gen_kind,
                                       seed, d_syms, sym_bytes, d_status, s);
    const fast::ChunkInit ini{gen_kind, seed};
    switch (sym_bytes) {
    case 1: return launch_decode_var<uint8_t>(gt, d_in, d_offsets, slot_cap, d_lens, nchunks, d_starts, gen_kind, d_syms, d_status, s, ini, lmax);
    case 2: return launch_decode_var<uint16_t>(gt, d_in, d_offsets, slot_cap, d_lens, nchunks, d_starts, gen_kind, d_syms, d_status, s, ini, lmax);
    default: return launch_decode_var<uint32_t>(gt, d_in, d_offsets, slot_cap, d_lens, nchunks, d_starts, gen_kind, d_syms, d_status, s, ini, lmax);
    }
} ANS_CATCH

int ans_dev_decode_var_chunks_ex(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap,
                                 const uint32_t* d_lens, uint64_t nchunks, const uint64_t* d_starts, int gen_kind,
                                 uint64_t seed, void* d_syms, int sym_bytes, uint32_t* d_status, void* stream) try {
    (void)hipGetLastError();
    if (!gt || !valid_width(sym_bytes)) return ANS_E_ARG;
    if (nchunks && !d_starts) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    uint64_t lmax = 0;
    if (!gt->ts64) {
        const int rc = device_lmax(d_starts, nchunks, sym_bytes, pick(gt, stream), &lmax);
        if (rc) return rc;
    }
    return dev_decode_var(gt, d_in, d_offsets, slot_cap, d_lens, nchunks, d_starts, gen_kind, seed, d_syms, sym_bytes,
                          d_status, stream, lmax);
} ANS_CATCH

int ans_dev_decode_var_chunks(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap,
                              const uint32_t* d_lens, uint64_t nchunks, const uint64_t* d_starts, int gen_kind,
                              void* d_syms, int sym_bytes, uint32_t* d_status, void* stream) try {
    if (gen_kind != ANS_GEN_ZEROS && gen_kind != ANS_GEN_EMPTY) return ANS_E_ARG;  // RANDOM needs a seed: _ex
    return ans_dev_decode_var_chunks_ex(gt, d_in, d_offsets, slot_cap, d_lens, nchunks, d_starts, gen_kind, 0, d_syms,
                                        sym_bytes, d_status, stream);
} ANS_CATCH

int ans_gpu_encode_var_chunks_ex(ans_gpu_table* gt, const void* syms, int sym_bytes, uint64_t nchunks,
                                 const uint64_t* starts, int gen_kind, uint64_t seed, uint8_t* out, uint64_t out_cap,
                                 uint64_t* offsets, uint64_t* lens, uint64_t* total) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !valid_width(sym_bytes) || !total || (nchunks && !starts) || !valid_kind(gen_kind)) return ANS_E_ARG;
    *total = 0;
    if (nchunks == 0) return ANS_OK;
    for (uint64_t c = 0; c < nchunks; ++c)
        if (starts[c + 1] < starts[c]) return ANS_E_ARG;
    const uint64_t n = starts[nchunks];
    if (n && !syms) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(gt->g->device));
    DevBuf d_syms;
    HIP_TRY(d_syms.alloc(n * sym_bytes));
    if (n) HIP_TRY(hipMemcpyAsync(d_syms.p, syms, n * sym_bytes, hipMemcpyHostToDevice, gt->g->stream));
    return ans_encode_var_from_device(gt, d_syms.p, sym_bytes, nchunks, starts, out, out_cap, offsets, lens, total,
                                      gen_kind, seed);
} ANS_CATCH

int ans_gpu_encode_var_chunks(ans_gpu_table* gt, const void* syms, int sym_bytes, uint64_t nchunks,
                              const uint64_t* starts, uint8_t* out, uint64_t out_cap, uint64_t* offsets,
                              uint64_t* lens, uint64_t* total) try {
    return ans_gpu_encode_var_chunks_ex(gt, syms, sym_bytes, nchunks, starts, ANS_GEN_ZEROS, 0, out, out_cap, offsets,
                                        lens, total);
} ANS_CATCH

int ans_gpu_decode_var_chunks_ex(ans_gpu_table* gt, const uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                                 const uint64_t* lens, uint64_t nchunks, const uint64_t* starts, int gen_kind,
                                 uint64_t seed, void* out, int sym_bytes) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !valid_width(sym_bytes) || (nchunks && (!starts || !offsets || !lens)) || !valid_kind(gen_kind))
        return ANS_E_ARG;
    if (nchunks == 0) return ANS_OK;
    std::vector<uint32_t> l32(nchunks);
    for (uint64_t c = 0; c < nchunks; ++c) {
        if (starts[c + 1] < starts[c]) return ANS_E_ARG;
        if (lens[c] > 0xffffffffull || offsets[c] > in_len || lens[c] > in_len - offsets[c]) return ANS_E_LEN;
        l32[c] = static_cast<uint32_t>(lens[c]);
    }
    const uint64_t n = starts[nchunks];
    if ((n && !out) || (in_len && !in)) return ANS_E_ARG;
    uint64_t maxlen = 0;
    for (uint64_t c = 0; c < nchunks; ++c) maxlen = std::max(maxlen, starts[c + 1] - starts[c]);
    HIP_TRY(hipSetDevice(gt->g->device));
    const hipStream_t s = gt->g->stream;
    DevBuf d_in, d_offs, d_lens, d_starts, d_out, d_status;
    HIP_TRY(d_in.alloc(in_len + 128));  // the fast decoders read whole 128-B lines
    HIP_TRY(d_offs.alloc(8 * nchunks));
    HIP_TRY(d_lens.alloc(4 * nchunks));
    HIP_TRY(d_starts.alloc(8 * (nchunks + 1)));
    HIP_TRY(d_out.alloc(n * sym_bytes));
    HIP_TRY(d_status.alloc(4));
    if (in_len) HIP_TRY(hipMemcpyAsync(d_in.p, in, in_len, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_offs.p, offsets, 8 * nchunks, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_lens.p, l32.data(), 4 * nchunks, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_starts.p, starts, 8 * (nchunks + 1), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(d_status.p, 0, 4, s));
    int rc = dev_decode_var(gt, static_cast<uint8_t*>(d_in.p), static_cast<uint64_t*>(d_offs.p), 0,
                            static_cast<uint32_t*>(d_lens.p), nchunks, static_cast<uint64_t*>(d_starts.p), gen_kind,
                            seed, d_out.p, sym_bytes, static_cast<uint32_t*>(d_status.p), s,
                            staged_lmax(nchunks, maxlen, n, sym_bytes));
    if (rc) return rc;
    int st = 0;
    if ((rc = ans_dev_status(gt->g, static_cast<uint32_t*>(d_status.p), s, &st))) return rc;
    if (st) return st;
    if (n) HIP_TRY(hipMemcpy(out, d_out.p, n * sym_bytes, hipMemcpyDeviceToHost));
    return ANS_OK;
} ANS_CATCH

int ans_gpu_decode_var_chunks(ans_gpu_table* gt, const uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                              const uint64_t* lens, uint64_t nchunks, const uint64_t* starts, int gen_kind, void* out,
                              int sym_bytes) try {
    if (gen_kind != ANS_GEN_ZEROS && gen_kind != ANS_GEN_EMPTY) return ANS_E_ARG;  // RANDOM needs a seed: _ex
    return ans_gpu_decode_var_chunks_ex(gt, in, in_len, offsets, lens, nchunks, starts, gen_kind, 0, out, sym_bytes);
} ANS_CATCH

int ans_dev_compact(ans_gpu* g, const uint8_t* d_slots, uint64_t slot_cap, const uint32_t* d_lens,
                    const uint64_t* d_offsets, uint64_t nchunks, uint8_t* d_out, void* stream) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!g) return ANS_E_ARG;
    if (nchunks == 0) return ANS_OK;
    HIP_TRY(hipSetDevice(g->device));
    const hipStream_t s = stream ? static_cast<hipStream_t>(stream) : g->stream;
    k_compact<<<grid_for(nchunks * 64), kBlock, 0, s>>>(d_slots, slot_cap, d_lens, d_offsets, nchunks, d_out);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
} ANS_CATCH

int ans_dev_expand(ans_gpu* g, const uint8_t* d_in, const uint64_t* d_offsets, const uint32_t* d_lens,
                   uint64_t nchunks, uint8_t* d_slots, uint64_t slot_cap, void* stream) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!g) return ANS_E_ARG;
    if (nchunks == 0) return ANS_OK;
    if (!d_in || !d_offsets || !d_lens || !d_slots) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(g->device));
    const hipStream_t s = stream ? static_cast<hipStream_t>(stream) : g->stream;
    k_expand<<<grid_for(nchunks * 64), kBlock, 0, s>>>(d_in, d_offsets, d_lens, nchunks, d_slots, slot_cap);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
} ANS_CATCH

uint64_t ans_dense_offsets_entries(uint64_t nchunks) { return nchunks + 1 + (nchunks + kScanTile - 1) / kScanTile; }

int ans_dev_encode_dense_ex(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                            int gen_kind, uint64_t seed, uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens,
                            uint64_t* d_offsets, uint8_t* d_out, uint64_t out_cap, uint32_t* d_status, void* stream) try {
    if (n && (!d_offsets || !d_out)) return ANS_E_ARG;
    int rc = ans_dev_encode_chunks_ex(gt, d_syms, sym_bytes, n, chunk_len, gen_kind, seed, d_slots, slot_cap, d_lens,
                                      d_status, stream);
    if (rc) return rc;
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    const hipStream_t s = pick(gt, stream);
    if (nchunks == 0) {
        if (d_offsets) HIP_TRY(hipMemsetAsync(d_offsets, 0, sizeof(uint64_t), s));
        return ANS_OK;
    }
    const uint64_t ntiles = (nchunks + kScanTile - 1) / kScanTile;
    uint64_t* tile = d_offsets + nchunks + 1;
    k_scan_tiles<<<static_cast<unsigned>(ntiles), 1024, 0, s>>>(d_lens, nchunks, slot_cap, d_offsets, tile);
    k_scan_tile_sums<<<1, 1024, 0, s>>>(tile, ntiles, d_offsets + nchunks);
    k_compact_dense<<<grid_for(nchunks * 64), kBlock, 0, s>>>(d_slots, slot_cap, d_lens, d_offsets, tile, nchunks,
                                                              d_out, out_cap, d_status);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
} ANS_CATCH

int ans_dev_encode_dense(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                         uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens, uint64_t* d_offsets, uint8_t* d_out,
                         uint64_t out_cap, uint32_t* d_status, void* stream) try {
    return ans_dev_encode_dense_ex(gt, d_syms, sym_bytes, n, chunk_len, ANS_GEN_ZEROS, 0, d_slots, slot_cap, d_lens,
                                   d_offsets, d_out, out_cap, d_status, stream);
} ANS_CATCH

int ans_dev_status(ans_gpu* g, const uint32_t* d_status, void* stream, int* status) try {
    if (!g || !d_status || !status) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(g->device));
    const hipStream_t s = stream ? static_cast<hipStream_t>(stream) : g->stream;
    uint32_t bits = 0;
    HIP_TRY(hipMemcpyAsync(&bits, d_status, sizeof(bits), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *status = lowest_status(bits);
    return ANS_OK;
} ANS_CATCH

int ans_gpu_encode_chunks_ex(ans_gpu_table* gt, const void* syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                             int gen_kind, uint64_t seed, uint8_t* out, uint64_t out_cap, uint64_t* offsets,
                             uint64_t* lens, uint64_t* total) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !valid_width(sym_bytes) || chunk_len == 0 || !total || !valid_kind(gen_kind)) return ANS_E_ARG;
    const fast::ChunkInit ini{gen_kind, seed};
    if (n && !syms) return ANS_E_ARG;
    if (gt->ts64) {
        const uint64_t nc = (n + chunk_len - 1) / chunk_len;
        if (out && nc && (!offsets || !lens)) return ANS_E_ARG;
        return ans_tableset_host_encode(gt->ts64, syms, sym_bytes, n, chunk_len, nullptr, nc, gen_kind, seed, out,
                                        out_cap, offsets, lens, total);
    }
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    if (out && nchunks && (!offsets || !lens)) return ANS_E_ARG;
    *total = 0;
    if (nchunks == 0) return ANS_OK;
    HIP_TRY(hipSetDevice(gt->g->device));
    // page-locked symbols and container (or a size query): device-driven copies
    uint8_t* syms_dev = pipe_kernel_copies() ? mapped_ptr(syms) : nullptr;
    uint8_t* out_dev = out && syms_dev ? mapped_ptr(out) : nullptr;
    if (syms_dev && (!out || out_dev)) {
        switch (sym_bytes) {
        case 1: return pipe_encode_mapped<uint8_t>(gt, syms_dev, n, chunk_len, out_dev, out_cap, offsets, lens, total, ini);
        case 2: return pipe_encode_mapped<uint16_t>(gt, syms_dev, n, chunk_len, out_dev, out_cap, offsets, lens, total, ini);
        default: return pipe_encode_mapped<uint32_t>(gt, syms_dev, n, chunk_len, out_dev, out_cap, offsets, lens, total, ini);
        }
    }
    switch (sym_bytes) {
    case 1: return pipe_encode<uint8_t>(gt, syms, n, chunk_len, out, out_cap, offsets, lens, total, ini);
    case 2: return pipe_encode<uint16_t>(gt, syms, n, chunk_len, out, out_cap, offsets, lens, total, ini);
    default: return pipe_encode<uint32_t>(gt, syms, n, chunk_len, out, out_cap, offsets, lens, total, ini);
    }
} ANS_CATCH

int ans_gpu_encode_chunks(ans_gpu_table* gt, const void* syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                          uint8_t* out, uint64_t out_cap, uint64_t* offsets, uint64_t* lens, uint64_t* total) try {
    return ans_gpu_encode_chunks_ex(gt, syms, sym_bytes, n, chunk_len, ANS_GEN_ZEROS, 0, out, out_cap, offsets, lens,
                                    total);
} ANS_CATCH

int ans_gpu_decode_chunks_ex(ans_gpu_table* gt, const uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                             const uint64_t* lens, uint64_t n, uint64_t chunk_len, int gen_kind, uint64_t seed,
                             void* out, int sym_bytes) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !valid_width(sym_bytes) || chunk_len == 0) return ANS_E_ARG;
    const uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    if (nchunks && (!in || !offsets || !lens || !out)) return ANS_E_ARG;
    if (!valid_kind(gen_kind)) return ANS_E_ARG;
    if (gt->ts64)
        return ans_tableset_host_decode(gt->ts64, in, in_len, offsets, lens, n, chunk_len, nullptr, nchunks, gen_kind,
                                        seed, out, sym_bytes);
    const fast::ChunkInit ini{gen_kind, seed};
    if ((sym_bytes == 1 && gt->t.nsym > 256) || (sym_bytes == 2 && gt->t.nsym > 65536)) return ANS_E_ARG;
    std::vector<uint32_t> l32(nchunks);
    for (uint64_t j = 0; j < nchunks; ++j) {
        if (lens[j] > 0xffffffffull || offsets[j] > in_len || lens[j] > in_len - offsets[j]) return ANS_E_LEN;
        l32[j] = static_cast<uint32_t>(lens[j]);
    }
    // The fast decoders read the container in place (any stream alignment); slot_cap (widened
    // if a possibly corrupt stream is longer than a valid one can be) sizes the pipeline's
    // batches and tells a dense container from a scattered one.
    uint64_t slot_cap = 0, max_len = 0;
    ans_gpu_slot_capacity(gt, chunk_len, &slot_cap);
    for (uint64_t j = 0; j < nchunks; ++j) max_len = std::max<uint64_t>(max_len, l32[j]);
    slot_cap = std::max<uint64_t>(slot_cap, (max_len + 64 + 127) & ~uint64_t(127));
    HIP_TRY(hipSetDevice(gt->g->device));
    if (nchunks) {  // dense containers (the encoder's output) take the pipelined path
        int rc = kPipeScattered;
        uint8_t* in_dev = pipe_kernel_copies() ? mapped_ptr(in) : nullptr;
        uint8_t* out_dev = in_dev ? mapped_ptr(out) : nullptr;
        if (in_dev && out_dev) {
            switch (sym_bytes) {
            case 1: rc = pipe_decode_mapped<uint8_t>(gt, in_dev, offsets, l32.data(), slot_cap, n, chunk_len, gen_kind, out_dev, ini); break;
            case 2: rc = pipe_decode_mapped<uint16_t>(gt, in_dev, offsets, l32.data(), slot_cap, n, chunk_len, gen_kind, out_dev, ini); break;
            default: rc = pipe_decode_mapped<uint32_t>(gt, in_dev, offsets, l32.data(), slot_cap, n, chunk_len, gen_kind, out_dev, ini); break;
            }
            if (rc != kPipeScattered) return rc;
        }
        switch (sym_bytes) {
        case 1: rc = pipe_decode<uint8_t>(gt, in, offsets, l32.data(), slot_cap, n, chunk_len, gen_kind, out, ini); break;
        case 2: rc = pipe_decode<uint16_t>(gt, in, offsets, l32.data(), slot_cap, n, chunk_len, gen_kind, out, ini); break;
        default: rc = pipe_decode<uint32_t>(gt, in, offsets, l32.data(), slot_cap, n, chunk_len, gen_kind, out, ini); break;
        }
        if (rc != kPipeScattered) return rc;
    }
    // streams scattered over the buffer: one upload of the whole input, decoded in place (+256:
    // the fast decoders read whole aligned 128-B lines around each stream)
    const hipStream_t s = gt->g->stream;
    DevBuf d_in, d_off, d_lens, d_status, d_out;
    HIP_TRY(d_in.alloc(in_len + 256));
    HIP_TRY(d_off.alloc(nchunks * sizeof(uint64_t)));
    HIP_TRY(d_lens.alloc(nchunks * sizeof(uint32_t)));
    HIP_TRY(d_status.alloc(sizeof(uint32_t)));
    HIP_TRY(d_out.alloc(n * sym_bytes));
    if (in_len) HIP_TRY(hipMemcpyAsync(d_in.p, in, in_len, hipMemcpyHostToDevice, s));
    if (nchunks) {
        HIP_TRY(hipMemcpyAsync(d_off.p, offsets, nchunks * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_lens.p, l32.data(), nchunks * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    }
    HIP_TRY(hipMemsetAsync(d_status.p, 0, sizeof(uint32_t), s));
    int rc = ans_dev_decode_chunks_ex(gt, static_cast<uint8_t*>(d_in.p), static_cast<uint64_t*>(d_off.p), slot_cap,
                                      static_cast<uint32_t*>(d_lens.p), n, chunk_len, gen_kind, seed, d_out.p,
                                      sym_bytes, static_cast<uint32_t*>(d_status.p), s);
    if (rc) return rc;
    int st = 0;
    rc = ans_dev_status(gt->g, static_cast<uint32_t*>(d_status.p), s, &st);
    if (rc) return rc;
    if (st) return st;
    if (n) HIP_TRY(hipMemcpy(out, d_out.p, n * sym_bytes, hipMemcpyDeviceToHost));
    return ANS_OK;
} ANS_CATCH

int ans_gpu_decode_chunks(ans_gpu_table* gt, const uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                          const uint64_t* lens, uint64_t n, uint64_t chunk_len, int gen_kind, void* out,
                          int sym_bytes) try {
    if (gen_kind != ANS_GEN_ZEROS && gen_kind != ANS_GEN_EMPTY) return ANS_E_ARG;  // RANDOM needs a seed: _ex
    return ans_gpu_decode_chunks_ex(gt, in, in_len, offsets, lens, n, chunk_len, gen_kind, 0, out, sym_bytes);
} ANS_CATCH

}  // extern "C"
