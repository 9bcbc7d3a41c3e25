// ans_table.hpp — host-side table objects shared by the C ABI (ans_capi.cpp) and the
// GPU launchers (ans_kernels.hip).
#pragma once

#include <cstdint>

#include "ans_core.hpp"

// Opaque C-ABI handles (include/ans_capi.h).
struct ans_msg {
    shuffle_coding::Message m;
};

struct ans_table {
    shuffle_coding::Categorical cat;  // Categorical::new(masses)  src/codec.rs:72-80
};

namespace shuffle_coding {

// One symbol's row of the device table (16 B, so a 256-symbol alphabet is 4 KiB of LDS).
// Entry nsym is a sentinel {0, norm, 0} so the icdf search never runs past the end.
struct DevSym {
    uint32_t mass;  // pmf(x)                            src/codec.rs:63
    uint32_t cum;   // cummasses[x]                      src/codec.rs:64
    double rcp;     // 1.0 / mass, for the quotient estimate in the fast path
};

// Everything a kernel needs, passed by value in the kernel arguments.
struct DevTable {
    const DevSym* sym;       // nsym + 1 rows
    const uint16_t* bucket;  // nbucket entries: bucket[j] = icdf(j << shift).x
    uint32_t nsym;
    uint32_t norm;           // sum of masses, < 2^32
    uint32_t shift;          // icdf bucket width = 2^shift
    uint32_t nbucket;
    uint64_t K;              // MAX_MIN_HEAD / norm      (src/ans.rs:100,109)
    uint64_t L;              // norm * K: decode lower bound of the head interval
    double rcp_norm;         // 1.0 / norm
    uint32_t fast;           // 2^16 <= norm <= 2^31: f64 quotient estimate is exact after one fix-up
    uint32_t pmin;           // smallest non-zero mass (sizes the worst-case slot)
};

constexpr uint32_t kBucketBits = 12;
constexpr uint32_t kLdsTableLimit = 64 * 1024;  // table + buckets staged in LDS when they fit

// ---- fast-path tables (ans_fast.hpp); built when FastTable::usable.
// Encode row (16 B, one ds_read_b128): the thresholds p*K*2^(8j) are formed in registers.
struct EncRow {
    double rcp;     // 1.0 / mass (0 for the zero-mass sentinel)
    uint32_t mass;
    uint32_t cum;
};
// Decode bucket (16 B, one ds_read_b128): bucket j covers cdf values [j << dec_shift,
// (j+1) << dec_shift).  s0 = icdf(j << dec_shift) and c[i] = cdf(s0 + i), i = 0..3 (norm past
// the last symbol), so one LDS round trip resolves every cf in the bucket below c[3]; the
// rest (a bucket holding three or more boundaries, voted per wave) scan the cdf table staged
// after the buckets.  The s0 values follow the buckets as a u32 array (read off the chain's
// critical path: they only name the output symbol).
struct alignas(16) DecBucket {
    uint32_t c[4];
};
// Decode bucket for large alphabets (32 B, two 16-B global loads): cdf(s0..s0+5) and s0, so
// five candidates per bucket.
struct alignas(16) DecBucketG {
    uint32_t c[6];
    uint32_t s0;
    uint32_t pad;
};
// Compact large-alphabet bucket (16 B, one global load): c0 = cdf(s0) and the offsets
// d[k] = cdf(s0 + 1 + k) - c0, k = 0..4, as u16 (built only when every offset fits), so the
// same five candidates as DecBucketG in one L2 request instead of two.
struct alignas(16) DecBucketC {
    uint32_t c0;
    uint16_t s0;
    uint16_t d[5];
};
static_assert(sizeof(DecBucketC) == 16, "one 16-B load");
struct FastTable {
    const EncRow* enc;        // enc_rows = nsym + 1 rows (last = zero-mass sentinel)
    const DecBucket* dbkt;    // dec_buckets entries, then dec_buckets u32 s0 values (16-aligned region)
    const uint32_t* cum;      // cdf(s) for s = 0..nsym+5 (norm from nsym on): the slow icdf path
    const DecBucketG* dbkt_g; // large alphabets: dec_buckets entries in global memory
    uint32_t nsym;
    uint32_t enc_rows;
    uint32_t dec_buckets;
    uint32_t norm;
    uint32_t dec_shift;
    uint32_t enc_lds_bytes;   // LDS bytes of the staged encode rows (16-aligned)
    uint32_t dec_lds_bytes;   // LDS bytes of the staged decode buckets + cdf table (16-aligned)
    uint32_t dec_s0_off;      // offset of the s0 array from the buckets (LDS and global)
    uint32_t dec_cum_off;     // LDS offset of the cdf table
    uint32_t kmax;            // max bytes one push (and so one pop) moves (1..4)
    uint32_t pmax;            // largest mass (decode picks a 24-bit multiply below 2^24)
    uint64_t K;
    uint64_t L;
    double rcp_norm;
    uint32_t usable;      // fast paths available (2^16 <= norm <= 2^31, or nsym <= 256 at any norm)
    uint32_t nr;          // norm range: fast::kNormStd / kNormSmall / kNormBig (ans_fast.hpp)
    uint32_t p24;         // k_decode's 24-bit high-word product applies (pmax < 2^24, norm > 2^8)
    uint32_t enc_global;  // rows read from global memory (nsym > 256; ans_fast.hpp kGlobalRows)
    uint32_t dec_usable;  // decode fast path available (nsym <= 256: buckets in LDS)
    uint32_t dec_global;  // decode fast path for nsym > 256 (k_decode_g, buckets in global memory)
    uint32_t dec_far;     // some LDS bucket holds three or more cdf boundaries (slow path needed)
    uint32_t enc_wide;    // large alphabet with norm >= 2^22: ans_wide.hpp k_encode_w (cdf rows)
    uint32_t enc_nl;      // k_encode_w: symbols below enc_nl read their cdf pair from LDS
    // k_decode_w (ans_wide.hpp): the icdf of cf < dec_w_cpre = cdf(dec_w_nlp) from LDS
    const uint16_t* dec_w_s0;  // dec_w_nbp bucket starts icdf(b << dec_w_shp) (u16), staged in LDS
    uint32_t dec_wide;
    uint32_t dec_w_nlp;
    uint32_t dec_w_cpre;
    uint32_t dec_w_shp;
    uint32_t dec_w_nbp;
    uint32_t dec_w_cum_off;    // LDS offset of the cdf prefix from the s0 array (16-aligned)
    // k_encode_w with a packed LDS prefix (enc_pack): B[b] = cdf(16 b) (u32, enc_nl/16 + 2
    // entries) at the image's start and O[s] = cdf(s) mod 2^16 (u16, enc_nl + 2 entries) at byte
    // enc_pack_ooff, for tables whose masses are below 2^16 and whose blocks of 16 masses keep
    // cdf(s) - B[s >> 4] below 2^16: cdf(s) = B + ((O[s] - B) mod 2^16), pmf(s) = (O[s+1] - O[s])
    // mod 2^16.  2.25 B per symbol instead of 4, so a longer prefix fits
    const uint32_t* enc_pack_img;
    uint32_t enc_pack;
    uint32_t enc_pack_ooff;
    uint32_t enc_pack_bytes;  // image bytes (a multiple of 4), staged into LDS as u32 words
    // ... and its global rows for s >= enc_nl in the LDS rows' form (B, O(s) | O(s+1) << 16):
    // (cdf(s), cdf(s) mod 2^16 | cdf(s+1) << 16), 8 B per symbol 0..nsym, one load each
    const uint32_t* enc_grow;
    // k_encode_w<kSa> (every mass <= fast::kWideSaMax, with the packed prefix): the renorm shift
    // of each mass, sa(p) = 8 (k0(p) + 1) with T = p*K << sa(p) (ans_renorm.hpp enc_sa), one
    // byte per mass at LDS offset 0 (fast::kWideSaBytes, staged from enc_sa_img)
    const uint32_t* enc_sa_img;
    uint32_t enc_sa;
    // k_decode_w past the prefix: compact buckets (dec_c) of width 2^dec_c_shift, else dbkt_g
    const DecBucketC* dbkt_c;
    uint32_t dec_c;
    uint32_t dec_c_shift;
    uint32_t dec_c_nlb;  // k_decode_w<kCompact, !kPrefix>: the first buckets staged in LDS (set per launch)
    // ... staged from dbkt_cl, buckets of width 2^dec_cl_shift: dbkt_c itself, or (tables with more
    // buckets than the LDS holds) the first kWideDecBktLds buckets at twice dbkt_c's width
    const DecBucketC* dbkt_cl;
    uint32_t dec_cl_shift;
    // k_decode kModeU (ans_fast.hpp): the quotient from below without a fix-up; u = head - q_m*norm
    // in [0, 2 norm) indexes a virtual 512-symbol alphabet whose buckets (width 2^dec_u_shift)
    // all resolve among three candidates.  dec_u_img is the LDS image (fast::kDecTableBytes).
    const uint32_t* dec_u_img;
    uint32_t dec_u;
    uint32_t dec_u_shift;
};

}  // namespace shuffle_coding
