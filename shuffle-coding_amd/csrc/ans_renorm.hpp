// ans_renorm.hpp — the LDS-row encoder's per-row renorm word (ans_fast.hpp k_encode).  Plain
// C++ (a constexpr function is host and device code alike under hipcc), so the CPU test suite
// checks it against the reference's renorm loop with g++ (tests/test_renorm_word.py).
#pragma once
#include <cstdint>

namespace shuffle_coding {
namespace fast {

// The LDS-row encoder's renorm word for a row with bound pK = p*K (src/ans.rs:100, 246-253):
// a push emits k = #{j >= 1 : head >= pK * 2^8j} bytes.  Every push starts from head in
// [L, 2^8 L) (L = norm*K > 2^56 - norm: a push leaves head = norm*q + cdf < norm*2^8 K, and a
// chain's initial head, Message::zeros / empty / random, lies in [2^56, 2^57)), and a
// factor-2^8 interval holds at most one of the bounds pK*2^8j strictly inside it, so
// k = k0 + [head >= T] with k0 = #{j : pK*2^8j <= L} and T = pK*2^8(k0+1): ONE compare.  T's low
// byte is zero, so the word carries 8 k0 there: w = T + 8 k0.  Where T >= 2^8 L the test never
// holds and the row uses (k0 - 1, T / 2^8 <= L: always holds) instead; for k0 = 0 that is p = norm,
// T = 2^8 L, and with L < 2^56 no head reaches T (L = 2^56 with a mass equal to norm leaves the
// table off the fast path: ans_kernels.hip build_fast_table).  Zero mass: never, k0 = 0.
constexpr uint64_t enc_thr(uint64_t pK, uint64_t L) {
    if (pK == 0) return ~0xFFull;
    uint32_t k0 = 0;
    while (k0 < 7 && pK <= (L >> (8 * (k0 + 1)))) ++k0;  // pK * 2^8(k0+1) <= L
    const uint64_t A = pK << (8 * k0);                    // <= L <= 2^56
    if (A < L) return (A << 8) + 8 * k0;                  // T = 2^8 A < 2^8 L
    if (k0 > 0) return A + 8 * (k0 - 1);                  // A = L: always
    return L < (1ull << 56) ? (L << 8) : ~0xFFull;         // p = norm: never
}

// The same test as a shift of pK (the large-alphabet encoder, ans_wide.hpp k_encode_w<kSa>, which
// has no per-symbol LDS row but a byte per MASS): with w = enc_thr(pK, L), T = pK << sa and
// k = sa/8 - 1 + [head >= T] for sa = 8 + (w & 0xFF), in all three cases above (T = 2^8 A,
// A = pK << 8 k0: sa = 8 (k0 + 1); A = L: T = A, sa = 8 k0; p = norm: T = L << 8 = pK << 8).
// Returns 0 where no such shift exists (the caller then keeps the bit-length renorm).
constexpr uint32_t enc_sa(uint64_t pK, uint64_t L) {
    if (pK == 0) return 8;  // zero mass: the push is recorded as an error, any k will do
    const uint64_t w = enc_thr(pK, L);
    const uint32_t sa = 8 + static_cast<uint32_t>(w & 0xFF);
    if (sa >= 64 || (pK << sa) >> sa != pK || (pK << sa) != (w & ~0xFFull)) return 0;
    return sa;
}

}  // namespace fast
}  // namespace shuffle_coding
