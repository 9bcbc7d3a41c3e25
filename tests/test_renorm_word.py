"""The fast encoders' one-compare renorms (shuffle-coding_amd/csrc/ans_renorm.hpp: the LDS-row
encoder's word enc_thr, DESIGN.md §3.1, and the large-alphabet encoder's per-mass shift enc_sa,
§3.3) against the reference's renorm loop, on the CPU.

The reference pushes a symbol of mass p after `renorm(p * K)` (src/ans.rs:100), whose
renorm_down emits head's low byte while `head >> 8 >= p * K` (src/ans.rs:246-253).  The kernel
computes the same count k from one 64-bit compare of (head | 0xFF) with the row's word
w = T + 8 k0, exact for every head in [L, 2^8 L): the heads a push leaves, and the initial heads
of Message::zeros / empty (2^56) and Message::random ([2^56, 2^57), src/ans.rs:285-299).  This
test compiles a brute-force checker with g++ against the product header and compares the rule
with the reference loop over random tables (norms 2^16..2^31, masses from 1 to norm) and heads
drawn uniformly, next to the interval ends, within a few units of every bound p*K*2^8j, and
from the initial-head range.  The shift rule k = sa/8 - 1 + [head >= p*K << sa] is checked on
the same heads wherever enc_sa gives a shift (every table but the off-path p = norm, L = 2^56).
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "shuffle-coding_amd", "csrc")

CHECKER = r"""
#include <cstdint>
#include <cstdio>
#include <random>
#include "ans_renorm.hpp"
using shuffle_coding::fast::enc_thr;
using shuffle_coding::fast::enc_sa;
typedef unsigned __int128 u128;

static uint32_t ref_k(uint64_t head, uint64_t pK) {  // src/ans.rs:246-253
    uint32_t k = 0;
    while ((head >> 8) >= pK) { head >>= 8; ++k; }
    return k;
}
static uint32_t kernel_k(uint64_t head, uint64_t w) {  // ans_fast.hpp k_encode bytes_out_w8
    return (uint32_t)((w & 0xFF) + ((head | 0xFF) > w ? 8 : 0)) / 8;
}
static uint32_t shift_k(uint64_t head, uint64_t pK, uint32_t sa) {  // ans_wide.hpp k_encode_w<kSa>
    return (head >= (pK << sa) ? sa : sa - 8) / 8;
}

int main(int argc, char** argv) {
    std::mt19937_64 R(12345);
    const int tables = argc > 1 ? atoi(argv[1]) : 50000;
    long n = 0, bad = 0, skipped = 0, nsa = 0;
    for (int it = 0; it < tables; ++it) {
        const int nb = 16 + (int)(R() % 16);
        uint64_t norm = (1ull << nb) + (R() % 3 == 0 ? 0 : R() % (1ull << nb));
        if (norm > (1ull << 31)) norm = 1ull << 31;
        const uint64_t K = (1ull << 56) / norm, L = norm * K;
        uint64_t p;
        switch (R() % 5) {
        case 0: p = 1 + R() % 4; break;
        case 1: p = norm; break;
        case 2: p = norm - R() % 4; break;
        case 3: p = 1 + (norm >> (R() % 31)); break;
        default: p = 1 + R() % norm;
        }
        if (p > norm) p = norm;
        if (p == norm && L == (1ull << 56)) { ++skipped; continue; }  // kept off the fast path
        const uint64_t pK = p * K, w = enc_thr(pK, L);
        const uint32_t sa = enc_sa(pK, L);
        if (sa == 0) { ++bad; printf("no shift norm=%llu p=%llu\n", (unsigned long long)norm, (unsigned long long)p); }
        const u128 top = (u128)L << 8;  // the heads of every push: [L, 2^8 L)
        for (int h = 0; h < 48; ++h) {
            uint64_t head;
            switch (h % 4) {
            case 0: head = L + R() % 1000; break;
            case 1: head = (uint64_t)(top - 1 - R() % 1000); break;
            case 2: {  // within a few units of a bound inside the interval
                uint64_t b = L;
                for (int j = 1; j <= 7; ++j) {
                    const u128 t = (u128)pK << (8 * j);
                    if (t > L && t < top) b = (uint64_t)t;
                }
                head = b - 3 + R() % 7;
                if (head < L) head = L;
                if ((u128)head >= top) head = (uint64_t)(top - 1);
                break;
            }
            default: head = L + (uint64_t)((((u128)R() << 64) | R()) % (top - L));
            }
            ++n;
            if (kernel_k(head, w) != ref_k(head, pK)) {
                if (bad < 5) printf("bad norm=%llu p=%llu head=%llx\n", (unsigned long long)norm, (unsigned long long)p, (unsigned long long)head);
                ++bad;
            }
            if (sa) {
                ++nsa;
                if (shift_k(head, pK, sa) != ref_k(head, pK)) {
                    if (bad < 5) printf("bad shift norm=%llu p=%llu head=%llx\n", (unsigned long long)norm, (unsigned long long)p, (unsigned long long)head);
                    ++bad;
                }
            }
        }
        // initial heads: Message::zeros / empty (2^56) and Message::random, [2^56, 2^57)
        for (int h = 0; h < 8; ++h) {
            const uint64_t head = h == 0 ? (1ull << 56) : (1ull << 56) | (R() >> 8);
            if (head < L || (u128)head >= top) { ++bad; printf("initial head outside [L, 2^8 L)\n"); }
            ++n;
            if (kernel_k(head, w) != ref_k(head, pK) || (sa && shift_k(head, pK, sa) != ref_k(head, pK))) {
                if (bad < 5) printf("bad initial head norm=%llu p=%llu head=%llx\n", (unsigned long long)norm, (unsigned long long)p, (unsigned long long)head);
                ++bad;
            }
        }
    }
    printf("shift-checked %ld\n", nsa);
    printf("checked %ld skipped %ld bad %ld\n", n, skipped, bad);
    return bad != 0;
}
"""


def test_renorm_word_matches_reference_loop(tmp_path):
    src = tmp_path / "renorm_check.cpp"
    exe = tmp_path / "renorm_check"
    src.write_text(CHECKER)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", CSRC, str(src), "-o", str(exe)])
    out = subprocess.run([str(exe), "50000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    line = out.stdout.strip().splitlines()[-1]
    assert line.startswith("checked") and line.endswith("bad 0"), line
    assert int(line.split()[1]) > 2_000_000
    nsa = int(out.stdout.strip().splitlines()[-2].split()[1])
    assert nsa > 2_000_000, out.stdout
