// Native check of the host half of the C ABI (include/ans_capi.h sections 1-3) under
// AddressSanitizer + UndefinedBehaviorSanitizer: random operation sequences on the library's
// Message / Categorical / Uniform / two-phase / IID entry points, each mirrored on the C oracle
// (oracle/ans_oracle.c, test infrastructure) and compared head by head and byte by byte, plus
// the error paths the reference panics on.  Built and run by tests/test_native_sanitize.py with
// host code only (ans_capi.cpp + the oracle; no HIP), so it runs without a GPU.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../include/ans_capi.h"

extern "C" {
struct orc_msg;
struct orc_cat;
orc_msg* orc_msg_new(int kind, uint64_t seed);
void orc_msg_free(orc_msg* m);
uint64_t orc_msg_head(const orc_msg* m);
uint64_t orc_msg_flatten(const orc_msg* m, uint8_t* out, uint64_t cap);
orc_cat* orc_cat_new(const uint64_t* masses, uint32_t nsym);
void orc_cat_free(orc_cat* c);
int orc_cat_push(orc_msg* m, const orc_cat* c, uint64_t x);
int orc_cat_pop(orc_msg* m, const orc_cat* c, uint64_t* x);
int orc_uniform_push(orc_msg* m, uint64_t size, uint64_t x);
int orc_uniform_pop(orc_msg* m, uint64_t size, uint64_t* x);
int orc_iid_push(orc_msg* m, const orc_cat* c, const uint32_t* syms, uint64_t n);
int orc_iid_pop(orc_msg* m, const orc_cat* c, uint32_t* out, uint64_t n);
}

static int failures = 0;
#define CHECK(cond)                                                          \
    do {                                                                     \
        if (!(cond)) {                                                       \
            std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #cond); \
            if (++failures > 10) std::exit(1);                               \
        }                                                                    \
    } while (0)

static std::vector<uint8_t> flat(const ans_msg* m) {
    size_t len = 0;
    ans_msg_flatten(m, nullptr, 0, &len);
    std::vector<uint8_t> b(len);
    CHECK(ans_msg_flatten(m, b.data(), b.size(), &len) == ANS_OK);
    return b;
}
static std::vector<uint8_t> flat(const orc_msg* m) {
    std::vector<uint8_t> b(orc_msg_flatten(m, nullptr, 0));
    orc_msg_flatten(m, b.data(), b.size());
    return b;
}

int main() {
    std::mt19937_64 rng(2024);
    const std::vector<std::vector<uint64_t>> tables = {
        {0, 1, 2, 3, 0, 0, 1, 0}, {8, 2}, {1, 1, 1, 1, 1, 1, 1}, {1ull << 40, 3, 1ull << 30}, {5, 0, 9, 1, 300000, 17}};
    std::vector<ans_table*> lt;
    std::vector<orc_cat*> ot;
    for (const auto& t : tables) {
        ans_table* h = nullptr;
        CHECK(ans_table_create(t.data(), static_cast<uint32_t>(t.size()), &h) == ANS_OK);
        lt.push_back(h);
        ot.push_back(orc_cat_new(t.data(), static_cast<uint32_t>(t.size())));
    }
    for (int kind : {ANS_GEN_ZEROS, ANS_GEN_RANDOM}) {
        for (uint64_t seed : {0ull, 7ull}) {
            ans_msg* m = nullptr;
            CHECK(ans_msg_new(kind, seed, &m) == ANS_OK);
            orc_msg* o = orc_msg_new(kind, seed);
            for (int step = 0; step < 20000; ++step) {
                const int op = static_cast<int>(rng() % 6);
                const size_t k = rng() % tables.size();
                if (op < 2) {
                    std::vector<uint32_t> nz;
                    for (uint32_t i = 0; i < tables[k].size(); ++i)
                        if (tables[k][i]) nz.push_back(i);
                    const uint64_t x = nz[rng() % nz.size()];
                    CHECK(ans_cat_push(m, lt[k], x) == ANS_OK);
                    CHECK(orc_cat_push(o, ot[k], x) == 0);
                } else if (op < 4) {
                    uint64_t x = 0, y = 0;
                    CHECK(ans_cat_pop(m, lt[k], &x) == ANS_OK);
                    CHECK(orc_cat_pop(o, ot[k], &y) == 0);
                    CHECK(x == y);
                } else if (op == 4) {
                    const uint64_t sizes[] = {2, 3, 1ull << 28, (1ull << 46) - 1, 1000003};
                    const uint64_t size = sizes[rng() % 5];
                    if (rng() & 1) {
                        const uint64_t x = rng() % size;
                        CHECK(ans_uniform_push(m, size, x) == ANS_OK);
                        CHECK(orc_uniform_push(o, size, x) == 0);
                    } else {
                        uint64_t x = 0, y = 0;
                        CHECK(ans_uniform_pop(m, size, &x) == ANS_OK);
                        CHECK(orc_uniform_pop(o, size, &y) == 0);
                        CHECK(x == y);
                    }
                } else {  // the two-phase op as a Categorical would drive it (src/ans.rs:96-116)
                    const auto& t = tables[k];
                    uint64_t norm = 0;
                    for (uint64_t v : t) norm += v;
                    if (rng() & 1) {
                        std::vector<uint32_t> nz;
                        for (uint32_t i = 0; i < t.size(); ++i)
                            if (t[i]) nz.push_back(i);
                        const uint64_t x = nz[rng() % nz.size()];
                        uint64_t cum = 0;
                        for (uint64_t i = 0; i < x; ++i) cum += t[i];
                        uint64_t q = 0, r = 0;
                        CHECK(ans_push_begin(m, t[x], norm, &q, &r) == ANS_OK);
                        CHECK(ans_push_end(m, norm, q, cum + r) == ANS_OK);
                        CHECK(orc_cat_push(o, ot[k], x) == 0);
                    } else {
                        uint64_t q = 0, cf = 0, y = 0;
                        CHECK(ans_pop_begin(m, norm, &q, &cf) == ANS_OK);
                        uint64_t x = 0, cum = 0;
                        while (x + 1 < t.size() && cum + t[x] <= cf) cum += t[x++];
                        while (t[x] == 0) cum += t[x++];  // the last symbol with cdf <= cf has mass > 0
                        CHECK(ans_pop_end(m, t[x], q, cf - cum) == ANS_OK);
                        CHECK(orc_cat_pop(o, ot[k], &y) == 0);
                        CHECK(x == y);
                    }
                }
                uint64_t head = 0, tl = 0, ng = 0;
                ans_msg_state(m, &head, &tl, &ng);
                CHECK(head == orc_msg_head(o));
            }
            CHECK(flat(m) == flat(o));
            // IID bulk ops (src/codec.rs:415-424)
            std::vector<uint32_t> syms(5000), back(5000), oback(5000);
            for (auto& s : syms) s = static_cast<uint32_t>(1 + rng() % 3);
            CHECK(ans_push_iid(m, lt[0], syms.data(), syms.size()) == ANS_OK);
            CHECK(orc_iid_push(o, ot[0], syms.data(), syms.size()) == 0);
            CHECK(flat(m) == flat(o));
            CHECK(ans_pop_iid(m, lt[0], back.data(), back.size()) == ANS_OK);
            CHECK(orc_iid_pop(o, ot[0], oback.data(), oback.size()) == 0);
            CHECK(back == syms && oback == syms);
            ans_msg* c = nullptr;
            CHECK(ans_msg_clone(m, &c) == ANS_OK);
            int eq = 0;
            CHECK(ans_msg_equal(m, c, &eq) == ANS_OK && eq == 1);
            ans_msg_free(c);
            ans_msg_free(m);
            orc_msg_free(o);
        }
    }
    // error paths (the reference panics): zero mass, out-of-range symbol, exhausted Empty tail
    ans_msg* m = nullptr;
    CHECK(ans_msg_new(ANS_GEN_ZEROS, 0, &m) == ANS_OK);
    CHECK(ans_cat_push(m, lt[0], 0) == ANS_E_ZERO_MASS);
    CHECK(ans_cat_push(m, lt[0], 99) == ANS_E_SYMBOL);
    ans_msg_free(m);
    CHECK(ans_msg_new(ANS_GEN_EMPTY, 0, &m) == ANS_OK);
    int rc = ANS_OK;
    uint64_t x = 0;
    for (int i = 0; i < 64 && rc == ANS_OK; ++i) rc = ans_cat_pop(m, lt[1], &x);
    CHECK(rc == ANS_E_EXHAUSTED);
    ans_msg_free(m);
    std::vector<uint8_t> junk(3, 0xAB);
    CHECK(ans_msg_unflatten(junk.data(), junk.size(), ANS_GEN_ZEROS, 0, &m) == ANS_OK);
    ans_msg_free(m);
    for (auto* h : lt) ans_table_free(h);
    for (auto* h : ot) orc_cat_free(h);
    if (failures) return 1;
    std::printf("abi_sanitize ok\n");
    return 0;
}
