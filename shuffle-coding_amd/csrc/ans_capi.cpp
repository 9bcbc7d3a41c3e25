// ans_capi.cpp — host part of the C ABI (include/ans_capi.h sections 1-3).
//
// Message handles, the two-phase scalar op and the single-message IID path run on the
// host because the reference drives them one symbol at a time from sequential callers
// (src/recursive/mod.rs:117-148, src/recursive/prefix_orbit.rs:95-110): there is no
// data parallelism inside one message.  The data-parallel path is section 4
// (ans_kernels.hip); nothing here is a fallback for it.
#include <new>

#include "ans_table.hpp"

using namespace shuffle_coding;

namespace {

template <class F>
int guarded(F&& f) {
    try {
        f();
        return ANS_OK;
    } catch (const AnsError& e) {
        return e.code;
    } catch (const std::bad_alloc&) {
        return ANS_E_ALLOC;
    } catch (...) {
        return ANS_E_ARG;
    }
}

void check_norm(uint64_t norm) {
    if (norm == 0 || norm > MAX_MIN_HEAD) throw AnsError(ANS_E_NORM_RANGE, "norm out of range");
}

}  // namespace

extern "C" {

const char* ans_status_string(int status) {
    switch (status) {
    case ANS_OK: return "ok";
    case ANS_E_ZERO_MASS: return "zero probability mass for symbol";
    case ANS_E_EXHAUSTED: return "Message exhausted whilst attempting decode.";
    case ANS_E_LEN: return "length mismatch or buffer too small";
    case ANS_E_SYMBOL: return "symbol out of range";
    case ANS_E_NORM_RANGE: return "normaliser / alphabet outside the supported range";
    case ANS_E_DEVICE: return "HIP device error";
    case ANS_E_ALLOC: return "allocation failed";
    case ANS_E_ARG: return "invalid argument";
    case ANS_E_MISMATCH: return "message did not round-trip";
    default: return "unknown status";
    }
}

int ans_abi_version(void) { return 1; }

// ---------------------------------------------------------------- (1) Message
int ans_msg_new(int gen_kind, uint64_t seed, ans_msg** out) {
    if (!out) return ANS_E_ARG;
    *out = nullptr;
    return guarded([&] { *out = new ans_msg{Message::of_kind(gen_kind, seed)}; });
}

void ans_msg_free(ans_msg* m) { delete m; }

int ans_msg_clone(const ans_msg* m, ans_msg** out) {
    if (!m || !out) return ANS_E_ARG;
    *out = nullptr;
    return guarded([&] { *out = new ans_msg{m->m}; });
}

int ans_msg_flatten(const ans_msg* m, uint8_t* out, size_t cap, size_t* len) {
    if (!m || !len) return ANS_E_ARG;
    return guarded([&] {
        const Tail t = m->m.flatten();
        *len = t.elements().size();
        if (!out) return;
        if (cap < *len) throw AnsError(ANS_E_LEN, "flatten buffer too small");
        std::memcpy(out, t.elements().data(), *len);
    });
}

int ans_msg_unflatten(const uint8_t* bytes, size_t len, int gen_kind, uint64_t seed, ans_msg** out) {
    if (!out || (len && !bytes)) return ANS_E_ARG;
    *out = nullptr;
    return guarded([&] {
        std::vector<TailElement> el(bytes, bytes + len);
        *out = new ans_msg{Message::unflatten(Tail(std::move(el), TailGenerator::of_kind(gen_kind, seed)))};
    });
}

int ans_msg_reflatten(const ans_msg* m, ans_msg** out) {
    if (!m || !out) return ANS_E_ARG;
    *out = nullptr;
    return guarded([&] { *out = new ans_msg{Message::unflatten(m->m.flatten())}; });
}

int ans_msg_bits(const ans_msg* m, uint64_t* bits) {
    if (!m || !bits) return ANS_E_ARG;
    return guarded([&] { *bits = m->m.bits(); });
}

int ans_msg_virtual_bits(const ans_msg* m, double* bits) {
    if (!m || !bits) return ANS_E_ARG;
    return guarded([&] { *bits = m->m.virtual_bits(); });
}

int ans_msg_equal(const ans_msg* a, const ans_msg* b, int* equal) {
    if (!a || !b || !equal) return ANS_E_ARG;
    return guarded([&] { *equal = (a->m == b->m) ? 1 : 0; });
}

int ans_msg_state(const ans_msg* m, uint64_t* head, uint64_t* tail_len, uint64_t* num_generated) {
    if (!m) return ANS_E_ARG;
    if (head) *head = m->m.head;
    if (tail_len) *tail_len = m->m.tail.elements().size();
    if (num_generated) *num_generated = m->m.tail.num_generated();
    return ANS_OK;
}

// ---------------------------------------------------------------- (2) two-phase scalar op
int ans_push_begin(ans_msg* m, uint64_t p, uint64_t norm, uint64_t* q, uint64_t* r) {
    if (!m || !q || !r) return ANS_E_ARG;
    return guarded([&] {
        if (p == 0) throw AnsError(ANS_E_ZERO_MASS, "assertion failed: p != 0");  // src/ans.rs:98
        check_norm(norm);
        m->m.renorm(p * (MAX_MIN_HEAD / norm));  // src/ans.rs:100
        *q = m->m.head / p;                      // src/ans.rs:101
        *r = m->m.head % p;                      // src/ans.rs:102
    });
}

int ans_push_end(ans_msg* m, uint64_t norm, uint64_t q, uint64_t cdf) {
    if (!m) return ANS_E_ARG;
    m->m.head = norm * q + cdf;  // src/ans.rs:104
    return ANS_OK;
}

int ans_pop_begin(ans_msg* m, uint64_t norm, uint64_t* q, uint64_t* cf) {
    if (!m || !q || !cf) return ANS_E_ARG;
    return guarded([&] {
        check_norm(norm);
        m->m.renorm(norm * (MAX_MIN_HEAD / norm));  // src/ans.rs:109
        *q = m->m.head / norm;                      // src/ans.rs:110
        *cf = m->m.head % norm;                     // src/ans.rs:111
    });
}

int ans_pop_end(ans_msg* m, uint64_t p, uint64_t q, uint64_t r) {
    if (!m) return ANS_E_ARG;
    m->m.head = p * q + r;  // src/ans.rs:114
    return ANS_OK;
}

int ans_uniform_push(ans_msg* m, uint64_t size, uint64_t x) {
    if (!m) return ANS_E_ARG;
    return guarded([&] {
        const Uniform u(size);
        if (x >= size) throw AnsError(ANS_E_SYMBOL, "symbol out of range");
        u.push(m->m, x);
    });
}

int ans_uniform_pop(ans_msg* m, uint64_t size, uint64_t* x) {
    if (!m || !x) return ANS_E_ARG;
    return guarded([&] {
        const Uniform u(size);
        *x = u.pop(m->m);
    });
}

// ---------------------------------------------------------------- (3) tables
int ans_table_create(const uint64_t* masses, uint32_t nsym, ans_table** out) {
    if (!out || (nsym && !masses)) return ANS_E_ARG;
    *out = nullptr;
    return guarded([&] {
        uint64_t acc = 0;
        for (uint32_t s = 0; s < nsym; ++s) {
            if (masses[s] > MAX_MIN_HEAD - acc) throw AnsError(ANS_E_NORM_RANGE, "sum of masses overflows");
            acc += masses[s];
        }
        *out = new ans_table{Categorical(std::vector<uint64_t>(masses, masses + nsym))};
    });
}

int ans_table_create_bernoulli(uint64_t mass, uint64_t norm, ans_table** out) {
    if (!out) return ANS_E_ARG;
    *out = nullptr;
    return guarded([&] {
        const Bernoulli b(mass, norm);
        *out = new ans_table{b.categorical};
    });
}

void ans_table_free(ans_table* t) { delete t; }

int ans_table_info(const ans_table* t, uint32_t* nsym, uint64_t* norm) {
    if (!t) return ANS_E_ARG;
    if (nsym) *nsym = static_cast<uint32_t>(t->cat.masses.size());
    if (norm) *norm = t->cat.norm();
    return ANS_OK;
}

int ans_cat_push(ans_msg* m, const ans_table* t, uint64_t x) {
    if (!m || !t) return ANS_E_ARG;
    return guarded([&] { t->cat.push(m->m, x); });
}

int ans_cat_pop(ans_msg* m, const ans_table* t, uint64_t* x) {
    if (!m || !t || !x) return ANS_E_ARG;
    return guarded([&] { *x = t->cat.pop(m->m); });
}

int ans_push_iid(ans_msg* m, const ans_table* t, const uint32_t* syms, size_t n) {
    if (!m || !t || (n && !syms)) return ANS_E_ARG;
    return guarded([&] {
        for (size_t k = n; k-- > 0;) t->cat.push(m->m, static_cast<uint64_t>(syms[k]));  // src/codec.rs:417
    });
}

int ans_pop_iid(ans_msg* m, const ans_table* t, uint32_t* out, size_t n) {
    if (!m || !t || (n && !out)) return ANS_E_ARG;
    return guarded([&] {
        for (size_t k = 0; k < n; ++k) out[k] = static_cast<uint32_t>(t->cat.pop(m->m));  // src/codec.rs:423
    });
}

}  // extern "C"
