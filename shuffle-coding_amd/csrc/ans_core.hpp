// ans_core.hpp — host-side C++ mirror of the reference's ANS surface.
//
// The reference (entropy-coding/shuffle-coding, Rust) exposes its coder as
//   trait Codec        { push(&self, &mut Message, &Symbol); pop(&self, &mut Message) -> Symbol; bits }  src/ans.rs:28-75
//   trait Distribution { norm(); pmf(x); cdf(x, i); icdf(cf) -> (x, i) }                            src/ans.rs:80-91
//   impl<D: Distribution> Codec for D                                                                 src/ans.rs:93-121
//   struct Message { head: u64, tail: Tail }                                                          src/ans.rs:225-310
// and the static codecs Uniform / Categorical / Bernoulli / Independent / IID (src/codec.rs).
// This header restates that surface with the same names, argument meaning and error
// behaviour (reference panics -> AnsError carrying the C-ABI status code) so that the
// sequential shuffle-coding layers can sit on top of it unchanged.  The bulk,
// data-parallel part (IID<Categorical> over many independent chunks) runs on the GPU in
// ans_kernels.hip; nothing in this header is a fallback for that path.
#pragma once

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/ans_capi.h"

namespace shuffle_coding {

using Head = uint64_t;         // src/ans.rs:14
using TailElement = uint8_t;   // src/ans.rs:15
constexpr int HEAD_PREC = 64;  // src/ans.rs:17
constexpr int TAIL_PREC = 8;   // src/ans.rs:18
constexpr Head MAX_MIN_HEAD = Head(1) << (HEAD_PREC - TAIL_PREC);  // src/ans.rs:19
constexpr uint64_t MAX_SIZE = MAX_MIN_HEAD >> 10;                   // src/ans.rs:22

struct AnsError : std::runtime_error {
    int code;
    AnsError(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

// ---------------------------------------------------------------- TailGenerator (ans.rs:131-164)
// Random = rand_pcg 0.3.1 Pcg64Mcg seeded via rand_core 0.6 seed_from_u64, bytes via
// rand 0.8.5 Standard<u8> (= next_u32() as u8).  Restated from those crates' published
// algorithms; no reference test pins the bytes ("parity unpinned").
class TailGenerator {
public:
    enum Kind : int { Zeros = ANS_GEN_ZEROS, Empty = ANS_GEN_EMPTY, Random = ANS_GEN_RANDOM };

    static TailGenerator zeros() { return TailGenerator(Zeros, 0); }
    static TailGenerator empty() { return TailGenerator(Empty, 0); }
    static TailGenerator random(uint64_t seed) { return TailGenerator(Random, seed); }
    static TailGenerator of_kind(int kind, uint64_t seed) {
        if (kind != Zeros && kind != Empty && kind != Random) throw AnsError(ANS_E_ARG, "unknown generator kind");
        return TailGenerator(static_cast<Kind>(kind), seed);
    }

    TailElement pop() {
        switch (kind_) {
        case Random: {
            state_ *= mcg_multiplier();
            const unsigned rot = static_cast<unsigned>(state_ >> 122);
            const uint64_t xsl = static_cast<uint64_t>(state_ >> 64) ^ static_cast<uint64_t>(state_);
            const uint64_t out = (xsl >> rot) | (xsl << ((64 - rot) & 63));
            return static_cast<TailElement>(static_cast<uint32_t>(out));
        }
        case Zeros: return 0;
        default: throw AnsError(ANS_E_EXHAUSTED, "Message exhausted whilst attempting decode.");  // ans.rs:144
        }
    }

    TailGenerator reset_clone() const { return TailGenerator(kind_, seed_); }  // ans.rs:148-154
    Kind kind() const { return kind_; }
    uint64_t seed() const { return seed_; }

    // ans.rs:180-185: generators compare by kind (and seed for Random), not by state.
    bool same_source(const TailGenerator& o) const {
        return kind_ == o.kind_ && (kind_ != Random || seed_ == o.seed_);
    }

private:
    using u128 = unsigned __int128;
    TailGenerator(Kind k, uint64_t seed) : kind_(k), seed_(seed) {
        if (k == Random) state_ = seed_from_u64(seed);
    }
    static u128 mcg_multiplier() { return (u128(0x2360ED051FC65DA4ull) << 64) | 0x4385DF649FCCF645ull; }
    static u128 seed_from_u64(uint64_t st) {
        uint8_t seed[16];
        for (int c = 0; c < 4; ++c) {  // rand_core 0.6: pcg32 fills the seed 4 bytes at a time
            st = st * 6364136223846793005ull + 11634580027462260723ull;
            const uint32_t xs = static_cast<uint32_t>(((st >> 18) ^ st) >> 27);
            const unsigned rot = static_cast<unsigned>(st >> 59);
            const uint32_t x = (xs >> rot) | (xs << ((32 - rot) & 31));
            for (int b = 0; b < 4; ++b) seed[4 * c + b] = static_cast<uint8_t>(x >> (8 * b));
        }
        u128 s = 0;
        for (int i = 15; i >= 0; --i) s = (s << 8) | seed[i];
        return s | 3;  // Mcg128Xsl64::new
    }

    Kind kind_;
    uint64_t seed_;
    u128 state_ = 0;
};

// ---------------------------------------------------------------- Tail (ans.rs:166-223)
class Tail {
public:
    Tail() : generator_(TailGenerator::zeros()) {}
    Tail(std::vector<TailElement> elements, TailGenerator generator)
        : elements_(std::move(elements)), generator_(generator) {}

    void push(TailElement e) { elements_.push_back(e); }
    TailElement pop() {
        if (!elements_.empty()) {
            const TailElement e = elements_.back();
            elements_.pop_back();
            return e;
        }
        num_generated_ += 1;
        return generator_.pop();
    }
    int64_t len_minus_generated() const {
        return static_cast<int64_t>(elements_.size()) - static_cast<int64_t>(num_generated_);
    }
    void normalize() {
        if (num_generated_ == 0) return;
        TailGenerator g = generator_.reset_clone();
        std::vector<TailElement> generated(num_generated_);
        for (auto& e : generated) e = g.pop();
        std::reverse(generated.begin(), generated.end());
        size_t k = 0;
        while (k < generated.size() && k < elements_.size() && generated[k] == elements_[k]) ++k;
        elements_.erase(elements_.begin(), elements_.begin() + static_cast<std::ptrdiff_t>(k));
        num_generated_ -= k;
        generator_ = generator_.reset_clone();
        for (size_t i = 0; i < num_generated_; ++i) generator_.pop();
    }
    bool operator==(const Tail& o) const {
        Tail a = *this, b = o;
        a.normalize();
        b.normalize();
        return a.elements_ == b.elements_ && a.num_generated_ == b.num_generated_ &&
               a.generator_.same_source(b.generator_);
    }

    const std::vector<TailElement>& elements() const { return elements_; }
    const TailGenerator& generator() const { return generator_; }
    size_t num_generated() const { return num_generated_; }

private:
    std::vector<TailElement> elements_;
    TailGenerator generator_;
    size_t num_generated_ = 0;
};

// ---------------------------------------------------------------- Message (ans.rs:225-310)
class Message {
public:
    Head head = MAX_MIN_HEAD;
    Tail tail;

    Message() = default;
    Message(Head h, Tail t) : head(h), tail(std::move(t)) {}

    void renorm(Head min_head) {  // ans.rs:233-236
        renorm_up(min_head);
        renorm_down(min_head);
    }
    void renorm_up(Head min_head) {  // ans.rs:239-243
        while (head < min_head) head = (head << TAIL_PREC) | static_cast<Head>(tail.pop());
    }
    void renorm_down(Head min_head) {  // ans.rs:246-253
        for (;;) {
            const Head new_head = head >> TAIL_PREC;
            if (new_head < min_head) break;
            tail.push(static_cast<TailElement>(head));
            head = new_head;
        }
    }
    Tail flatten() const {  // ans.rs:255-260 (on a copy, as callers always clone first)
        Message m = *this;
        m.renorm_down(1);
        m.tail.push(static_cast<TailElement>(m.head));
        return m.tail;
    }
    static Message unflatten(Tail tail) { return Message(0, std::move(tail)); }  // ans.rs:262-264
    size_t bits() const { return TAIL_PREC * flatten().elements().size(); }    // ans.rs:267-269
    double virtual_bits() const {                                               // ans.rs:274-283
        if (head > (Head(1) << 32))
            return std::log2(static_cast<double>(head)) + static_cast<double>(TAIL_PREC * tail.len_minus_generated());
        Message c = *this;
        c.renorm_up(MAX_MIN_HEAD);
        return std::log2(static_cast<double>(c.head)) + static_cast<double>(TAIL_PREC * c.tail.len_minus_generated());
    }
    static Message random(uint64_t seed) {  // ans.rs:285-290
        Message m(1, Tail({}, TailGenerator::random(seed)));
        m.renorm_up(MAX_MIN_HEAD);
        return m;
    }
    static Message zeros() { return Message(MAX_MIN_HEAD, Tail({}, TailGenerator::zeros())); }  // ans.rs:292-294
    static Message empty() { return Message(MAX_MIN_HEAD, Tail({}, TailGenerator::empty())); }  // ans.rs:297-299
    static Message of_kind(int kind, uint64_t seed) {
        switch (kind) {
        case ANS_GEN_ZEROS: return zeros();
        case ANS_GEN_EMPTY: return empty();
        case ANS_GEN_RANDOM: return random(seed);
        default: throw AnsError(ANS_E_ARG, "unknown generator kind");
        }
    }
    bool operator==(const Message& o) const {  // ans.rs:302-310
        Message m = *this, c = o;
        m.renorm(MAX_MIN_HEAD);
        c.renorm(MAX_MIN_HEAD);
        return m.tail == c.tail && m.head == c.head;
    }
    bool operator!=(const Message& o) const { return !(*this == o); }
};

// ---------------------------------------------------------------- blanket Distribution codec
// ans.rs:93-121.  A Distribution D provides norm(), pmf(x), cdf(x, i), icdf(cf).
template <class D>
void dist_push(const D& d, Message& m, const typename D::Symbol& x) {  // ans.rs:96-105
    const Head p = static_cast<Head>(d.pmf(x));
    if (p == 0) throw AnsError(ANS_E_ZERO_MASS, "assertion failed: pmf(x) != 0");
    const Head norm = static_cast<Head>(d.norm());
    if (norm == 0 || norm > MAX_MIN_HEAD) throw AnsError(ANS_E_NORM_RANGE, "norm out of range");
    m.renorm(p * (MAX_MIN_HEAD / norm));
    const Head h_div_p = m.head / p;
    const Head h_mod_p = m.head % p;
    const Head i = static_cast<Head>(d.cdf(x, h_mod_p));
    m.head = norm * h_div_p + i;
}

template <class D>
typename D::Symbol dist_pop(const D& d, Message& m) {  // ans.rs:107-116
    const Head norm = static_cast<Head>(d.norm());
    if (norm == 0 || norm > MAX_MIN_HEAD) throw AnsError(ANS_E_NORM_RANGE, "norm out of range");
    m.renorm(norm * (MAX_MIN_HEAD / norm));
    const Head h_div_p = m.head / norm;
    const Head i = m.head % norm;
    auto xr = d.icdf(i);
    const Head p = static_cast<Head>(d.pmf(xr.first));
    m.head = p * h_div_p + static_cast<Head>(xr.second);
    return xr.first;
}

template <class D>
double dist_bits(const D& d, const typename D::Symbol& x) {  // ans.rs:118-120
    return std::log2(static_cast<double>(d.norm())) - std::log2(static_cast<double>(d.pmf(x)));
}

// CRTP base giving every Distribution the Codec methods, as the blanket impl does.
template <class Derived>
struct DistributionCodec {
    template <class S>
    void push(Message& m, const S& x) const { dist_push(static_cast<const Derived&>(*this), m, x); }
    auto pop(Message& m) const { return dist_pop(static_cast<const Derived&>(*this), m); }
    template <class S>
    double bits(const S& x) const { return dist_bits(static_cast<const Derived&>(*this), x); }
};

// ---------------------------------------------------------------- Uniform (codec.rs:13-49)
struct Uniform : DistributionCodec<Uniform> {
    using Symbol = uint64_t;
    uint64_t size;
    explicit Uniform(uint64_t s) : size(s) {
        if (s > MAX_SIZE) throw AnsError(ANS_E_NORM_RANGE, "assertion failed: size <= MAX_SIZE");  // codec.rs:35
    }
    uint64_t norm() const { return size; }
    uint64_t pmf(const Symbol&) const { return 1; }
    uint64_t cdf(const Symbol& x, uint64_t i) const {
        if (i != 0) throw AnsError(ANS_E_ARG, "assertion failed: i == 0");
        return x;
    }
    std::pair<Symbol, uint64_t> icdf(uint64_t cf) const { return {cf, 0}; }
    double uni_bits() const { return std::log2(static_cast<double>(size)); }
};

// ---------------------------------------------------------------- Categorical (codec.rs:51-92)
struct Categorical : DistributionCodec<Categorical> {
    using Symbol = uint64_t;
    std::vector<uint64_t> masses;
    std::vector<uint64_t> cummasses;
    uint64_t norm_ = 0;

    explicit Categorical(std::vector<uint64_t> m) : masses(std::move(m)) {  // codec.rs:72-80
        cummasses.resize(masses.size());
        uint64_t acc = 0;
        for (size_t s = 0; s < masses.size(); ++s) {
            cummasses[s] = acc;
            acc += masses[s];
        }
        norm_ = acc;
    }
    uint64_t norm() const { return norm_; }
    uint64_t pmf(const Symbol& x) const {
        if (x >= masses.size()) throw AnsError(ANS_E_SYMBOL, "symbol index out of bounds");
        return masses[x];
    }
    uint64_t cdf(const Symbol& x, uint64_t i) const {
        if (x >= masses.size()) throw AnsError(ANS_E_SYMBOL, "symbol index out of bounds");
        return cummasses[x] + i;
    }
    std::pair<Symbol, uint64_t> icdf(uint64_t cf) const {  // codec.rs:65-68
        const auto it = std::partition_point(cummasses.begin(), cummasses.end(), [cf](uint64_t c) { return c <= cf; });
        const size_t x = static_cast<size_t>(it - cummasses.begin()) - 1;
        return {x, cf - cummasses[x]};
    }
    double prob(size_t x) const { return static_cast<double>(masses[x]) / static_cast<double>(norm_); }
    double entropy() const {
        double h = 0;
        for (size_t x = 0; x < masses.size(); ++x) {
            const double p = prob(x);
            if (p != 0.) h += -std::log2(p) * p;
        }
        return h;
    }
};

// ---------------------------------------------------------------- Bernoulli (codec.rs:94-129)
struct Bernoulli : DistributionCodec<Bernoulli> {
    using Symbol = bool;
    Categorical categorical;
    Bernoulli(uint64_t mass, uint64_t norm) : categorical(make(mass, norm)) {}
    uint64_t norm() const { return categorical.norm(); }
    uint64_t pmf(const Symbol& x) const { return categorical.pmf(x ? 1 : 0); }
    uint64_t cdf(const Symbol& x, uint64_t i) const { return categorical.cdf(x ? 1 : 0, i); }
    std::pair<Symbol, uint64_t> icdf(uint64_t cf) const {
        auto xr = categorical.icdf(cf);
        return {xr.first != 0, xr.second};
    }
    double prob() const { return categorical.prob(1); }

private:
    static Categorical make(uint64_t mass, uint64_t norm) {
        if (mass > norm) throw AnsError(ANS_E_ARG, "assertion failed: mass <= norm");  // codec.rs:126
        return Categorical({norm - mass, mass});
    }
};

// ---------------------------------------------------------------- IID / Independent (codec.rs:366-443)
template <class C>
struct IID {
    using Item = decltype(std::declval<const C&>().pop(std::declval<Message&>()));
    using Symbol = std::vector<Item>;
    C item;
    size_t len;
    IID(C c, size_t n) : item(std::move(c)), len(n) {}
    void push(Message& m, const Symbol& x) const {  // codec.rs:415-420: reverse order
        if (x.size() != len) throw AnsError(ANS_E_LEN, "assertion failed: x.len() == self.len");
        for (size_t k = x.size(); k-- > 0;) item.push(m, x[k]);
    }
    Symbol pop(Message& m) const {  // codec.rs:422-424: forward order
        Symbol out;
        out.reserve(len);
        for (size_t k = 0; k < len; ++k) out.push_back(item.pop(m));
        return out;
    }
    double bits(const Symbol& x) const {
        double t = 0;
        for (const auto& e : x) t += item.bits(e);
        return t;
    }
};

template <class C>
struct Independent {
    using Item = decltype(std::declval<const C&>().pop(std::declval<Message&>()));
    using Symbol = std::vector<Item>;
    std::vector<C> codecs;
    explicit Independent(std::vector<C> cs) : codecs(std::move(cs)) {}
    void push(Message& m, const Symbol& x) const {  // codec.rs:376-381
        if (x.size() != codecs.size()) throw AnsError(ANS_E_LEN, "assertion failed: x.len() == self.codecs.len()");
        for (size_t k = x.size(); k-- > 0;) codecs[k].push(m, x[k]);
    }
    Symbol pop(Message& m) const {
        Symbol out;
        out.reserve(codecs.size());
        for (const auto& c : codecs) out.push_back(c.pop(m));
        return out;
    }
    double bits(const Symbol& x) const {
        double t = 0;
        for (size_t k = 0; k < x.size(); ++k) t += codecs[k].bits(x[k]);
        return t;
    }
};

// ---------------------------------------------------------------- Codec::test (ans.rs:47-68, 318-332)
struct CodecTestResults {
    size_t bits;
    double amortized_bits;
    double enc_sec;
    double dec_sec;
};

inline void assert_bits_close(double expected, double bits, double tol) {  // ans.rs:329-332
    const double mismatch = std::fabs(bits - expected) / std::max(std::fabs(expected), 1.0);
    if (!(mismatch < tol))
        throw AnsError(ANS_E_MISMATCH, "Expected " + std::to_string(expected) + " bits, but got " + std::to_string(bits));
}

template <class C>
CodecTestResults test_invertibility(const C& codec, const typename C::Symbol& x, const Message& initial) {
    using clk = std::chrono::steady_clock;
    Message m = initial;
    auto t0 = clk::now();
    codec.push(m, x);
    const double enc_sec = std::chrono::duration<double>(clk::now() - t0).count();
    const size_t bits = m.bits();
    const double amortized = m.virtual_bits() - initial.virtual_bits();
    if (!(static_cast<double>(bits) >= amortized)) throw AnsError(ANS_E_MISMATCH, "bits < amortized bits");
    t0 = clk::now();
    auto decoded = codec.pop(m);
    const double dec_sec = std::chrono::duration<double>(clk::now() - t0).count();
    if (!(decoded == x)) throw AnsError(ANS_E_MISMATCH, "decoded != x");
    if (!(initial == m)) throw AnsError(ANS_E_MISMATCH, "initial != message after decode");
    if (!(initial == Message::unflatten(m.flatten()))) throw AnsError(ANS_E_MISMATCH, "flatten/unflatten mismatch");
    return {bits, amortized, enc_sec, dec_sec};
}

template <class C>
CodecTestResults test(const C& codec, const typename C::Symbol& x, const Message& initial) {
    CodecTestResults r = test_invertibility(codec, x, initial);
    assert_bits_close(codec.bits(x), r.amortized_bits, 1e-5);  // ans.rs:64-66
    return r;
}

}  // namespace shuffle_coding
