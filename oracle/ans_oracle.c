/*
 * ans_oracle.c — CPU restatement of the reference rANS hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (shuffle-coding_amd/) links,
 * loads or calls this file.  Only tests/, __graft_entry__.smoke() and the
 * `cpu_baseline` leg of bench.py may use it, and only as the checker / the timed
 * CPU baseline — never as the thing that is shipped or measured on the GPU.
 *
 * What it restates (reference = entropy-coding/shuffle-coding @ 2024_08_07):
 *   src/ans.rs:14-22    constants Head=u64, TailElement=u8, MAX_MIN_HEAD=2^56
 *   src/ans.rs:96-105   blanket Distribution::push
 *   src/ans.rs:107-116  blanket Distribution::pop
 *   src/ans.rs:139-164  TailGenerator {Random(Pcg64Mcg), Zeros, Empty}
 *   src/ans.rs:189-223  Tail push/pop/normalize
 *   src/ans.rs:233-253  Message::renorm / renorm_up / renorm_down
 *   src/ans.rs:255-264  Message::flatten / unflatten (the wire format of one chunk)
 *   src/ans.rs:267-283  Message::bits / virtual_bits
 *   src/ans.rs:285-299  Message::random / zeros / empty
 *   src/ans.rs:302-310  canonical Message equality
 *   src/codec.rs:59-69  Categorical pmf / cdf / icdf (partition_point semantics)
 *   src/codec.rs:18-31  Uniform
 *   src/codec.rs:413-425 IID push (symbols in REVERSE) / pop (forward)
 *
 * Parity status: the reference is Rust and cannot be compiled in this image (no
 * cargo/rustc) and ships no byte-level golden vectors.  Byte
 * parity of this restatement is pinned by (i) the reference's own property
 * tests re-run against it (tests/test_oracle.py: ans.rs:47-68, codec.rs:646-669),
 * (ii) the reference's fixtures multiset-data/{1000,10000,100000}.txt with the benchmark_multiset
 * table rule (multiset.rs:158,169-170), and (iii) byte-for-byte agreement with an
 * independent pure-Python restatement (tests/golden/make_golden.py) whose
 * outputs are committed as tests/golden/golden_*.json.  Message::random's generator
 * (rand_pcg 0.3.1 Pcg64Mcg seeded by rand_core 0.6 seed_from_u64, bytes by
 * rand 0.8.5 Standard<u8>) is restated from those crates' published algorithms
 * and is "parity unpinned": no reference test pins its bytes.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_E_ZERO_MASS 1
#define ORC_E_EXHAUSTED 2
#define ORC_E_LEN 3
#define ORC_E_SYMBOL 4
#define ORC_E_NORM_RANGE 5
#define ORC_E_ALLOC 7

#define TAIL_PREC 8
#define MAX_MIN_HEAD (1ull << 56) /* ans.rs:19 */

enum { GEN_ZEROS = 0, GEN_EMPTY = 1, GEN_RANDOM = 2 };

typedef unsigned __int128 u128;

/* ---------------- TailGenerator (ans.rs:131-164) ---------------- */
typedef struct {
    int kind;
    uint64_t seed;
    u128 state; /* Pcg64Mcg state */
} gen_t;

/* rand_core 0.6 SeedableRng::seed_from_u64: PCG32 stream fills the 16-byte seed. */
static uint32_t pcg32_step(uint64_t *st) {
    const uint64_t MUL = 6364136223846793005ull, INC = 11634580027462260723ull;
    *st = *st * MUL + INC;
    uint64_t s = *st;
    uint32_t xorshifted = (uint32_t)(((s >> 18) ^ s) >> 27);
    uint32_t rot = (uint32_t)(s >> 59);
    return (xorshifted >> rot) | (xorshifted << ((32 - rot) & 31));
}

static void gen_init(gen_t *g, int kind, uint64_t seed) {
    g->kind = kind;
    g->seed = seed;
    g->state = 0;
    if (kind == GEN_RANDOM) {
        uint64_t st = seed;
        uint8_t bytes[16];
        for (int c = 0; c < 4; ++c) {
            uint32_t v = pcg32_step(&st);
            memcpy(bytes + 4 * c, &v, 4); /* to_le_bytes on little-endian host */
        }
        u128 s = 0;
        for (int i = 15; i >= 0; --i) s = (s << 8) | bytes[i]; /* u128::from_le_bytes */
        g->state = s | 3; /* Mcg128Xsl64::new */
    }
}

static uint8_t gen_pop(gen_t *g, int *err) {
    switch (g->kind) {
    case GEN_RANDOM: {
        const u128 MUL = ((u128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
        g->state = g->state * MUL;
        uint32_t rot = (uint32_t)(g->state >> 122);
        uint64_t xsl = (uint64_t)(g->state >> 64) ^ (uint64_t)g->state;
        uint64_t out = (xsl >> rot) | (xsl << ((64 - rot) & 63));
        return (uint8_t)(uint32_t)out; /* Standard<u8> = next_u32() as u8 */
    }
    case GEN_ZEROS:
        return 0;
    default:
        *err = ORC_E_EXHAUSTED; /* ans.rs:144 panics */
        return 0;
    }
}

/* ---------------- Tail (ans.rs:166-223) and Message (ans.rs:225-310) ---------------- */
typedef struct {
    uint8_t *el;
    size_t len, cap;
    gen_t gen;
    size_t num_generated;
} tail_t;

typedef struct {
    uint64_t head;
    tail_t tail;
    int err;
} orc_msg;

static int tail_reserve(tail_t *t, size_t need) {
    if (need <= t->cap) return 0;
    size_t nc = t->cap ? t->cap : 64;
    while (nc < need) nc *= 2;
    uint8_t *p = (uint8_t *)realloc(t->el, nc);
    if (!p) return -1;
    t->el = p;
    t->cap = nc;
    return 0;
}

static void tail_push(orc_msg *m, uint8_t e) {
    if (tail_reserve(&m->tail, m->tail.len + 1)) { m->err = ORC_E_ALLOC; return; }
    m->tail.el[m->tail.len++] = e;
}

static uint8_t tail_pop(orc_msg *m) {
    if (m->tail.len) return m->tail.el[--m->tail.len];
    m->tail.num_generated += 1;
    return gen_pop(&m->tail.gen, &m->err);
}

/* ans.rs:239-243 */
static void renorm_up(orc_msg *m, uint64_t min_head) {
    while (m->head < min_head && !m->err) m->head = (m->head << TAIL_PREC) | (uint64_t)tail_pop(m);
}

/* ans.rs:246-253 */
static void renorm_down(orc_msg *m, uint64_t min_head) {
    for (;;) {
        uint64_t new_head = m->head >> TAIL_PREC;
        if (new_head < min_head) break;
        tail_push(m, (uint8_t)m->head);
        m->head = new_head;
    }
}

/* ans.rs:233-236 */
static void renorm(orc_msg *m, uint64_t min_head) {
    renorm_up(m, min_head);
    renorm_down(m, min_head);
}

orc_msg *orc_msg_new(int kind, uint64_t seed) {
    orc_msg *m = (orc_msg *)calloc(1, sizeof(orc_msg));
    if (!m) return NULL;
    gen_init(&m->tail.gen, kind, seed);
    if (kind == GEN_RANDOM) { /* ans.rs:285-290 */
        m->head = 1;
        renorm_up(m, MAX_MIN_HEAD);
    } else { /* ans.rs:292-299 */
        m->head = MAX_MIN_HEAD;
    }
    return m;
}

void orc_msg_free(orc_msg *m) {
    if (!m) return;
    free(m->tail.el);
    free(m);
}

orc_msg *orc_msg_clone(const orc_msg *m) {
    orc_msg *c = (orc_msg *)malloc(sizeof(orc_msg));
    if (!c) return NULL;
    *c = *m;
    c->tail.el = NULL;
    c->tail.cap = 0;
    if (tail_reserve(&c->tail, m->tail.len ? m->tail.len : 1)) { free(c); return NULL; }
    if (m->tail.len) memcpy(c->tail.el, m->tail.el, m->tail.len);
    return c;
}

int orc_msg_err(const orc_msg *m) { return m->err; }
uint64_t orc_msg_head(const orc_msg *m) { return m->head; }
uint64_t orc_msg_tail_len(const orc_msg *m) { return m->tail.len; }
uint64_t orc_msg_num_generated(const orc_msg *m) { return m->tail.num_generated; }

/* ans.rs:255-260: flatten consumes a clone; returns the byte count, copies up to cap bytes. */
uint64_t orc_msg_flatten(const orc_msg *m, uint8_t *out, uint64_t cap) {
    orc_msg *c = orc_msg_clone(m);
    if (!c) return 0;
    renorm_down(c, 1);
    tail_push(c, (uint8_t)c->head);
    uint64_t n = c->tail.len;
    if (out) memcpy(out, c->tail.el, n < cap ? n : cap);
    orc_msg_free(c);
    return n;
}

/* ans.rs:262-264: head = 0, tail = the given bytes with a fresh generator. */
orc_msg *orc_msg_unflatten(const uint8_t *bytes, uint64_t len, int kind, uint64_t seed) {
    orc_msg *m = (orc_msg *)calloc(1, sizeof(orc_msg));
    if (!m) return NULL;
    gen_init(&m->tail.gen, kind, seed);
    if (tail_reserve(&m->tail, len ? len : 1)) { free(m); return NULL; }
    if (len) memcpy(m->tail.el, bytes, len);
    m->tail.len = len;
    m->head = 0;
    return m;
}

/* Message::unflatten(m.clone().flatten()) keeping the tail's generator (ans.rs:57). */
orc_msg *orc_msg_reflatten(const orc_msg *m) {
    orc_msg *c = orc_msg_clone(m);
    if (!c) return NULL;
    renorm_down(c, 1);
    tail_push(c, (uint8_t)c->head);
    c->head = 0;
    return c;
}

/* ans.rs:267-269 */
uint64_t orc_msg_bits(const orc_msg *m) { return TAIL_PREC * orc_msg_flatten(m, NULL, 0); }

/* ans.rs:274-283 */
double orc_msg_virtual_bits(const orc_msg *m) {
    const orc_msg *use = m;
    orc_msg *c = NULL;
    if (!(m->head > (1ull << 32))) {
        c = orc_msg_clone(m);
        renorm_up(c, MAX_MIN_HEAD);
        use = c;
    }
    double v = log2((double)use->head) +
               (double)(TAIL_PREC * ((int64_t)use->tail.len - (int64_t)use->tail.num_generated));
    if (c) orc_msg_free(c);
    return v;
}

/* ans.rs:207-222: drop the leading elements that are exactly the generated bytes. */
static void tail_normalize(tail_t *t) {
    if (t->num_generated == 0) return;
    size_t ng = t->num_generated;
    uint8_t *g = (uint8_t *)malloc(ng);
    gen_t fresh;
    gen_init(&fresh, t->gen.kind, t->gen.seed);
    int dummy = 0;
    for (size_t i = 0; i < ng; ++i) g[ng - 1 - i] = gen_pop(&fresh, &dummy); /* generated.reverse() */
    size_t k = 0;
    while (k < ng && k < t->len && g[k] == t->el[k]) ++k;
    memmove(t->el, t->el + k, t->len - k);
    t->len -= k;
    t->num_generated -= k;
    gen_init(&t->gen, t->gen.kind, t->gen.seed);
    for (size_t i = 0; i < t->num_generated; ++i) gen_pop(&t->gen, &dummy);
    free(g);
}

/* ans.rs:173-187 + 302-310 */
int orc_msg_equal(const orc_msg *a, const orc_msg *b) {
    orc_msg *x = orc_msg_clone(a), *y = orc_msg_clone(b);
    renorm(x, MAX_MIN_HEAD);
    renorm(y, MAX_MIN_HEAD);
    tail_normalize(&x->tail);
    tail_normalize(&y->tail);
    int eq = x->head == y->head && x->tail.len == y->tail.len &&
             (x->tail.len == 0 || memcmp(x->tail.el, y->tail.el, x->tail.len) == 0) &&
             x->tail.num_generated == y->tail.num_generated && x->tail.gen.kind == y->tail.gen.kind &&
             (x->tail.gen.kind != GEN_RANDOM || x->tail.gen.seed == y->tail.gen.seed);
    orc_msg_free(x);
    orc_msg_free(y);
    return eq;
}

/* ---------------- blanket Distribution push / pop (ans.rs:96-116) ---------------- */
/* push given p = pmf(x), norm, and c0 such that cdf(x, i) = c0 + i (Categorical/Uniform). */
static int push_linear(orc_msg *m, uint64_t p, uint64_t norm, uint64_t c0) {
    if (p == 0) return ORC_E_ZERO_MASS; /* ans.rs:98 assert_ne!(p, 0) */
    if (norm == 0 || norm > MAX_MIN_HEAD) return ORC_E_NORM_RANGE;
    renorm(m, p * (MAX_MIN_HEAD / norm));
    uint64_t q = m->head / p, r = m->head % p;
    m->head = norm * q + (c0 + r);
    return m->err;
}

/* ---------------- Categorical (codec.rs:51-92) ---------------- */
typedef struct {
    uint32_t nsym;
    uint64_t *mass;
    uint64_t *cum; /* cummasses (exclusive scan) */
    uint64_t norm;
} orc_cat;

orc_cat *orc_cat_new(const uint64_t *masses, uint32_t nsym) {
    orc_cat *c = (orc_cat *)calloc(1, sizeof(orc_cat));
    c->nsym = nsym;
    c->mass = (uint64_t *)malloc(sizeof(uint64_t) * (nsym ? nsym : 1));
    c->cum = (uint64_t *)malloc(sizeof(uint64_t) * (nsym ? nsym : 1));
    uint64_t acc = 0;
    for (uint32_t s = 0; s < nsym; ++s) {
        c->mass[s] = masses[s];
        c->cum[s] = acc;
        acc += masses[s];
    }
    c->norm = acc;
    return c;
}

void orc_cat_free(orc_cat *c) {
    if (!c) return;
    free(c->mass);
    free(c->cum);
    free(c);
}

uint64_t orc_cat_norm(const orc_cat *c) { return c->norm; }

/* codec.rs:65-68: x = partition_point(cum <= cf) - 1, i.e. the LAST symbol with cum[x] <= cf. */
static uint32_t cat_icdf(const orc_cat *c, uint64_t cf) {
    uint32_t lo = 0, hi = c->nsym; /* first index with cum > cf */
    while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (c->cum[mid] <= cf) lo = mid + 1; else hi = mid;
    }
    return lo - 1;
}

int orc_cat_push(orc_msg *m, const orc_cat *c, uint64_t x) {
    if (x >= c->nsym) return ORC_E_SYMBOL; /* codec.rs:63 index panic */
    return push_linear(m, c->mass[x], c->norm, c->cum[x]);
}

int orc_cat_pop(orc_msg *m, const orc_cat *c, uint64_t *x_out) {
    uint64_t norm = c->norm;
    if (norm == 0 || norm > MAX_MIN_HEAD) return ORC_E_NORM_RANGE;
    renorm(m, norm * (MAX_MIN_HEAD / norm));
    if (m->err) return m->err;
    uint64_t q = m->head / norm, i = m->head % norm;
    uint32_t x = cat_icdf(c, i);
    uint64_t r = i - c->cum[x];
    m->head = c->mass[x] * q + r;
    *x_out = x;
    return ORC_OK;
}

/* Uniform (codec.rs:18-31): norm = size, pmf = 1, cdf(x, 0) = x, icdf(cf) = (cf, 0). */
int orc_uniform_push(orc_msg *m, uint64_t size, uint64_t x) {
    if (x >= size) return ORC_E_SYMBOL;
    return push_linear(m, 1, size, x);
}

int orc_uniform_pop(orc_msg *m, uint64_t size, uint64_t *x_out) {
    if (size == 0 || size > MAX_MIN_HEAD) return ORC_E_NORM_RANGE;
    renorm(m, size * (MAX_MIN_HEAD / size));
    if (m->err) return m->err;
    uint64_t q = m->head / size, i = m->head % size;
    m->head = 1 * q + 0;
    *x_out = i;
    return ORC_OK;
}

/* IID (codec.rs:415-424): push in REVERSE order, pop forward. */
int orc_iid_push(orc_msg *m, const orc_cat *c, const uint32_t *syms, uint64_t n) {
    for (uint64_t k = n; k-- > 0;) {
        int e = orc_cat_push(m, c, syms[k]);
        if (e) return e;
    }
    return ORC_OK;
}

int orc_iid_pop(orc_msg *m, const orc_cat *c, uint32_t *out, uint64_t n) {
    for (uint64_t k = 0; k < n; ++k) {
        uint64_t x;
        int e = orc_cat_pop(m, c, &x);
        if (e) return e;
        out[k] = (uint32_t)x;
    }
    return ORC_OK;
}

/* ---------------- chunked streams (the GPU path's unit of work) ----------------
 * Chunk j covers symbols [j*L, min(n, (j+1)*L)) and is ONE independent reference
 * Message (initial Message::zeros() for GEN_ZEROS) encoded with IID<Categorical>
 * and flattened.  Streams are written densely: offsets[j] = sum of lens[<j].
 */
int orc_encode_chunks(const uint64_t *masses, uint32_t nsym, const uint32_t *syms, uint64_t n,
                      uint64_t chunk_len, int kind, uint64_t seed, uint8_t *out, uint64_t out_cap,
                      uint64_t *offsets, uint64_t *lens) {
    if (chunk_len == 0) return ORC_E_LEN;
    orc_cat *c = orc_cat_new(masses, nsym);
    uint64_t nchunks = (n + chunk_len - 1) / chunk_len, pos = 0;
    int rc = ORC_OK;
    for (uint64_t j = 0; j < nchunks && rc == ORC_OK; ++j) {
        uint64_t a = j * chunk_len, b = a + chunk_len < n ? a + chunk_len : n;
        orc_msg *m = orc_msg_new(kind, seed + j);
        rc = orc_iid_push(m, c, syms + a, b - a);
        if (rc == ORC_OK) {
            uint64_t len = orc_msg_flatten(m, NULL, 0);
            if (pos + len > out_cap) rc = ORC_E_LEN;
            else {
                orc_msg_flatten(m, out + pos, len);
                offsets[j] = pos;
                lens[j] = len;
                pos += len;
            }
        }
        orc_msg_free(m);
    }
    orc_cat_free(c);
    return rc;
}

/* Decodes every chunk and checks the reference invariant that the message returns to
 * its initial state (ans.rs:56 assert_eq!(initial, m)); returns ORC_E_LEN if not. */
int orc_decode_chunks(const uint64_t *masses, uint32_t nsym, const uint8_t *in, const uint64_t *offsets,
                      const uint64_t *lens, uint64_t n, uint64_t chunk_len, int kind, uint64_t seed,
                      uint32_t *out) {
    if (chunk_len == 0) return ORC_E_LEN;
    orc_cat *c = orc_cat_new(masses, nsym);
    uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    int rc = ORC_OK;
    for (uint64_t j = 0; j < nchunks && rc == ORC_OK; ++j) {
        uint64_t a = j * chunk_len, b = a + chunk_len < n ? a + chunk_len : n;
        orc_msg *m;
        if (kind == GEN_RANDOM) {
            /* Message::unflatten(m.flatten()) of a message begun as Message::random(seed + j):
             * the tail keeps its generator state and num_generated (ans.rs:57, 255-264), so
             * the round trip ends equal to Message::random(seed + j) (ans.rs:56) */
            m = orc_msg_new(kind, seed + j);
            if (m && tail_reserve(&m->tail, lens[j] ? lens[j] : 1) == 0) {
                if (lens[j]) memcpy(m->tail.el, in + offsets[j], lens[j]);
                m->tail.len = lens[j];
                m->head = 0;
            }
        } else {
            m = orc_msg_unflatten(in + offsets[j], lens[j], kind, seed + j);
        }
        rc = orc_iid_pop(m, c, out + a, b - a);
        if (rc == ORC_OK) {
            orc_msg *init = orc_msg_new(kind, seed + j);
            if (!orc_msg_equal(init, m)) rc = ORC_E_LEN;
            orc_msg_free(init);
        }
        orc_msg_free(m);
    }
    orc_cat_free(c);
    return rc;
}

/* ---------------- synthetic iid generator ----------------
 * symbol i of seed k: r = splitmix64((k << 48) ^ i); cf = floor(r * norm / 2^64); x = icdf(cf). */
static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t orc_splitmix64(uint64_t x) { return splitmix64(x); }

int orc_gen_iid(const uint64_t *masses, uint32_t nsym, uint64_t seed, uint64_t start, uint64_t n, uint32_t *out) {
    orc_cat *c = orc_cat_new(masses, nsym);
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t r = splitmix64((seed << 48) ^ (start + i));
        uint64_t cf = (uint64_t)(((u128)r * c->norm) >> 64);
        out[i] = cat_icdf(c, cf);
    }
    orc_cat_free(c);
    return ORC_OK;
}

/* ---------------- the other static codecs in chunks (GPU section 4b) ----------------
 * Chunk j covers symbols [j*L, min(n, (j+1)*L)) and is one message from the initial message of
 * `kind` (seed + j for RANDOM), pushed in reverse (IID/Independent, codec.rs:388-391,415-420). */
enum { ORC_CODEC_UNIFORM = 0, ORC_CODEC_LOGUNIFORM = 1, ORC_CODEC_INDEPENDENT = 2 };

typedef struct {
    int codec;
    uint64_t param;          /* Uniform: size; LogUniform: excl_max_bits */
    orc_cat **tables;        /* Independent */
    const uint32_t *tids;
} codec_t;

/* LogUniform (codec.rs:568-586): get_bits = 64 - leading_zeros */
static uint64_t get_bits(uint64_t x) { return x ? 64u - (uint64_t)__builtin_clzll(x) : 0u; }

static int codec_push(orc_msg *m, const codec_t *c, uint64_t x, uint64_t k) {
    switch (c->codec) {
    case ORC_CODEC_UNIFORM:
        if (c->param > (1ull << 46)) return ORC_E_NORM_RANGE; /* Uniform::new (codec.rs:34-37) */
        return orc_uniform_push(m, c->param, x);
    case ORC_CODEC_LOGUNIFORM: {
        uint64_t nbits = c->param + 1, bits = get_bits(x);
        if (bits >= nbits) return ORC_E_SYMBOL; /* assert!(bits < self.bits.size) */
        if (bits != 0) {
            uint64_t size = 1ull << (bits - 1);
            if (size > (1ull << 46)) return ORC_E_NORM_RANGE;
            int e = orc_uniform_push(m, size, x & ~size);
            if (e) return e;
        }
        return orc_uniform_push(m, nbits, bits);
    }
    default:
        return orc_cat_push(m, c->tables[c->tids[k]], x);
    }
}

static int codec_pop(orc_msg *m, const codec_t *c, uint64_t k, uint64_t *x) {
    switch (c->codec) {
    case ORC_CODEC_UNIFORM:
        return orc_uniform_pop(m, c->param, x);
    case ORC_CODEC_LOGUNIFORM: {
        uint64_t bits = 0, low = 0;
        int e = orc_uniform_pop(m, c->param + 1, &bits);
        if (e) return e;
        if (bits == 0) { *x = 0; return ORC_OK; }
        uint64_t size = 1ull << (bits - 1);
        e = orc_uniform_pop(m, size, &low);
        *x = low | size;
        return e;
    }
    default:
        return orc_cat_pop(m, c->tables[c->tids[k]], x);
    }
}

static codec_t codec_make(int codec, uint64_t param, uint32_t ntables, const uint64_t *masses, const uint32_t *nsyms,
                          const uint32_t *tids) {
    codec_t c = {codec, param, NULL, tids};
    if (codec == ORC_CODEC_INDEPENDENT) {
        c.tables = (orc_cat **)calloc(ntables ? ntables : 1, sizeof(orc_cat *));
        for (uint32_t t = 0; t < ntables; ++t) {
            c.tables[t] = orc_cat_new(masses, nsyms[t]);
            masses += nsyms[t];
        }
    }
    return c;
}

static void codec_free(codec_t *c, uint32_t ntables) {
    if (!c->tables) return;
    for (uint32_t t = 0; t < ntables; ++t) orc_cat_free(c->tables[t]);
    free(c->tables);
}

int orc_codec_encode_chunks(int codec, uint64_t param, uint32_t ntables, const uint64_t *masses, const uint32_t *nsyms,
                            const uint32_t *tids, const uint64_t *syms, uint64_t n, uint64_t chunk_len, int kind,
                            uint64_t seed, uint8_t *out, uint64_t out_cap, uint64_t *offsets, uint64_t *lens) {
    if (chunk_len == 0) return ORC_E_LEN;
    codec_t c = codec_make(codec, param, ntables, masses, nsyms, tids);
    uint64_t nchunks = (n + chunk_len - 1) / chunk_len, pos = 0;
    int rc = ORC_OK;
    for (uint64_t j = 0; j < nchunks && rc == ORC_OK; ++j) {
        uint64_t a = j * chunk_len, b = a + chunk_len < n ? a + chunk_len : n;
        orc_msg *m = orc_msg_new(kind, seed + j);
        for (uint64_t k = b; k-- > a && rc == ORC_OK;) rc = codec_push(m, &c, syms[k], k);
        if (rc == ORC_OK) {
            uint64_t len = orc_msg_flatten(m, NULL, 0);
            if (pos + len > out_cap) rc = ORC_E_LEN;
            else {
                orc_msg_flatten(m, out + pos, len);
                offsets[j] = pos;
                lens[j] = len;
                pos += len;
            }
        }
        orc_msg_free(m);
    }
    codec_free(&c, ntables);
    return rc;
}

/* Decodes every chunk and checks that it returns to its initial message (ans.rs:56); for RANDOM
 * the tail keeps the encoder's generator state (Message::unflatten(m.flatten()), ans.rs:57). */
int orc_codec_decode_chunks(int codec, uint64_t param, uint32_t ntables, const uint64_t *masses, const uint32_t *nsyms,
                            const uint32_t *tids, const uint8_t *in, const uint64_t *offsets, const uint64_t *lens,
                            uint64_t n, uint64_t chunk_len, int kind, uint64_t seed, uint64_t *out) {
    if (chunk_len == 0) return ORC_E_LEN;
    codec_t c = codec_make(codec, param, ntables, masses, nsyms, tids);
    uint64_t nchunks = (n + chunk_len - 1) / chunk_len;
    int rc = ORC_OK;
    for (uint64_t j = 0; j < nchunks && rc == ORC_OK; ++j) {
        uint64_t a = j * chunk_len, b = a + chunk_len < n ? a + chunk_len : n;
        orc_msg *m;
        if (kind == GEN_RANDOM) {
            m = orc_msg_new(kind, seed + j);
            if (m && tail_reserve(&m->tail, lens[j] ? lens[j] : 1) == 0) {
                if (lens[j]) memcpy(m->tail.el, in + offsets[j], lens[j]);
                m->tail.len = lens[j];
                m->head = 0;
            }
        } else {
            m = orc_msg_unflatten(in + offsets[j], lens[j], kind, seed + j);
        }
        for (uint64_t k = a; k < b && rc == ORC_OK; ++k) rc = codec_pop(m, &c, k, &out[k]);
        if (rc == ORC_OK) {
            orc_msg *init = orc_msg_new(kind, seed + j);
            if (!orc_msg_equal(init, m)) rc = ORC_E_LEN;
            orc_msg_free(init);
        }
        orc_msg_free(m);
    }
    codec_free(&c, ntables);
    return rc;
}
