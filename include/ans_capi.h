/*
 * ans_capi.h — C ABI of the MI355X-native rANS coder (libshufflecoding_amd.so).
 *
 * This is the drop-in boundary for the reference's ANS hot path
 * (entropy-coding/shuffle-coding @ 2024_08_07).  Plain pointers and sizes only; no
 * exceptions cross it; caller-owned buffers; no pointer is retained after a call
 * returns (handles excepted).  Every entry point names the reference interface it
 * replaces.  A Rust caller binds it with an `extern "C"` block.
 *
 * Threading: a Message handle is single-threaded (the reference's `&mut Message`);
 * tables are immutable after creation and may be shared; GPU handles are per device,
 * one HIP stream each, and must not be used from two threads at once.  A GPU table or
 * table set may be freed before or after its context (the free touches only the table,
 * e.g. from a garbage collector that finalizes both in any order); every other call on it
 * needs its context alive.
 */
#ifndef ANS_CAPI_H
#define ANS_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (the reference panics; we return these instead) ---- */
#define ANS_OK 0
#define ANS_E_ZERO_MASS 1   /* src/ans.rs:98     assert_ne!(p, 0)                        */
#define ANS_E_EXHAUSTED 2   /* src/ans.rs:144    "Message exhausted whilst attempting decode." */
#define ANS_E_LEN 3         /* src/codec.rs:416  IID length assert / output buffer too small  */
#define ANS_E_SYMBOL 4      /* src/codec.rs:63   symbol index out of range                */
#define ANS_E_NORM_RANGE 5  /* src/codec.rs:35   size/norm outside what the coder supports */
#define ANS_E_DEVICE 6      /* HIP runtime error or no GPU                                */
#define ANS_E_ALLOC 7       /* host or device allocation failed                           */
#define ANS_E_ARG 8         /* invalid argument (NULL handle, bad width, ...)             */
#define ANS_E_MISMATCH 9    /* a reference property check failed (src/ans.rs:52-57)       */

/* ---- tail generators: src/ans.rs:131-136 TailGenerator ---- */
#define ANS_GEN_ZEROS 0  /* Message::zeros()  src/ans.rs:292 */
#define ANS_GEN_EMPTY 1  /* Message::empty()  src/ans.rs:297 */
#define ANS_GEN_RANDOM 2 /* Message::random() src/ans.rs:285 (PCG bytes parity-unpinned) */

const char *ans_status_string(int status);
int ans_abi_version(void); /* bumps on any incompatible change */

/* ======================================================================
 * (1) Message handle — replaces `pub struct Message { head, tail }`
 *     (src/ans.rs:225-310).
 * ====================================================================== */
typedef struct ans_msg ans_msg;

/* Message::zeros()/empty()/random(seed)  src/ans.rs:285-299 */
int ans_msg_new(int gen_kind, uint64_t seed, ans_msg **out);
void ans_msg_free(ans_msg *m);
/* Clone  (#[derive(Clone)] src/ans.rs:225) */
int ans_msg_clone(const ans_msg *m, ans_msg **out);
/* m.clone().flatten().elements  src/ans.rs:255-260.  *len receives the byte count;
 * with out == NULL or cap < *len nothing is copied (size query / ANS_E_LEN). */
int ans_msg_flatten(const ans_msg *m, uint8_t *out, size_t cap, size_t *len);
/* Message::unflatten(Tail::new(bytes, generator))  src/ans.rs:262-264 */
int ans_msg_unflatten(const uint8_t *bytes, size_t len, int gen_kind, uint64_t seed, ans_msg **out);
/* Message::unflatten(m.clone().flatten()) keeping the Tail's generator state and
 * num_generated, as the reference's round-trip check does (src/ans.rs:57) */
int ans_msg_reflatten(const ans_msg *m, ans_msg **out);
/* Message::bits / virtual_bits  src/ans.rs:267-283 */
int ans_msg_bits(const ans_msg *m, uint64_t *bits);
int ans_msg_virtual_bits(const ans_msg *m, double *bits);
/* PartialEq for Message (canonicalising)  src/ans.rs:302-310 */
int ans_msg_equal(const ans_msg *a, const ans_msg *b, int *equal);
/* field access: m.head, m.tail.elements.len(), m.tail.num_generated */
int ans_msg_state(const ans_msg *m, uint64_t *head, uint64_t *tail_len, uint64_t *num_generated);

/* ======================================================================
 * (2) Two-phase scalar op — replaces the blanket `impl<D: Distribution> Codec for D`
 *     (src/ans.rs:93-121) for ANY Distribution, including ones whose cdf depends on i
 *     (e.g. PlainOrbitCodec, src/recursive/plain_orbit.rs:33-49).
 *       push: ans_push_begin(m, pmf(x), norm, &q, &r); c = cdf(x, r); ans_push_end(m, norm, q, c)
 *       pop:  ans_pop_begin(m, norm, &q, &cf); (x, r) = icdf(cf); ans_pop_end(m, pmf(x), q, r)
 * ====================================================================== */
int ans_push_begin(ans_msg *m, uint64_t p, uint64_t norm, uint64_t *q, uint64_t *r); /* ans.rs:97-102 */
int ans_push_end(ans_msg *m, uint64_t norm, uint64_t q, uint64_t cdf);               /* ans.rs:103-104 */
int ans_pop_begin(ans_msg *m, uint64_t norm, uint64_t *q, uint64_t *cf);             /* ans.rs:108-111 */
int ans_pop_end(ans_msg *m, uint64_t p, uint64_t q, uint64_t r);                     /* ans.rs:112-114 */
/* Uniform::push/pop  src/codec.rs:18-31 (size <= MAX_SIZE = 2^46, src/ans.rs:22) */
int ans_uniform_push(ans_msg *m, uint64_t size, uint64_t x);
int ans_uniform_pop(ans_msg *m, uint64_t size, uint64_t *x);

/* ======================================================================
 * (3) Static tables — replaces `Categorical` / `Bernoulli` (src/codec.rs:51-129) and
 *     `IID<Categorical>` on ONE message (src/codec.rs:405-443), on the host.
 * ====================================================================== */
typedef struct ans_table ans_table;

/* Categorical::new(masses)  src/codec.rs:72-80 */
int ans_table_create(const uint64_t *masses, uint32_t nsym, ans_table **out);
/* Bernoulli::new(mass, norm) = Categorical[norm-mass, mass]  src/codec.rs:125-128 */
int ans_table_create_bernoulli(uint64_t mass, uint64_t norm, ans_table **out);
void ans_table_free(ans_table *t);
int ans_table_info(const ans_table *t, uint32_t *nsym, uint64_t *norm);
/* Categorical as a Codec (blanket impl)  src/ans.rs:96-116 */
int ans_cat_push(ans_msg *m, const ans_table *t, uint64_t x);
int ans_cat_pop(ans_msg *m, const ans_table *t, uint64_t *x);
/* IID::push (reverse order) / IID::pop (forward)  src/codec.rs:415-424 */
int ans_push_iid(ans_msg *m, const ans_table *t, const uint32_t *syms, size_t n);
int ans_pop_iid(ans_msg *m, const ans_table *t, uint32_t *out, size_t n);

/* ======================================================================
 * (4) GPU bulk path (MI355X / gfx950) — the data-parallel hot path.
 *     n symbols are cut into chunks of chunk_len (the last may be shorter); chunk j is
 *     ONE independent reference message: Message::zeros(), IID<Categorical>::push of
 *     its symbols (src/codec.rs:415-420, src/ans.rs:96-105), flatten (src/ans.rs:255).
 *     Its stream is byte-identical to that.  Decode is IID::pop on
 *     Message::unflatten(stream) (src/codec.rs:422-424, src/ans.rs:107-116,262).
 *     Symbols are unsigned integers of sym_bytes = 1, 2 or 4 bytes.
 *     Tables with 1 <= nsym <= 65536 and norm < 2^32 take the table kernels; larger ones the
 *     exact 64-bit kernels of section 4b (norm <= 2^56, else ANS_E_NORM_RANGE).
 * ====================================================================== */
typedef struct ans_gpu ans_gpu;
typedef struct ans_gpu_table ans_gpu_table;

int ans_gpu_device_count(int *count);
/* one context per device; owns a HIP stream */
int ans_gpu_create(int device, ans_gpu **out);
void ans_gpu_free(ans_gpu *g);
/* Page-locked host memory for the host-buffer calls below (hipHostMalloc): their copies
 * then run asynchronously and overlap; pageable buffers go through the runtime's staging. */
int ans_host_alloc(size_t bytes, void **out);
void ans_host_free(void *p);
/* Symbol bytes per batch of the host-buffer pipeline below (0 = the default, 128 MiB).
 * Batches overlap their H2D copy, kernels and D2H copy on separate streams. */
int ans_gpu_set_batch_bytes(ans_gpu *g, uint64_t batch_bytes);
/* The pipeline's workspace slots: 0 until the first host-buffer call builds the pipeline, then
 * ANS_PIPE_DEPTH as read at that moment (2..8; default 6). */
int ans_gpu_pipe_depth(const ans_gpu *g, int *depth);
/* uploads the table (and its derived reciprocal / icdf-bucket data) to the device */
int ans_gpu_table_create(ans_gpu *g, const ans_table *t, ans_gpu_table **out);
void ans_gpu_table_free(ans_gpu_table *gt);
/* Which kernels full chunks of this table take (bit flags; chunks outside them, e.g. a ragged
 * last chunk, take the generic one-lane-per-chunk kernels): */
#define ANS_PATH_ENC_LDS 1u     /* fast encoder, rows staged in LDS (<= 256 symbols) */
#define ANS_PATH_ENC_GLOBAL 2u  /* fast encoder, rows read from global memory (larger alphabets) */
#define ANS_PATH_DEC_LDS 4u     /* fast decoder, icdf buckets in LDS */
#define ANS_PATH_DEC_GLOBAL 8u  /* fast decoder, icdf buckets in global memory */
#define ANS_PATH_ENC_WIDE 16u   /* large alphabet, norm >= 2^22: cdf-pair rows, LDS prefix (128-B symbol groups) */
#define ANS_PATH_DEC_WIDE 32u   /* large alphabet: LDS prefix icdf + global buckets */
#define ANS_PATH_DEC_COMPACT 64u /* ... whose global buckets are 16 B (u16 candidate offsets) */
#define ANS_PATH_ENC_PACKED 128u /* large-alphabet encoder with the packed (u32 base + u16) LDS prefix */
#define ANS_PATH_DEC_U 256u     /* LDS decoder without the quotient fix-up (u-domain tables): applies to
                                  * sym_bytes == 1 only; u16 / u32 decodes of the same table run the
                                  * row decoder (kModeRows: the same bytes, one fix-up more) */
#define ANS_PATH_ENC_SHIFT 512u /* packed large-alphabet encoder whose renorm reads a shift byte per
                                  * mass (every mass <= 4096) instead of comparing bit lengths */
int ans_gpu_table_paths(const ans_gpu_table *gt, uint32_t *paths);
/* worst-case stream bytes of one chunk of chunk_len symbols, rounded up to 16 */
int ans_gpu_slot_capacity(const ans_gpu_table *gt, uint64_t chunk_len, uint64_t *slot_cap);

/* Host buffers in, host buffers out (synchronous; includes H2D/D2H), pipelined in batches
 * of chunks over a persistent device workspace.  Page-locked host buffers let the copies
 * run asynchronously; pageable ones still work (the runtime stages them).
 * Encode writes the streams densely: chunk j at out[offsets[j] .. offsets[j]+lens[j]).
 * out_cap must hold the total (query the exact total by passing out == NULL: *total is
 * set and nothing else is written). */
int ans_gpu_encode_chunks(ans_gpu_table *gt, const void *syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                          uint8_t *out, uint64_t out_cap, uint64_t *offsets, uint64_t *lens, uint64_t *total);
/* gen_kind = ANS_GEN_ZEROS or ANS_GEN_EMPTY (what an exhausted stream yields); returns
 * ANS_E_MISMATCH if a chunk does not return to Message::zeros() (src/ans.rs:56). */
int ans_gpu_decode_chunks(ans_gpu_table *gt, const uint8_t *in, uint64_t in_len, const uint64_t *offsets,
                          const uint64_t *lens, uint64_t n, uint64_t chunk_len, int gen_kind, void *out,
                          int sym_bytes);

/* Chunks from another initial message (the _ex variants of this section): gen_kind = ANS_GEN_ZEROS
 * (Message::zeros(), what the plain calls use), ANS_GEN_EMPTY (Message::empty(): same bytes, an
 * exhausted tail is ANS_E_EXHAUSTED on decode) or ANS_GEN_RANDOM (chunk c starts from
 * Message::random(seed + c), src/ans.rs:285-290: head 1 then seven generator bytes pulled, the
 * reference harness' initial message, src/multiset.rs:174, src/benchmark.rs:698-700).  A push
 * never pulls, so a chunk's stream holds no generated byte; decode is
 * Message::unflatten(m.flatten()) of that message (src/ans.rs:57: the tail keeps its generator
 * state) and must end back at Message::random(seed + c) (src/ans.rs:56), else ANS_E_MISMATCH.
 * A corrupt RANDOM stream that reaches past its start is reported, not decoded further. */
int ans_gpu_encode_chunks_ex(ans_gpu_table *gt, const void *syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                             int gen_kind, uint64_t seed, uint8_t *out, uint64_t out_cap, uint64_t *offsets,
                             uint64_t *lens, uint64_t *total);
int ans_gpu_decode_chunks_ex(ans_gpu_table *gt, const uint8_t *in, uint64_t in_len, const uint64_t *offsets,
                             const uint64_t *lens, uint64_t n, uint64_t chunk_len, int gen_kind, uint64_t seed,
                             void *out, int sym_bytes);

/* Device-resident variants: all pointers are device pointers; asynchronous on `stream`
 * (a hipStream_t; NULL = the context's stream).  Streams live in fixed slots: chunk j at
 * d_slots + j*slot_cap (slot_cap from ans_gpu_slot_capacity).  Errors found on the
 * device are OR-ed into *d_status as (1u << status) bits; read with ans_dev_status. */
int ans_dev_encode_chunks(ans_gpu_table *gt, const void *d_syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                          uint8_t *d_slots, uint64_t slot_cap, uint32_t *d_lens, uint32_t *d_status, void *stream);
/* d_offsets == NULL: chunk j's stream starts at d_in + j*slot_cap (the encoder's layout);
 * otherwise at d_in + d_offsets[j] (e.g. a dense container, at any alignment: the fast decoders
 * read it in place).  The fast decoders (k_decode, k_decode_w) read no byte outside the
 * stream; k_decode_g (norm < 2^22 with more than 256 symbols) may read every byte of the
 * aligned 128-B lines holding a stream, so such a container needs 128 readable bytes past its end.
 * A d_lens entry above slot_cap (slot layout) or of 2^27 bytes or more (no stream of a chunk
 * the fast decoders take reaches that) is foreign or corrupt: ANS_E_LEN. */
int ans_dev_decode_chunks(ans_gpu_table *gt, const uint8_t *d_in, const uint64_t *d_offsets, uint64_t slot_cap,
                          const uint32_t *d_lens, uint64_t n, uint64_t chunk_len, int gen_kind, void *d_syms,
                          int sym_bytes, uint32_t *d_status, void *stream);
int ans_dev_encode_chunks_ex(ans_gpu_table *gt, const void *d_syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                             int gen_kind, uint64_t seed, uint8_t *d_slots, uint64_t slot_cap, uint32_t *d_lens,
                             uint32_t *d_status, void *stream);
int ans_dev_decode_chunks_ex(ans_gpu_table *gt, const uint8_t *d_in, const uint64_t *d_offsets, uint64_t slot_cap,
                             const uint32_t *d_lens, uint64_t n, uint64_t chunk_len, int gen_kind, uint64_t seed,
                             void *d_syms, int sym_bytes, uint32_t *d_status, void *stream);
/* Synthetic iid symbols, counter-based: symbol i of seed k is
 * icdf(floor(splitmix64((k << 48) ^ (start + i)) * norm / 2^64)). */
int ans_dev_gen_iid(ans_gpu_table *gt, uint64_t seed, uint64_t start, uint64_t n, void *d_syms, int sym_bytes,
                    void *stream);
/* Codec::samples (src/ans.rs:38-44) in bulk: chunk c of chunk_len symbols (the last may be
 * shorter) is IID::new(codec, len).sample(seed + c), i.e. len pops from
 * Message::random(seed + c).  The Random generator restates rand_pcg 0.3.1 Pcg64Mcg /
 * rand_core 0.6 seed_from_u64 / rand 0.8.5 (bytes parity-unpinned: no reference test pins
 * them), identically to the host's ANS_GEN_RANDOM. */
int ans_dev_sample_iid(ans_gpu_table *gt, uint64_t seed, uint64_t n, uint64_t chunk_len, void *d_syms, int sym_bytes,
                       void *stream);
int ans_gpu_sample_iid(ans_gpu_table *gt, uint64_t seed, uint64_t n, uint64_t chunk_len, void *out, int sym_bytes);
/* Variable-length chunks: chunk c is symbols [starts[c], starts[c+1]) (nchunks + 1
 * non-decreasing entries), still one reference message each, e.g. one graph or one record per
 * chunk.  One lane per chunk; slot_cap = ans_gpu_slot_capacity of the longest chunk.  Symbols
 * live at their absolute index (the buffers span [0, starts[nchunks])).  The chunks are staged
 * for the fast kernels when the padded layout stays within twice the symbols plus 64 MiB (else
 * the generic kernels); the ans_dev_ entries find the longest chunk on the device, which costs
 * one 16-byte copy back and a synchronisation of `stream` before the kernels are queued. */
int ans_dev_encode_var_chunks(ans_gpu_table *gt, const void *d_syms, int sym_bytes, uint64_t nchunks,
                              const uint64_t *d_starts, uint8_t *d_slots, uint64_t slot_cap, uint32_t *d_lens,
                              uint32_t *d_status, void *stream);
/* d_offsets == NULL: chunk c's stream at d_in + c*slot_cap; else at d_in + d_offsets[c] */
int ans_dev_decode_var_chunks(ans_gpu_table *gt, const uint8_t *d_in, const uint64_t *d_offsets, uint64_t slot_cap,
                              const uint32_t *d_lens, uint64_t nchunks, const uint64_t *d_starts, int gen_kind,
                              void *d_syms, int sym_bytes, uint32_t *d_status, void *stream);
int ans_gpu_encode_var_chunks(ans_gpu_table *gt, const void *syms, int sym_bytes, uint64_t nchunks,
                              const uint64_t *starts, uint8_t *out, uint64_t out_cap, uint64_t *offsets,
                              uint64_t *lens, uint64_t *total);
int ans_gpu_decode_var_chunks(ans_gpu_table *gt, const uint8_t *in, uint64_t in_len, const uint64_t *offsets,
                              const uint64_t *lens, uint64_t nchunks, const uint64_t *starts, int gen_kind, void *out,
                              int sym_bytes);
/* ... from the initial messages of the _ex note above (chunk c: Message::random(seed + c)) */
int ans_dev_encode_var_chunks_ex(ans_gpu_table *gt, const void *d_syms, int sym_bytes, uint64_t nchunks,
                                 const uint64_t *d_starts, int gen_kind, uint64_t seed, uint8_t *d_slots,
                                 uint64_t slot_cap, uint32_t *d_lens, uint32_t *d_status, void *stream);
int ans_dev_decode_var_chunks_ex(ans_gpu_table *gt, const uint8_t *d_in, const uint64_t *d_offsets, uint64_t slot_cap,
                                 const uint32_t *d_lens, uint64_t nchunks, const uint64_t *d_starts, int gen_kind,
                                 uint64_t seed, void *d_syms, int sym_bytes, uint32_t *d_status, void *stream);
int ans_gpu_encode_var_chunks_ex(ans_gpu_table *gt, const void *syms, int sym_bytes, uint64_t nchunks,
                                 const uint64_t *starts, int gen_kind, uint64_t seed, uint8_t *out, uint64_t out_cap,
                                 uint64_t *offsets, uint64_t *lens, uint64_t *total);
int ans_gpu_decode_var_chunks_ex(ans_gpu_table *gt, const uint8_t *in, uint64_t in_len, const uint64_t *offsets,
                                 const uint64_t *lens, uint64_t nchunks, const uint64_t *starts, int gen_kind,
                                 uint64_t seed, void *out, int sym_bytes);
/* Device-resident dense container (the wire format ans_gpu_encode_chunks returns): the chunks
 * are encoded into d_slots (scratch, nchunks * slot_cap bytes), their lengths scanned into
 * d_offsets and the streams packed: chunk j at d_out[d_offsets[j] .. + d_lens[j]),
 * d_offsets[nchunks] = the total.  d_offsets holds ans_dense_offsets_entries(nchunks) entries
 * (those past nchunks + 1 are scratch).  d_out must hold the total (nchunks * slot_cap always
 * does); a stream that would end past out_cap is not written and sets ANS_E_LEN in *d_status.
 * Asynchronous on `stream`.  ans_dev_decode_chunks(_ex) reads the container in place (the
 * fast decoders fetch the aligned 128-B lines around each stream).  Replaces the encode side of
 * src/codec.rs:411-419 IID::push over many messages plus their concatenation. */
uint64_t ans_dense_offsets_entries(uint64_t nchunks);
int ans_dev_encode_dense(ans_gpu_table *gt, const void *d_syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                         uint8_t *d_slots, uint64_t slot_cap, uint32_t *d_lens, uint64_t *d_offsets, uint8_t *d_out,
                         uint64_t out_cap, uint32_t *d_status, void *stream);
int ans_dev_encode_dense_ex(ans_gpu_table *gt, const void *d_syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                            int gen_kind, uint64_t seed, uint8_t *d_slots, uint64_t slot_cap, uint32_t *d_lens,
                            uint64_t *d_offsets, uint8_t *d_out, uint64_t out_cap, uint32_t *d_status, void *stream);
/* Compacts slot streams into a dense buffer: d_out[d_offsets[j] ..] = slot j. */
int ans_dev_compact(ans_gpu *g, const uint8_t *d_slots, uint64_t slot_cap, const uint32_t *d_lens,
                    const uint64_t *d_offsets, uint64_t nchunks, uint8_t *d_out, void *stream);
/* The inverse of ans_dev_compact: dense-container streams into the slot layout (which the
 * fast decode kernels read). */
int ans_dev_expand(ans_gpu *g, const uint8_t *d_in, const uint64_t *d_offsets, const uint32_t *d_lens,
                   uint64_t nchunks, uint8_t *d_slots, uint64_t slot_cap, void *stream);
/* Test hook: the fast decoders' renorm step (renorm_up, src/ans.rs:239-243, with the next four
 * stream bytes in the window, first byte on top) on n caller-chosen (head, window) pairs:
 * resulting heads and byte counts.  Heads must be >= 2^24 (at most four bytes pulled). */
int ans_dev_check_renorm(ans_gpu *g, const uint64_t *d_heads, const uint32_t *d_windows, uint64_t L, uint64_t n,
                         uint64_t *d_out_heads, uint32_t *d_out_k, void *stream);
/* Synchronises `stream` and maps the device status word to the lowest set status. */
int ans_dev_status(ans_gpu *g, const uint32_t *d_status, void *stream, int *status);

/* ======================================================================
 * (4b) The other static codecs of src/codec.rs in bulk, one lane per chunk; chunk c is one
 *      reference message from the initial message gen_kind / seed gives it, as in the _ex calls
 *      of section 4.  sym_bytes may also be 8 here.  Fixed chunks whose symbols are whole 128-B
 *      lines (chunk_len * sym_bytes % 128 == 0) run their full chunks on the fast kernels
 *      (ans_mfast.hpp: LDS stream rings, f64 / magic-reciprocal division); the ragged last chunk,
 *      variable chunks, other layouts and Independent sets beyond the fast range run on the
 *      exact 64-bit kernels.  Both give the same bytes.
 *      A Categorical with norm >= 2^32 (up to 2^56) or more than 65536 symbols takes these
 *      kernels through the section-4 calls themselves (ans_gpu_table_create accepts it; its
 *      paths flags are 0; ans_dev_gen_iid / sample_iid return ANS_E_NORM_RANGE for it).
 * ====================================================================== */
/* IID<Uniform(size)>  src/codec.rs:13-49; size <= MAX_SIZE = 2^46 (src/ans.rs:22, ANS_E_NORM_RANGE
 * beyond).  A symbol >= size is ANS_E_SYMBOL (the reference does not check it and codes garbage). */
int ans_gpu_uniform_encode_chunks(ans_gpu *g, uint64_t size, const void *syms, int sym_bytes, uint64_t n,
                                  uint64_t chunk_len, int gen_kind, uint64_t seed, uint8_t *out, uint64_t out_cap,
                                  uint64_t *offsets, uint64_t *lens, uint64_t *total);
int ans_gpu_uniform_decode_chunks(ans_gpu *g, uint64_t size, const uint8_t *in, uint64_t in_len,
                                  const uint64_t *offsets, const uint64_t *lens, uint64_t n, uint64_t chunk_len,
                                  int gen_kind, uint64_t seed, void *out, int sym_bytes);
/* IID<LogUniform::new(excl_max_bits)>  src/codec.rs:561-611 (excl_max_bits <= 64): per symbol a
 * Uniform(2^(bits-1)) push of its low bits, then Uniform(excl_max_bits + 1) of bits = 64 - clz(x);
 * MaxBenfordIID's item (src/param_codec.rs:117-119).  bits > excl_max_bits is ANS_E_SYMBOL,
 * x >= 2^47 is ANS_E_NORM_RANGE (Uniform::new's assert).  A chunk whose pushes would draw from
 * the tail generator (the tail's num_generated, which no byte container carries) is
 * ANS_E_MISMATCH. */
int ans_gpu_loguniform_encode_chunks(ans_gpu *g, uint32_t excl_max_bits, const void *syms, int sym_bytes, uint64_t n,
                                     uint64_t chunk_len, int gen_kind, uint64_t seed, uint8_t *out, uint64_t out_cap,
                                     uint64_t *offsets, uint64_t *lens, uint64_t *total);
int ans_gpu_loguniform_decode_chunks(ans_gpu *g, uint32_t excl_max_bits, const uint8_t *in, uint64_t in_len,
                                     const uint64_t *offsets, const uint64_t *lens, uint64_t n, uint64_t chunk_len,
                                     int gen_kind, uint64_t seed, void *out, int sym_bytes);
/* Independent<Categorical>  src/codec.rs:366-403: position k codes with table table_ids[k] of the set
 * (the Categoricals uploaded once; norms up to 2^56).  Chunk c = positions [c*chunk_len, ...). */
typedef struct ans_gpu_tableset ans_gpu_tableset;
int ans_gpu_tableset_create(ans_gpu *g, const ans_table *const *tables, uint32_t ntables, ans_gpu_tableset **out);
void ans_gpu_tableset_free(ans_gpu_tableset *ts);
int ans_gpu_independent_encode_chunks(ans_gpu_tableset *ts, const uint32_t *table_ids, const void *syms, int sym_bytes,
                                      uint64_t n, uint64_t chunk_len, int gen_kind, uint64_t seed, uint8_t *out,
                                      uint64_t out_cap, uint64_t *offsets, uint64_t *lens, uint64_t *total);
int ans_gpu_independent_decode_chunks(ans_gpu_tableset *ts, const uint32_t *table_ids, const uint8_t *in,
                                      uint64_t in_len, const uint64_t *offsets, const uint64_t *lens, uint64_t n,
                                      uint64_t chunk_len, int gen_kind, uint64_t seed, void *out, int sym_bytes);
/* Independent<Categorical> over variable-length chunks: chunk c is positions [starts[c], starts[c+1])
 * (nchunks + 1 non-decreasing entries; table_ids / syms / out span [0, starts[nchunks])), one
 * reference message each, e.g. one record of mixed fields per chunk.  These run on the exact
 * 64-bit kernels (one lane per chunk), which take any chunk length. */
int ans_gpu_independent_encode_var_chunks(ans_gpu_tableset *ts, const uint32_t *table_ids, const void *syms,
                                          int sym_bytes, uint64_t nchunks, const uint64_t *starts, int gen_kind,
                                          uint64_t seed, uint8_t *out, uint64_t out_cap, uint64_t *offsets,
                                          uint64_t *lens, uint64_t *total);
int ans_gpu_independent_decode_var_chunks(ans_gpu_tableset *ts, const uint32_t *table_ids, const uint8_t *in,
                                          uint64_t in_len, const uint64_t *offsets, const uint64_t *lens,
                                          uint64_t nchunks, const uint64_t *starts, int gen_kind, uint64_t seed,
                                          void *out, int sym_bytes);
/* 1 (fast kernels: every table has <= 256 symbols, the norms all in [2^16, 2^31], all below
 * 2^16 or all in (2^31, 2^32), and at most 15 tables: 257 encoder rows of 32 B per table beside
 * the 32-KiB stream ring in 160 KiB of LDS), 2 (the same, with rows of near-certain symbols that
 * take the voted exact renorm), 0 (exact kernels only: any other set) */
int ans_gpu_tableset_fast(const ans_gpu_tableset *ts, int *fast);
/* The fast kernels' workgroup layout for this set: 0 (default) picks 1,024-lane workgroups
 * sharing one LDS table image (the encoder's when it fits 32 KiB, the decoder's when it fits
 * 28 KiB) for calls of at least (compute units x 1,024) chunks, 256-lane ones below; 256 or
 * 1,024 force one where that image exists (ANS_E_ARG for 1,024 when neither fits).  The bytes
 * are the same either way. */
int ans_gpu_tableset_lanes(ans_gpu_tableset *ts, int lanes);

/* Device-resident 4b calls (replace the bulk IID::push / pop and Independent::push / pop of
 * src/codec.rs:388-399,415-424 on device memory): fixed chunks, chunk j's stream in its slot at
 * d_slots + j*slot_cap (slot_cap from the _slot_capacity calls), lengths in d_lens, errors OR-ed
 * into *d_status as (1u << status) bits (ans_dev_status); asynchronous on `stream` (NULL = the
 * context's).  Decoders read slots (d_offsets NULL) or a dense container at d_in + d_offsets[j].
 * d_tids: the table id of every position, one byte each (sets of at most 256 tables; ids are
 * not range-checked on the device, as the reference would index past its codec vector).
 * slot_cap is the codec's slot capacity (the _slot_capacity call for chunk_len) for every call,
 * dense-container decodes included: it bounds the fast kernels' stream positions, and any other
 * value sends every chunk to the exact kernels.  d_syms, d_tids and d_slots must be 16-byte
 * aligned (the fast kernels move symbols, table ids and slot pages with 16-B vector loads and
 * stores; hipMalloc and torch allocations are); a dense container's streams may start anywhere. */
int ans_gpu_uniform_slot_capacity(uint64_t size, uint64_t chunk_len, uint64_t *slot_cap);
int ans_gpu_loguniform_slot_capacity(uint32_t excl_max_bits, uint64_t chunk_len, uint64_t *slot_cap);
int ans_gpu_tableset_slot_capacity(const ans_gpu_tableset *ts, uint64_t chunk_len, uint64_t *slot_cap);
int ans_dev_uniform_encode(ans_gpu *g, uint64_t size, const void *d_syms, int sym_bytes, uint64_t n, uint64_t chunk_len,
                           int gen_kind, uint64_t seed, uint8_t *d_slots, uint64_t slot_cap, uint32_t *d_lens,
                           uint32_t *d_status, void *stream);
int ans_dev_uniform_decode(ans_gpu *g, uint64_t size, const uint8_t *d_in, const uint64_t *d_offsets, uint64_t slot_cap,
                           const uint32_t *d_lens, uint64_t n, uint64_t chunk_len, int gen_kind, uint64_t seed,
                           void *d_syms, int sym_bytes, uint32_t *d_status, void *stream);
int ans_dev_loguniform_encode(ans_gpu *g, uint32_t excl_max_bits, const void *d_syms, int sym_bytes, uint64_t n,
                              uint64_t chunk_len, int gen_kind, uint64_t seed, uint8_t *d_slots, uint64_t slot_cap,
                              uint32_t *d_lens, uint32_t *d_status, void *stream);
int ans_dev_loguniform_decode(ans_gpu *g, uint32_t excl_max_bits, const uint8_t *d_in, const uint64_t *d_offsets,
                              uint64_t slot_cap, const uint32_t *d_lens, uint64_t n, uint64_t chunk_len, int gen_kind,
                              uint64_t seed, void *d_syms, int sym_bytes, uint32_t *d_status, void *stream);
int ans_dev_independent_encode(ans_gpu_tableset *ts, const uint8_t *d_tids, const void *d_syms, int sym_bytes,
                               uint64_t n, uint64_t chunk_len, int gen_kind, uint64_t seed, uint8_t *d_slots,
                               uint64_t slot_cap, uint32_t *d_lens, uint32_t *d_status, void *stream);
int ans_dev_independent_decode(ans_gpu_tableset *ts, const uint8_t *d_tids, const uint8_t *d_in,
                               const uint64_t *d_offsets, uint64_t slot_cap, const uint32_t *d_lens, uint64_t n,
                               uint64_t chunk_len, int gen_kind, uint64_t seed, void *d_syms, int sym_bytes,
                               uint32_t *d_status, void *stream);
/* ... over variable-length chunks (d_starts: nchunks + 1 device entries; slot_cap from
 * ans_gpu_tableset_slot_capacity of the longest chunk; d_tids one byte per position) */
int ans_dev_independent_encode_var(ans_gpu_tableset *ts, const uint8_t *d_tids, const void *d_syms, int sym_bytes,
                                   uint64_t nchunks, const uint64_t *d_starts, int gen_kind, uint64_t seed,
                                   uint8_t *d_slots, uint64_t slot_cap, uint32_t *d_lens, uint32_t *d_status,
                                   void *stream);
int ans_dev_independent_decode_var(ans_gpu_tableset *ts, const uint8_t *d_tids, const uint8_t *d_in,
                                   const uint64_t *d_offsets, uint64_t slot_cap, const uint32_t *d_lens,
                                   uint64_t nchunks, const uint64_t *d_starts, int gen_kind, uint64_t seed,
                                   void *d_syms, int sym_bytes, uint32_t *d_status, void *stream);

/* ======================================================================
 * (5) Graph models' bulk-IID caller — DenseSetIID<EdgeIndex, AllEdgeIndices> with an
 *     IID<Bernoulli> (ErdosRenyi, src/graph_codec.rs:105-205).  Edges are uint32 pairs
 *     (i, j) (EdgeIndex, src/graph.rs:17), num_nodes < 2^32.  The alphabet is the reference's
 *     AllEdgeIndices order (src/graph_codec.rs:187-199): self-loops (i,i) first when `loops`,
 *     then for j in 0..n, i in 0..j: (i,j), followed by (j,i) when `directed`.  An edge outside
 *     the alphabet (undirected (j,i) with j > i, a loop without `loops`, a node >= n) is
 *     ANS_E_SYMBOL, where DenseSetIID::dense panics (src/graph_codec.rs:137).
 * ====================================================================== */
/* num_all_edge_indices  src/graph_codec.rs:203-205 */
int ans_edge_alphabet_len(uint64_t num_nodes, int directed, int loops, uint64_t *len);
/* DenseSetIID::dense  src/graph_codec.rs:133-138: d_dense[slot(edge)] = 1, others 0 (u8) */
int ans_dev_edges_to_dense(ans_gpu *g, uint64_t num_nodes, int directed, int loops, const uint32_t *d_edges,
                           uint64_t num_edges, uint8_t *d_dense, uint32_t *d_status, void *stream);
/* the filter of DenseSetIID::pop  src/graph_codec.rs:117-120: the set slots' edges in
 * alphabet order into d_edges (at most cap; ANS_E_LEN in *d_status beyond), count in *d_count */
int ans_dev_dense_to_edges(ans_gpu *g, uint64_t num_nodes, int directed, int loops, const uint8_t *d_dense,
                           uint32_t *d_edges, uint64_t cap, uint64_t *d_count, uint32_t *d_status, void *stream);
/* ErdosRenyi push / pop (src/graph_codec.rs:152-155), chunked like section (4): the dense
 * vector over the alphabet, coded with a Bernoulli table (ans_table_create_bernoulli; the
 * reference's Bernoulli::new(total_edges, total_possible_edges), src/benchmark.rs:556);
 * chunk j is one reference message over slots [j*chunk_len, (j+1)*chunk_len). */
int ans_gpu_dense_set_encode(ans_gpu_table *gt, uint64_t num_nodes, int directed, int loops, const uint32_t *edges,
                             uint64_t num_edges, uint64_t chunk_len, uint8_t *out, uint64_t out_cap,
                             uint64_t *offsets, uint64_t *lens, uint64_t *total);
int ans_gpu_dense_set_decode(ans_gpu_table *gt, uint64_t num_nodes, int directed, int loops, const uint8_t *in,
                             uint64_t in_len, const uint64_t *offsets, const uint64_t *lens, uint64_t chunk_len,
                             uint32_t *edges, uint64_t cap, uint64_t *num_edges);

/* Independent<GraphIID<ErdosRenyi>> over a dataset of graphs (GraphDatasetParamCodec with
 * ErdosRenyiParamCodec: one Bernoulli gt for every graph, src/param_codec.rs:171-199,243-293).
 * Graph g has num_nodes[g] nodes and the edges [edge_offsets[g], edge_offsets[g+1]) of `edges`
 * (uint32 pairs).  Graph g is chunk g of the variable-chunk path: its stream is the reference
 * message Message::zeros() + ErdosRenyi push of that graph alone.  Decode returns every graph's
 * edges in alphabet order, graph after graph, with edge_offsets (num_graphs + 1 entries) giving
 * each graph's range; ANS_E_LEN when they exceed cap (edge_offsets still complete). */
int ans_gpu_dense_sets_encode(ans_gpu_table *gt, uint64_t num_graphs, const uint32_t *num_nodes, int directed,
                              int loops, const uint32_t *edges, const uint64_t *edge_offsets, uint8_t *out,
                              uint64_t out_cap, uint64_t *offsets, uint64_t *lens, uint64_t *total);
int ans_gpu_dense_sets_decode(ans_gpu_table *gt, uint64_t num_graphs, const uint32_t *num_nodes, int directed,
                              int loops, const uint8_t *in, uint64_t in_len, const uint64_t *offsets,
                              const uint64_t *lens, uint32_t *edges, uint64_t cap, uint64_t *edge_offsets);

/* ======================================================================
 * (5b) GraphIID<NodeC, EdgeC, ErdosRenyi> over a dataset (src/graph_codec.rs:19-94), the model
 *      the reference's --er runs on node- and edge-labelled datasets: Independent of one
 *      GraphIID per graph (src/benchmark.rs:308-316, 349-358) with count-built Categorical labels
 *      (DatasetStats::node_label_dist / edge_label_dist, src/benchmark.rs:568-578) or, for
 *      --uniform-er, Uniform(size) labels (src/benchmark.rs:318-330, 360-372: pass the all-ones
 *      Categorical of that size, whose arithmetic is Uniform's: pmf 1, cdf x, norm size).
 *      Tables come from one table set: node_table and edge_table index it (ANS_NO_TABLE =
 *      EmptyCodec, nothing coded), edge_indicator_table is the Bernoulli (two symbols).  Graph g
 *      (num_nodes[g] nodes, node labels [sum of earlier num_nodes, + num_nodes[g]) of node_labels,
 *      edges [edge_offsets[g], edge_offsets[g+1]) of edges / edge_labels) is ONE message:
 *      Message::zeros() (or gen_kind / seed as in the _ex calls, graph g from seed + g), then
 *      GraphIID::push, i.e. EdgesIID::push (the edge labels sorted by edge index as a tuple
 *      (i, j), then the ErdosRenyi indicator vector) followed by IID<NodeC>::push of the node
 *      labels (src/graph_codec.rs:31-34, 61-65); its stream is that message flattened.
 *      Edges are uint32 pairs in the alphabet of section 5 (undirected: i <= j); an edge outside
 *      it, or with labelled edges a pair given twice, is ANS_E_SYMBOL; a label outside its table
 *      is ANS_E_SYMBOL.  Decode pops node labels, the indicator vector, then as many edge labels
 *      as the vector holds edges (src/graph_codec.rs:36-38, 67-71) and returns every graph's
 *      edges sorted by (i, j) -- EdgesIID::pop's `indices.sort_unstable()` -- with their labels
 *      beside them, graph after graph; edge_offsets (num_graphs + 1) gives each graph's range;
 *      ANS_E_LEN when the edges exceed cap (edge_offsets still complete).
 * ====================================================================== */
#define ANS_NO_TABLE 0xFFFFFFFFu
int ans_gpu_graphs_encode(ans_gpu_tableset *ts, uint32_t node_table, uint32_t edge_table,
                          uint32_t edge_indicator_table, int directed, int loops, uint64_t num_graphs,
                          const uint32_t *num_nodes, const uint32_t *node_labels, const uint32_t *edges,
                          const uint32_t *edge_labels, const uint64_t *edge_offsets, int gen_kind, uint64_t seed,
                          uint8_t *out, uint64_t out_cap, uint64_t *offsets, uint64_t *lens, uint64_t *total);
int ans_gpu_graphs_decode(ans_gpu_tableset *ts, uint32_t node_table, uint32_t edge_table,
                          uint32_t edge_indicator_table, int directed, int loops, uint64_t num_graphs,
                          const uint32_t *num_nodes, const uint8_t *in, uint64_t in_len, const uint64_t *offsets,
                          const uint64_t *lens, int gen_kind, uint64_t seed, uint32_t *node_labels, uint32_t *edges,
                          uint32_t *edge_labels, uint64_t cap, uint64_t *edge_offsets);

#ifdef __cplusplus
}
#endif
#endif /* ANS_CAPI_H */
