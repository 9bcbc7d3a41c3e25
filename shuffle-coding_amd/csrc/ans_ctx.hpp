// ans_ctx.hpp — the GPU context and table handles behind the C ABI (include/ans_capi.h),
// shared by the HIP translation units of the library (ans_kernels.hip, ans_graph.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <new>
#include <stdexcept>

#include "ans_fast.hpp"
#include "ans_table.hpp"

using namespace shuffle_coding;

// Host-buffer pipeline (ans_gpu_encode_chunks / ans_gpu_decode_chunks): batches of chunks
// flow through kPipeDepth workspace slots, so that the H2D copy of batch b+1, the kernels of
// batch b and the D2H copy of batch b-1 overlap.  Kernels alternate between
// two compute streams (the context's and s_comp2): a batch's kernels occupy few CUs for about
// one chain latency (~1 ms for 4096-symbol chunks), so consecutive batches must overlap too.
// The three pipeline streams each get a hardware queue of their own (CU-masked queues are
// never shared; ans_kernels.hip own_queue_stream).  The workspace persists in the context and
// grows on demand.
constexpr int kPipeDepthMax = 8;  // workspace slots: ANS_PIPE_DEPTH (default kPipeDepth) at creation
constexpr int kPipeDepth = 6;
struct PipeSlot {
    void* d_syms = nullptr;     // batch symbols
    uint8_t* d_slots = nullptr; // batch streams in the slot layout
    uint8_t* d_dense = nullptr; // batch streams, dense (encode output / decode input)
    uint32_t* d_lens = nullptr;
    uint64_t* d_offs = nullptr;  // batch offsets (+ total at [nchunks] after encode)
    uint32_t* h_lens = nullptr;  // pinned staging
    uint64_t* h_offs = nullptr;  // pinned staging
    hipEvent_t ev_in = nullptr, ev_comp = nullptr, ev_meta = nullptr, ev_out = nullptr;
    bool used = false;
};
struct HostPipe {
    hipStream_t s_in = nullptr, s_out = nullptr, s_comp2 = nullptr;
    PipeSlot slot[kPipeDepthMax];
    int depth = kPipeDepth;  // slots in use
    uint32_t* d_status = nullptr;
    size_t cap_syms = 0, cap_slots = 0, cap_dense = 0, cap_chunks = 0;  // per slot
    // page-locked callers (device-driven copies): per-call chunk metadata and the carry
    uint64_t* h_meta = nullptr;  // mapped host staging: offsets[nchunks], lens[nchunks]
    size_t cap_meta = 0;
    uint64_t* d_acc = nullptr;   // running container offset across batches
    hipEvent_t ev_scan = nullptr;
};

struct ans_gpu {
    int device;
    int ncu;  // compute units (launchers size per-CU LDS use by it)
    hipStream_t stream;
    HostPipe* pipe;
    uint64_t batch_bytes;  // symbol bytes per pipeline batch (0 = default)
    void* d_scratch;       // device scratch of the device-resident graph calls (ans_graph.hip)
    size_t cap_scratch;
};

struct ans_gpu_table {
    ans_gpu* g;
    int device;          // g->device, kept here: freeing the table never touches its context
    DevTable t;
    void* d_mem;
    uint32_t lds_bytes;  // 0 = table read from global memory (L2-resident)
    FastTable ft;        // throughput path (ans_fast.hpp) when ft.usable
    void* d_fast;
    struct ans_gpu_tableset* ts64;  // norm >= 2^32 or nsym > 65536: the exact 64-bit kernels (ans_codecs.hip)
};

#define ANS_HIP_TRY(expr)                                                                              \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) {                                                                        \
            std::fprintf(stderr, "[shuffle-coding_amd] %s failed: %s\n", #expr, hipGetErrorString(e_)); \
            return ANS_E_DEVICE;                                                                       \
        }                                                                                              \
    } while (0)

// No C++ exception crosses the C ABI: every extern "C" entry of the HIP units
// is a function-try-block ending in ANS_CATCH.  A host allocation that fails (std::bad_alloc, or
// std::length_error from a std::vector sized by caller input) is ANS_E_ALLOC; anything else that
// escapes is ANS_E_ARG.  (ans_capi.cpp's host entries do the same through guarded().)
#define ANS_CATCH                                         \
    catch (const std::bad_alloc&) { return ANS_E_ALLOC; } \
    catch (const std::length_error&) { return ANS_E_ALLOC; } \
    catch (...) { return ANS_E_ARG; }
#define ANS_CATCH_VOID \
    catch (...) {}

// Variable-chunk encode of device-resident symbols into a host container (ans_kernels.hip):
// the body of ans_gpu_encode_var_chunks; starts is a host array of nchunks + 1 entries.
int ans_encode_var_from_device(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t nchunks,
                               const uint64_t* starts, uint8_t* out, uint64_t out_cap, uint64_t* offsets,
                               uint64_t* lens, uint64_t* total, int gen_kind = ANS_GEN_ZEROS, uint64_t seed = 0);

// The exact 64-bit generic kernels over a table set (ans_codecs.hip): Independent<Categorical>,
// and IID<Categorical> of tables the u32 kernels do not take (norm >= 2^32, nsym > 65536).
int ans_tableset_build(ans_gpu* g, const Categorical* const* cats, uint32_t ntables, struct ans_gpu_tableset** out);
void ans_tableset_destroy(struct ans_gpu_tableset* ts);
uint64_t ans_tableset_slot_bytes(const struct ans_gpu_tableset* ts, uint64_t chunk_len);
ans_gpu* ans_tableset_gpu(const struct ans_gpu_tableset* ts);
int ans_tableset_dev_encode(struct ans_gpu_tableset* ts, const void* d_syms, int w, const uint64_t* d_starts, uint64_t n,
                            uint64_t chunk_len, uint64_t nchunks, uint8_t* d_slots, uint64_t slot_cap,
                            uint32_t* d_lens, uint32_t* d_status, int gen_kind, uint64_t seed, void* stream);
int ans_tableset_dev_decode(struct ans_gpu_tableset* ts, const uint8_t* d_in, const uint64_t* d_offsets,
                            uint64_t slot_cap, const uint32_t* d_lens, const uint64_t* d_starts, uint64_t n,
                            uint64_t chunk_len, uint64_t nchunks, int gen_kind, uint64_t seed, void* d_syms, int w,
                            uint32_t* d_status, void* stream);
int ans_tableset_host_encode(struct ans_gpu_tableset* ts, const void* syms, int w, uint64_t n, uint64_t chunk_len,
                             const uint64_t* starts, uint64_t nchunks, int gen_kind, uint64_t seed, uint8_t* out,
                             uint64_t out_cap, uint64_t* offsets, uint64_t* lens, uint64_t* total);
int ans_tableset_host_decode(struct ans_gpu_tableset* ts, const uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                             const uint64_t* lens, uint64_t n, uint64_t chunk_len, const uint64_t* starts,
                             uint64_t nchunks, int gen_kind, uint64_t seed, void* out, int w);

// GraphIID<NodeC, EdgeC, ErdosRenyi> per graph over a table set (ans_codecs.hip
// k_graph_encode64 / k_graph_decode64; composed by ans_graph.hip).  Graph g's node labels are
// [node_off[g], node_off[g+1]) of the node-label array, its edge-indicator slots (AllEdgeIndices
// order) [slot_off[g], slot_off[g+1]) of the dense vector, and (encode) its edge labels sorted by
// edge index [edge_off[g], edge_off[g+1]).  kNoTable: no node / edge labels (EmptyCodec).
constexpr uint32_t kNoTable = 0xFFFFFFFFu;
struct GraphLayout {
    const uint64_t* node_off;
    const uint64_t* slot_off;
    const uint64_t* edge_off;
    uint32_t t_node, t_edge, t_bern;
};
int ans_tableset_graph_encode(struct ans_gpu_tableset* ts, const GraphLayout& gl, uint64_t num_graphs,
                              const uint32_t* d_node_labels, const uint8_t* d_dense, const uint32_t* d_edge_labels,
                              int gen_kind, uint64_t seed, uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens,
                              uint32_t* d_status, hipStream_t s);
// edge labels land in pop order at d_edge_scratch[slot_off[g] ..]; d_edge_count[g] = graph g's edges
int ans_tableset_graph_decode(struct ans_gpu_tableset* ts, const GraphLayout& gl, uint64_t num_graphs,
                              const uint8_t* d_in, const uint64_t* d_offsets, const uint32_t* d_lens, int gen_kind,
                              uint64_t seed, uint32_t* d_node_labels, uint8_t* d_dense, uint32_t* d_edge_scratch,
                              uint64_t* d_edge_count, uint32_t* d_status, hipStream_t s);

// Variable-length chunks with the longest chunk's length known to the caller (lmax > 0): the
// staged fast kernels where the table has them (ans_kernels.hip launch_staged_*), else generic.
extern "C" __attribute__((visibility("hidden"))) int dev_encode_var(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t nchunks, const uint64_t* d_starts,
                   int gen_kind, uint64_t seed, uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens,
                   uint32_t* d_status, void* stream, uint64_t lmax);
extern "C" __attribute__((visibility("hidden"))) int dev_decode_var(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap,
                   const uint32_t* d_lens, uint64_t nchunks, const uint64_t* d_starts, int gen_kind, uint64_t seed,
                   void* d_syms, int sym_bytes, uint32_t* d_status, void* stream, uint64_t lmax);
// lmax for dev_*_var when the staged layout (every chunk padded to the longest, rounded to
// 128 B) stays within twice the symbols plus 64 MiB; 0 (the generic kernels) otherwise
inline uint64_t staged_lmax(uint64_t nchunks, uint64_t maxlen, uint64_t total, int sym_bytes) {
    const uint64_t per = ((maxlen * static_cast<uint64_t>(sym_bytes) + 127) / 128) * 128;
    const uint64_t staged = nchunks * per, budget = 2 * total * static_cast<uint64_t>(sym_bytes) + (64ull << 20);
    return (maxlen == 0 || staged > budget) ? 0 : maxlen;
}
