// ans_ctx.hpp — the GPU context and table handles behind the C ABI (include/ans_capi.h),
// shared by the HIP translation units of the library (ans_kernels.hip, ans_graph.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "ans_fast.hpp"
#include "ans_table.hpp"

using namespace shuffle_coding;

// Host-buffer pipeline (ans_gpu_encode_chunks / ans_gpu_decode_chunks): batches of chunks
// flow through kPipeDepth workspace slots, so that the H2D copy of batch b+1, the kernels of
// batch b and the D2H copy of batch b-1 overlap.  Kernels alternate between
// two compute streams (the context's and s_comp2): a batch's kernels occupy few CUs for about
// one chain latency (~1 ms for 4096-symbol chunks), so consecutive batches must overlap too.
// Four streams in all, the per-process hardware queue count.  The workspace persists in the
// context and grows on demand.
constexpr int kPipeDepth = 3;
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
    PipeSlot slot[kPipeDepth];
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
    hipStream_t stream;
    HostPipe* pipe;
    uint64_t batch_bytes;  // symbol bytes per pipeline batch (0 = default)
    void* d_scratch;       // device scratch of the device-resident graph calls (ans_graph.hip)
    size_t cap_scratch;
};

struct ans_gpu_table {
    ans_gpu* g;
    DevTable t;
    void* d_mem;
    uint32_t lds_bytes;  // 0 = table read from global memory (L2-resident)
    FastTable ft;        // throughput path (ans_fast.hpp) when ft.usable
    void* d_fast;
};

#define ANS_HIP_TRY(expr)                                                                              \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) {                                                                        \
            std::fprintf(stderr, "[shuffle-coding_amd] %s failed: %s\n", #expr, hipGetErrorString(e_)); \
            return ANS_E_DEVICE;                                                                       \
        }                                                                                              \
    } while (0)

// Variable-chunk encode of device-resident symbols into a host container (ans_kernels.hip):
// the body of ans_gpu_encode_var_chunks; starts is a host array of nchunks + 1 entries.
int ans_encode_var_from_device(ans_gpu_table* gt, const void* d_syms, int sym_bytes, uint64_t nchunks,
                               const uint64_t* starts, uint8_t* out, uint64_t out_cap, uint64_t* offsets,
                               uint64_t* lens, uint64_t* total, int gen_kind = ANS_GEN_ZEROS, uint64_t seed = 0);
