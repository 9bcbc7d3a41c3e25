// ans_graph.hip — the graph models' bulk-IID caller on the GPU: DenseSetIID over
// AllEdgeIndices (src/graph_codec.rs:105-205), i.e. ErdosRenyi's edge set coded as
// IID<Bernoulli> over every possible edge slot.
//
// An edge set becomes a dense u8 vector over the reference's alphabet order
// (AllEdgeIndices::into_iter, src/graph_codec.rs:187-199: the self-loops (i,i) first when
// allowed, then for j in 0..n, i in 0..j the pair (i,j), followed by (j,i) when directed).
// That vector is coded by the bulk chunk path (ans_kernels.hip) with the Bernoulli table, and
// decoding turns the dense vector back into the edge list in alphabet order, which is the
// order DenseSetIID::pop yields (src/graph_codec.rs:117-120).  The compaction is a tile count,
// a scan of the tile counts and an emit pass whose in-tile positions come from a wave prefix
// sum (DPP row shifts through __shfl_up) and a per-wave LDS carry.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "ans_ctx.hpp"

namespace {

#define HIP_TRY ANS_HIP_TRY

constexpr int kTileThreads = 256;
constexpr uint64_t kTileSlots = 16 * kTileThreads;  // 16 slots (one uint4) per thread

struct EdgeSpace {
    uint64_t n;
    uint32_t directed, loops;
};

// num_all_edge_indices (src/graph_codec.rs:203-205)
__host__ __device__ inline uint64_t alphabet_len(const EdgeSpace& e) {
    const uint64_t pairs = e.n > 0 ? e.n * (e.n - 1) / 2 : 0;
    return (e.loops ? e.n : 0) + (e.directed ? 2 * pairs : pairs);
}

// Position of edge (i, j) in AllEdgeIndices order; ~0 when it is not in the alphabet (the
// reference's DenseSetIID::dense then panics: assert!(x.is_empty()), graph_codec.rs:137).
__device__ inline uint64_t edge_slot(const EdgeSpace& e, uint32_t i, uint32_t j) {
    if (i >= e.n || j >= e.n) return ~0ull;
    if (i == j) return e.loops ? i : ~0ull;
    const uint64_t base = e.loops ? e.n : 0;
    if (!e.directed) {
        if (i > j) return ~0ull;  // undirected alphabet holds (i, j) with i < j only
        return base + static_cast<uint64_t>(j) * (j - 1) / 2 + i;
    }
    const uint64_t a = min(i, j), b = max(i, j);
    return base + 2 * (b * (b - 1) / 2 + a) + (i > j ? 1 : 0);
}

// Inverse of edge_slot for a slot of the alphabet.
__device__ inline void slot_edge(const EdgeSpace& e, uint64_t t, uint32_t& i, uint32_t& j) {
    if (e.loops) {
        if (t < e.n) {
            i = j = static_cast<uint32_t>(t);
            return;
        }
        t -= e.n;
    }
    const uint64_t pair = e.directed ? t >> 1 : t;
    // largest b with b(b-1)/2 <= pair
    uint64_t b = static_cast<uint64_t>((1.0 + sqrt(1.0 + 8.0 * static_cast<double>(pair))) * 0.5);
    while (b * (b - 1) / 2 > pair) --b;
    while ((b + 1) * b / 2 <= pair) ++b;
    const uint64_t a = pair - b * (b - 1) / 2;
    const bool flip = e.directed && (t & 1);
    i = static_cast<uint32_t>(flip ? b : a);
    j = static_cast<uint32_t>(flip ? a : b);
}

// DenseSetIID::dense (src/graph_codec.rs:133-138): one lane per edge sets its slot to 1
// (duplicates collapse, as the reference's HashSet does).
__global__ __launch_bounds__(256) void k_edges_to_dense(EdgeSpace e, const uint32_t* __restrict__ edges, uint64_t m,
                                                        uint8_t* __restrict__ dense, uint32_t* __restrict__ status) {
    const uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint64_t s = edge_slot(e, edges[2 * k], edges[2 * k + 1]);
    if (s == ~0ull) {
        atomicOr(status, 1u << ANS_E_SYMBOL);
        return;
    }
    dense[s] = 1;
}

__device__ inline uint32_t nonzero_bytes(uint32_t w) {
    // per byte: 1 if nonzero, then popcount of the flag bits
    const uint32_t t = (w | (w >> 1) | (w >> 2) | (w >> 3) | (w >> 4) | (w >> 5) | (w >> 6) | (w >> 7)) & 0x01010101u;
    return __builtin_popcount(t);
}

__device__ inline uint4 load_tile_word(const uint8_t* dense, uint64_t len, uint64_t pos) {
    if (pos + 16 <= len) return *reinterpret_cast<const uint4*>(dense + pos);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint64_t b = pos; b < len && b < pos + 16; ++b)
        w[(b - pos) / 4] |= static_cast<uint32_t>(dense[b] != 0) << (8 * ((b - pos) % 4));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ inline uint32_t count16(const uint4& v) {
    return nonzero_bytes(v.x) + nonzero_bytes(v.y) + nonzero_bytes(v.z) + nonzero_bytes(v.w);
}

// pass 1: set slots per tile
__global__ __launch_bounds__(kTileThreads) void k_tile_count(const uint8_t* __restrict__ dense, uint64_t len,
                                                             uint32_t* __restrict__ counts) {
    __shared__ uint32_t wsum[kTileThreads / 64];
    const uint64_t pos = blockIdx.x * kTileSlots + 16ull * threadIdx.x;
    uint32_t c = pos < len ? count16(load_tile_word(dense, len, pos)) : 0;
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x / 64] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kTileThreads / 64; ++w) t += wsum[w];
        counts[blockIdx.x] = t;
    }
}

// pass 2: exclusive scan of the tile counts (one workgroup, contiguous segments per thread)
__global__ __launch_bounds__(1024) void k_tile_scan(const uint32_t* __restrict__ counts, uint64_t ntiles,
                                                    uint64_t* __restrict__ base, uint64_t* __restrict__ total) {
    __shared__ uint64_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint64_t per = (ntiles + 1023) / 1024, b = t * per, e = b + per < ntiles ? b + per : ntiles;
    uint64_t sum = 0;
    for (uint64_t i = b; i < e; ++i) sum += counts[i];
    part[t] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - sum;
    for (uint64_t i = b; i < e; ++i) {
        base[i] = run;
        run += counts[i];
    }
    if (t == 1023) *total = part[1023];
}

// pass 3: each set slot becomes its edge at base[tile] + (set slots before it in the tile)
__global__ __launch_bounds__(kTileThreads) void k_tile_emit(EdgeSpace es, const uint8_t* __restrict__ dense,
                                                            uint64_t len, const uint64_t* __restrict__ base,
                                                            uint32_t* __restrict__ edges, uint64_t cap,
                                                            uint32_t* __restrict__ status) {
    __shared__ uint32_t wsum[kTileThreads / 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x / 64;
    const uint64_t pos = blockIdx.x * kTileSlots + 16ull * threadIdx.x;
    const uint4 v = pos < len ? load_tile_word(dense, len, pos) : make_uint4(0, 0, 0, 0);
    const uint32_t c = count16(v);
    uint32_t incl = c;  // inclusive wave prefix sum
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d);
        if (lane >= static_cast<uint32_t>(d)) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t carry = 0;
    for (uint32_t w = 0; w < wave; ++w) carry += wsum[w];
    if (c == 0) return;
    uint64_t out = base[blockIdx.x] + carry + incl - c;
    const uint32_t words[4] = {v.x, v.y, v.z, v.w};
    for (int b = 0; b < 16; ++b) {
        if (((words[b / 4] >> (8 * (b % 4))) & 0xFFu) == 0) continue;
        if (out >= cap) {
            atomicOr(status, 1u << ANS_E_LEN);
            return;
        }
        uint32_t i, j;
        slot_edge(es, pos + b, i, j);
        edges[2 * out] = i;
        edges[2 * out + 1] = j;
        ++out;
    }
}

// ---- datasets of graphs: graph g's alphabet occupies slots [S[g], S[g+1]) of one dense vector

// index of the graph holding position x: the last g with bounds[g] <= x (bounds non-decreasing)
__device__ inline uint64_t graph_of(const uint64_t* bounds, uint64_t num_graphs, uint64_t x) {
    uint64_t lo = 0, hi = num_graphs;  // bounds[lo] <= x < bounds[hi]
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) / 2;
        if (bounds[mid] <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}

// one lane per edge: its graph from the edge offsets, its slot inside that graph's alphabet
__global__ __launch_bounds__(256) void k_edges_to_dense_multi(uint32_t directed, uint32_t loops,
                                                              const uint32_t* __restrict__ num_nodes,
                                                              const uint64_t* __restrict__ S,
                                                              const uint64_t* __restrict__ edge_offsets,
                                                              uint64_t num_graphs, const uint32_t* __restrict__ edges,
                                                              uint64_t m, uint8_t* __restrict__ dense,
                                                              uint32_t* __restrict__ status) {
    const uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint64_t g = graph_of(edge_offsets, num_graphs, k);
    const EdgeSpace e{num_nodes[g], directed, loops};
    const uint64_t s = edge_slot(e, edges[2 * k], edges[2 * k + 1]);
    if (s == ~0ull) {
        atomicOr(status, 1u << ANS_E_SYMBOL);
        return;
    }
    dense[S[g] + s] = 1;
}

// pass 3 for datasets: like k_tile_emit, each set slot mapped to (graph, local slot) first
__global__ __launch_bounds__(kTileThreads) void k_tile_emit_multi(uint32_t directed, uint32_t loops,
                                                                  const uint32_t* __restrict__ num_nodes,
                                                                  const uint64_t* __restrict__ S, uint64_t num_graphs,
                                                                  const uint8_t* __restrict__ dense, uint64_t len,
                                                                  const uint64_t* __restrict__ base,
                                                                  uint32_t* __restrict__ edges, uint64_t cap,
                                                                  uint32_t* __restrict__ status) {
    __shared__ uint32_t wsum[kTileThreads / 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x / 64;
    const uint64_t pos = blockIdx.x * kTileSlots + 16ull * threadIdx.x;
    const uint4 v = pos < len ? load_tile_word(dense, len, pos) : make_uint4(0, 0, 0, 0);
    const uint32_t c = count16(v);
    uint32_t incl = c;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d);
        if (lane >= static_cast<uint32_t>(d)) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t carry = 0;
    for (uint32_t w = 0; w < wave; ++w) carry += wsum[w];
    if (c == 0) return;
    uint64_t out = base[blockIdx.x] + carry + incl - c;
    const uint32_t words[4] = {v.x, v.y, v.z, v.w};
    for (int b = 0; b < 16; ++b) {
        if (((words[b / 4] >> (8 * (b % 4))) & 0xFFu) == 0) continue;
        if (out >= cap) {
            atomicOr(status, 1u << ANS_E_LEN);
            return;
        }
        const uint64_t x = pos + b;
        const uint64_t g = graph_of(S, num_graphs, x);
        uint32_t i, j;
        slot_edge(EdgeSpace{num_nodes[g], directed, loops}, x - S[g], i, j);
        edges[2 * out] = i;
        edges[2 * out + 1] = j;
        ++out;
    }
}

// per graph: set slots before S[g] (tile base + the partial tile), i.e. graph g's first edge
__global__ __launch_bounds__(256) void k_graph_edge_offsets(const uint8_t* __restrict__ dense,
                                                            const uint64_t* __restrict__ S, uint64_t num_graphs,
                                                            const uint64_t* __restrict__ base,
                                                            const uint64_t* __restrict__ total,
                                                            uint64_t* __restrict__ edge_offsets) {
    const uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (g > num_graphs) return;
    if (g == num_graphs) {
        edge_offsets[g] = *total;
        return;
    }
    const uint64_t x = S[g], tile = x / kTileSlots;
    uint64_t cnt = base[tile];
    for (uint64_t y = tile * kTileSlots; y < x; ++y) cnt += dense[y] != 0;
    edge_offsets[g] = cnt;
}

// ---- labelled graphs (GraphIID, src/graph_codec.rs:19-94): EdgesIID::split sorts the (index,
// label) pairs by the index, an EdgeIndex = (usize, usize) compared as a tuple
// (src/graph_codec.rs:82-85), and EdgesIID::pop returns `indices.sort_unstable()` zipped with the
// labels (src/graph_codec.rs:67-71).  That lexicographic order is not the alphabet order
// (AllEdgeIndices runs j-major), so both sides rank edges through a second indicator vector over
// the same pairs laid out row-major: graph g's pairs occupy [S[g], S[g+1]) of it too, and a set
// slot's rank among the set slots (the tile count / scan above) is the edge's sorted position.

// Row-major position of an alphabet pair (i, j) (undirected pairs have i <= j).
__device__ inline uint64_t row_slot(const EdgeSpace& e, uint32_t i, uint32_t j) {
    const uint64_t n = e.n, a = i, b = j;
    if (e.directed) return e.loops ? a * n + b : a * (n - 1) + (b < a ? b : b - 1);
    return e.loops ? a * (2 * n - a + 1) / 2 + (b - a) : a * (2 * n - a - 1) / 2 + (b - a - 1);
}

// Inverse of row_slot.
__device__ inline void row_edge(const EdgeSpace& e, uint64_t r, uint32_t& i, uint32_t& j) {
    const uint64_t n = e.n;
    if (e.directed) {
        if (e.loops) {
            i = static_cast<uint32_t>(r / n);
            j = static_cast<uint32_t>(r % n);
        } else {
            const uint64_t a = r / (n - 1), c = r % (n - 1);
            i = static_cast<uint32_t>(a);
            j = static_cast<uint32_t>(c < a ? c : c + 1);
        }
        return;
    }
    auto start = [&](uint64_t a) { return e.loops ? a * (2 * n - a + 1) / 2 : a * (2 * n - a - 1) / 2; };
    uint64_t lo = 0, hi = e.loops ? n : n - 1;  // the last row a in [lo, hi) with start(a) <= r
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) / 2;
        if (start(mid) <= r) lo = mid;
        else hi = mid;
    }
    i = static_cast<uint32_t>(lo);
    j = static_cast<uint32_t>(lo + (e.loops ? 0 : 1) + (r - start(lo)));
}

// Encode side, one lane per edge: the alphabet-order indicator (DenseSetIID::dense) and, for
// labelled edges, the row-major indicator with the edge's index (row_edge_id = k + 1; a second
// edge on the same pair is ANS_E_SYMBOL: its label would have no slot of its own).
__global__ __launch_bounds__(256) void k_graph_edges_in(uint32_t directed, uint32_t loops,
                                                        const uint32_t* __restrict__ num_nodes,
                                                        const uint64_t* __restrict__ S,
                                                        const uint64_t* __restrict__ edge_offsets, uint64_t num_graphs,
                                                        const uint32_t* __restrict__ edges, uint64_t m,
                                                        uint8_t* __restrict__ dense, uint8_t* __restrict__ row_dense,
                                                        uint32_t* __restrict__ row_edge_id,
                                                        uint32_t* __restrict__ status) {
    const uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint64_t g = graph_of(edge_offsets, num_graphs, k);
    const EdgeSpace e{num_nodes[g], directed, loops};
    const uint32_t i = edges[2 * k], j = edges[2 * k + 1];
    const uint64_t s = edge_slot(e, i, j);
    if (s == ~0ull) {
        atomicOr(status, 1u << ANS_E_SYMBOL);
        return;
    }
    dense[S[g] + s] = 1;
    if (!row_dense) return;
    const uint64_t r = S[g] + row_slot(e, i, j);
    if (atomicCAS(&row_edge_id[r], 0u, static_cast<uint32_t>(k + 1)) != 0u) {
        atomicOr(status, 1u << ANS_E_SYMBOL);
        return;
    }
    row_dense[r] = 1;
}

// Encode side: every set row-major slot puts its edge's label at the slot's rank (the labels of
// all graphs sorted by (graph, edge index)).
__global__ __launch_bounds__(kTileThreads) void k_graph_sort_labels(const uint8_t* __restrict__ row_dense, uint64_t len,
                                                                    const uint64_t* __restrict__ base,
                                                                    const uint32_t* __restrict__ row_edge_id,
                                                                    const uint32_t* __restrict__ labels, uint64_t m,
                                                                    uint32_t* __restrict__ sorted) {
    __shared__ uint32_t wsum[kTileThreads / 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x / 64;
    const uint64_t pos = blockIdx.x * kTileSlots + 16ull * threadIdx.x;
    const uint4 v = pos < len ? load_tile_word(row_dense, len, pos) : make_uint4(0, 0, 0, 0);
    const uint32_t c = count16(v);
    uint32_t incl = c;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d);
        if (lane >= static_cast<uint32_t>(d)) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t carry = 0;
    for (uint32_t w = 0; w < wave; ++w) carry += wsum[w];
    if (c == 0) return;
    uint64_t out = base[blockIdx.x] + carry + incl - c;
    const uint32_t words[4] = {v.x, v.y, v.z, v.w};
    for (int b = 0; b < 16; ++b) {
        if (((words[b / 4] >> (8 * (b % 4))) & 0xFFu) == 0) continue;
        const uint32_t id = row_edge_id[pos + b];
        if (out < m && id) sorted[out] = labels[id - 1];
        ++out;
    }
}

// Decode side, one lane per alphabet slot: a set slot marks its pair's row-major slot.
__global__ __launch_bounds__(256) void k_graph_slots_to_rows(uint32_t directed, uint32_t loops,
                                                             const uint32_t* __restrict__ num_nodes,
                                                             const uint64_t* __restrict__ S, uint64_t num_graphs,
                                                             const uint8_t* __restrict__ dense, uint64_t len,
                                                             uint8_t* __restrict__ row_dense) {
    const uint64_t x = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (x >= len || !dense[x]) return;
    const uint64_t g = graph_of(S, num_graphs, x);
    const EdgeSpace e{num_nodes[g], directed, loops};
    uint32_t i, j;
    slot_edge(e, x - S[g], i, j);
    row_dense[S[g] + row_slot(e, i, j)] = 1;
}

// Decode side: each set row-major slot becomes edge number `rank` (edges sorted by (graph, edge
// index), EdgesIID::pop's order) with the graph's (rank - first)-th popped label beside it.
__global__ __launch_bounds__(kTileThreads) void k_graph_emit_rows(uint32_t directed, uint32_t loops,
                                                                  const uint32_t* __restrict__ num_nodes,
                                                                  const uint64_t* __restrict__ S, uint64_t num_graphs,
                                                                  const uint8_t* __restrict__ row_dense, uint64_t len,
                                                                  const uint64_t* __restrict__ base,
                                                                  const uint64_t* __restrict__ edge_offsets,
                                                                  const uint32_t* __restrict__ label_scratch,
                                                                  uint32_t* __restrict__ edges,
                                                                  uint32_t* __restrict__ labels, uint64_t cap,
                                                                  uint32_t* __restrict__ status) {
    __shared__ uint32_t wsum[kTileThreads / 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x / 64;
    const uint64_t pos = blockIdx.x * kTileSlots + 16ull * threadIdx.x;
    const uint4 v = pos < len ? load_tile_word(row_dense, len, pos) : make_uint4(0, 0, 0, 0);
    const uint32_t c = count16(v);
    uint32_t incl = c;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d);
        if (lane >= static_cast<uint32_t>(d)) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t carry = 0;
    for (uint32_t w = 0; w < wave; ++w) carry += wsum[w];
    if (c == 0) return;
    uint64_t out = base[blockIdx.x] + carry + incl - c;
    const uint32_t words[4] = {v.x, v.y, v.z, v.w};
    for (int b = 0; b < 16; ++b) {
        if (((words[b / 4] >> (8 * (b % 4))) & 0xFFu) == 0) continue;
        if (out >= cap) {
            atomicOr(status, 1u << ANS_E_LEN);
            return;
        }
        const uint64_t x = pos + b;
        const uint64_t g = graph_of(S, num_graphs, x);
        uint32_t i, j;
        row_edge(EdgeSpace{num_nodes[g], directed, loops}, x - S[g], i, j);
        edges[2 * out] = i;
        edges[2 * out + 1] = j;
        if (labels) labels[out] = label_scratch[S[g] + (out - edge_offsets[g])];
        ++out;
    }
}

inline unsigned blocks_for(uint64_t lanes, unsigned per) { return static_cast<unsigned>((lanes + per - 1) / per); }

int scratch(ans_gpu* g, size_t bytes, void** out) {
    if (bytes > g->cap_scratch) {
        HIP_TRY(hipStreamSynchronize(g->stream));
        if (g->d_scratch) (void)hipFree(g->d_scratch);
        g->d_scratch = nullptr;
        g->cap_scratch = 0;
        HIP_TRY(hipMalloc(&g->d_scratch, bytes));
        g->cap_scratch = bytes;
    }
    *out = g->d_scratch;
    return ANS_OK;
}

bool valid_space(uint64_t n) { return n < (1ull << 32); }

// Device buffer released at scope exit (host-level graph calls only).
struct Buf {
    void* p = nullptr;
    ~Buf() { if (p) (void)hipFree(p); }
    bool alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 16) == hipSuccess; }
    template <typename T> T* as() const { return static_cast<T*>(p); }
};


}  // namespace

extern "C" {

int ans_edge_alphabet_len(uint64_t num_nodes, int directed, int loops, uint64_t* len) try {
    if (!len || !valid_space(num_nodes)) return ANS_E_ARG;
    *len = alphabet_len(EdgeSpace{num_nodes, directed ? 1u : 0u, loops ? 1u : 0u});
    return ANS_OK;
} ANS_CATCH

int ans_dev_edges_to_dense(ans_gpu* g, uint64_t num_nodes, int directed, int loops, const uint32_t* d_edges,
                           uint64_t num_edges, uint8_t* d_dense, uint32_t* d_status, void* stream) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!g || !d_status || !valid_space(num_nodes) || (num_edges && !d_edges)) return ANS_E_ARG;
    const EdgeSpace e{num_nodes, directed ? 1u : 0u, loops ? 1u : 0u};
    const uint64_t len = alphabet_len(e);
    if (len && !d_dense) return ANS_E_ARG;
    HIP_TRY(hipSetDevice(g->device));
    const hipStream_t s = stream ? static_cast<hipStream_t>(stream) : g->stream;
    if (len) HIP_TRY(hipMemsetAsync(d_dense, 0, len, s));
    if (num_edges) {
        k_edges_to_dense<<<blocks_for(num_edges, 256), 256, 0, s>>>(e, d_edges, num_edges, d_dense, d_status);
        HIP_TRY(hipGetLastError());
    }
    return ANS_OK;
} ANS_CATCH

int ans_dev_dense_to_edges(ans_gpu* g, uint64_t num_nodes, int directed, int loops, const uint8_t* d_dense,
                           uint32_t* d_edges, uint64_t cap, uint64_t* d_count, uint32_t* d_status, void* stream) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!g || !d_status || !d_count || !valid_space(num_nodes) || (cap && !d_edges)) return ANS_E_ARG;
    const EdgeSpace e{num_nodes, directed ? 1u : 0u, loops ? 1u : 0u};
    const uint64_t len = alphabet_len(e);
    HIP_TRY(hipSetDevice(g->device));
    const hipStream_t s = stream ? static_cast<hipStream_t>(stream) : g->stream;
    if (len == 0) {
        HIP_TRY(hipMemsetAsync(d_count, 0, sizeof(uint64_t), s));
        return ANS_OK;
    }
    if (!d_dense) return ANS_E_ARG;
    const uint64_t ntiles = (len + kTileSlots - 1) / kTileSlots;
    if (ntiles > 0xFFFFFFFFull) return ANS_E_ARG;
    void* scr = nullptr;
    int rc = scratch(g, ntiles * (sizeof(uint32_t) + sizeof(uint64_t)) + 16, &scr);
    if (rc) return rc;
    auto* base = static_cast<uint64_t*>(scr);
    auto* counts = reinterpret_cast<uint32_t*>(base + ntiles);
    k_tile_count<<<static_cast<unsigned>(ntiles), kTileThreads, 0, s>>>(d_dense, len, counts);
    HIP_TRY(hipGetLastError());
    k_tile_scan<<<1, 1024, 0, s>>>(counts, ntiles, base, d_count);
    HIP_TRY(hipGetLastError());
    k_tile_emit<<<static_cast<unsigned>(ntiles), kTileThreads, 0, s>>>(e, d_dense, len, base, d_edges, cap, d_status);
    HIP_TRY(hipGetLastError());
    return ANS_OK;
} ANS_CATCH

// ErdosRenyi / DenseSetIID<EdgeIndex, AllEdgeIndices>::push (src/graph_codec.rs:111-115,
// 152-155), chunked: the edge set's dense vector, coded with the Bernoulli table gt
// (ans_table_create_bernoulli) by the bulk path; chunk j is one reference message over
// alphabet slots [j*chunk_len, (j+1)*chunk_len).  Container as ans_gpu_encode_chunks.
int ans_gpu_dense_set_encode(ans_gpu_table* gt, uint64_t num_nodes, int directed, int loops, const uint32_t* edges,
                             uint64_t num_edges, uint64_t chunk_len, uint8_t* out, uint64_t out_cap,
                             uint64_t* offsets, uint64_t* lens, uint64_t* total) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !total || chunk_len == 0 || !valid_space(num_nodes) || (num_edges && !edges)) return ANS_E_ARG;
    if (gt->t.nsym != 2) return ANS_E_ARG;  // a Bernoulli table
    const EdgeSpace e{num_nodes, directed ? 1u : 0u, loops ? 1u : 0u};
    const uint64_t len = alphabet_len(e), nchunks = (len + chunk_len - 1) / chunk_len;
    if (out && nchunks && (!offsets || !lens)) return ANS_E_ARG;
    *total = 0;
    ans_gpu* g = gt->g;
    HIP_TRY(hipSetDevice(g->device));
    const hipStream_t s = g->stream;
    uint64_t slot_cap = 0;
    ans_gpu_slot_capacity(gt, chunk_len, &slot_cap);
    Buf d_dense, d_edges, d_status, d_slots, d_lens, d_offs, d_out;
    if (!d_dense.alloc(len + 16) || !d_edges.alloc(8 * num_edges) || !d_status.alloc(16) ||
        !d_slots.alloc(nchunks * slot_cap) || !d_lens.alloc(4 * nchunks) || !d_offs.alloc(8 * nchunks))
        return ANS_E_DEVICE;
    if (num_edges) HIP_TRY(hipMemcpyAsync(d_edges.p, edges, 8 * num_edges, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(d_status.p, 0, 4, s));
    int rc = ans_dev_edges_to_dense(g, num_nodes, directed, loops, d_edges.as<uint32_t>(), num_edges,
                                    d_dense.as<uint8_t>(), d_status.as<uint32_t>(), s);
    if (rc) return rc;
    rc = ans_dev_encode_chunks(gt, d_dense.p, 1, len, chunk_len, d_slots.as<uint8_t>(), slot_cap,
                               d_lens.as<uint32_t>(), d_status.as<uint32_t>(), s);
    if (rc) return rc;
    int st = 0;
    if ((rc = ans_dev_status(g, d_status.as<uint32_t>(), s, &st))) return rc;
    if (st) return st;
    std::vector<uint32_t> hl(nchunks);
    if (nchunks) HIP_TRY(hipMemcpy(hl.data(), d_lens.p, 4 * nchunks, hipMemcpyDeviceToHost));
    std::vector<uint64_t> off(nchunks);
    uint64_t acc = 0;
    for (uint64_t j = 0; j < nchunks; ++j) {
        off[j] = acc;
        acc += hl[j];
    }
    *total = acc;
    if (!out) return ANS_OK;
    if (out_cap < acc) return ANS_E_LEN;
    for (uint64_t j = 0; j < nchunks; ++j) {
        offsets[j] = off[j];
        lens[j] = hl[j];
    }
    if (!acc) return ANS_OK;
    if (!d_out.alloc(acc + 16)) return ANS_E_DEVICE;
    HIP_TRY(hipMemcpyAsync(d_offs.p, off.data(), 8 * nchunks, hipMemcpyHostToDevice, s));
    if ((rc = ans_dev_compact(g, d_slots.as<uint8_t>(), slot_cap, d_lens.as<uint32_t>(), d_offs.as<uint64_t>(), nchunks,
                              d_out.as<uint8_t>(), s)))
        return rc;
    HIP_TRY(hipMemcpyAsync(out, d_out.p, acc, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return ANS_OK;
} ANS_CATCH

// DenseSetIID::pop (src/graph_codec.rs:117-120), chunked: decodes the dense vector and
// returns the edges in alphabet order (edges[2k], edges[2k+1]); *num_edges receives the
// count, ANS_E_LEN if it exceeds cap (edges then holds the first cap).
int ans_gpu_dense_set_decode(ans_gpu_table* gt, uint64_t num_nodes, int directed, int loops, const uint8_t* in,
                             uint64_t in_len, const uint64_t* offsets, const uint64_t* lens, uint64_t chunk_len,
                             uint32_t* edges, uint64_t cap, uint64_t* num_edges) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !num_edges || chunk_len == 0 || !valid_space(num_nodes) || (cap && !edges)) return ANS_E_ARG;
    if (gt->t.nsym != 2) return ANS_E_ARG;
    const EdgeSpace e{num_nodes, directed ? 1u : 0u, loops ? 1u : 0u};
    const uint64_t len = alphabet_len(e), nchunks = (len + chunk_len - 1) / chunk_len;
    if (nchunks && (!in || !offsets || !lens)) return ANS_E_ARG;
    *num_edges = 0;
    ans_gpu* g = gt->g;
    HIP_TRY(hipSetDevice(g->device));
    const hipStream_t s = g->stream;
    uint64_t slot_cap = 0, max_len = 0;
    ans_gpu_slot_capacity(gt, chunk_len, &slot_cap);
    std::vector<uint32_t> l32(nchunks);
    for (uint64_t j = 0; j < nchunks; ++j) {
        if (lens[j] > 0xffffffffull || offsets[j] > in_len || lens[j] > in_len - offsets[j]) return ANS_E_LEN;
        l32[j] = static_cast<uint32_t>(lens[j]);
        max_len = std::max<uint64_t>(max_len, l32[j]);
    }
    slot_cap = std::max<uint64_t>(slot_cap, (max_len + 64 + 127) & ~uint64_t(127));
    Buf d_in, d_offs, d_lens, d_slots, d_dense, d_status, d_edges, d_count;
    if (!d_in.alloc(in_len + 16) || !d_offs.alloc(8 * nchunks) || !d_lens.alloc(4 * nchunks) ||
        !d_slots.alloc(nchunks * slot_cap) || !d_dense.alloc(len + 16) || !d_status.alloc(16) ||
        !d_edges.alloc(8 * cap) || !d_count.alloc(16))
        return ANS_E_DEVICE;
    if (in_len) HIP_TRY(hipMemcpyAsync(d_in.p, in, in_len, hipMemcpyHostToDevice, s));
    if (nchunks) {
        HIP_TRY(hipMemcpyAsync(d_offs.p, offsets, 8 * nchunks, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_lens.p, l32.data(), 4 * nchunks, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(hipMemsetAsync(d_status.p, 0, 4, s));
    int rc = ans_dev_expand(g, d_in.as<uint8_t>(), d_offs.as<uint64_t>(), d_lens.as<uint32_t>(), nchunks,
                            d_slots.as<uint8_t>(), slot_cap, s);
    if (rc) return rc;
    rc = ans_dev_decode_chunks(gt, d_slots.as<uint8_t>(), nullptr, slot_cap, d_lens.as<uint32_t>(), len, chunk_len,
                               ANS_GEN_ZEROS, d_dense.p, 1, d_status.as<uint32_t>(), s);
    if (rc) return rc;
    rc = ans_dev_dense_to_edges(g, num_nodes, directed, loops, d_dense.as<uint8_t>(), d_edges.as<uint32_t>(), cap,
                                d_count.as<uint64_t>(), d_status.as<uint32_t>(), s);
    if (rc) return rc;
    int st = 0;
    if ((rc = ans_dev_status(g, d_status.as<uint32_t>(), s, &st))) return rc;
    uint64_t count = 0;
    HIP_TRY(hipMemcpy(&count, d_count.p, 8, hipMemcpyDeviceToHost));
    *num_edges = count;
    if (st && st != ANS_E_LEN) return st;
    const uint64_t got = std::min(count, cap);
    if (got) HIP_TRY(hipMemcpy(edges, d_edges.p, 8 * got, hipMemcpyDeviceToHost));
    return count > cap ? ANS_E_LEN : ANS_OK;
} ANS_CATCH

// Independent<GraphIID<ErdosRenyi>> over a dataset (GraphDatasetParamCodec, src/param_codec.rs:
// 243-293, whose ErdosRenyiParamCodec gives every graph the same Bernoulli, src/param_codec.rs:
// 171-199; DatasetStats::unlabelled, src/benchmark.rs:552-557): graph g is one chunk of the
// variable-chunk path, its stream the reference message of that graph's edge set.
static int dataset_space(uint64_t num_graphs, const uint32_t* num_nodes, int directed, int loops,
                         std::vector<uint64_t>& S) {
    S.assign(num_graphs + 1, 0);
    for (uint64_t g = 0; g < num_graphs; ++g)
        S[g + 1] = S[g] + alphabet_len(EdgeSpace{num_nodes[g], directed ? 1u : 0u, loops ? 1u : 0u});
    return ANS_OK;
}

int ans_gpu_dense_sets_encode(ans_gpu_table* gt, uint64_t num_graphs, const uint32_t* num_nodes, int directed,
                              int loops, const uint32_t* edges, const uint64_t* edge_offsets, uint8_t* out,
                              uint64_t out_cap, uint64_t* offsets, uint64_t* lens, uint64_t* total) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !total || (num_graphs && (!num_nodes || !edge_offsets))) return ANS_E_ARG;
    if (gt->t.nsym != 2) return ANS_E_ARG;
    *total = 0;
    if (num_graphs == 0) return ANS_OK;
    for (uint64_t g = 0; g < num_graphs; ++g)
        if (edge_offsets[g + 1] < edge_offsets[g]) return ANS_E_ARG;
    const uint64_t m = edge_offsets[num_graphs] - edge_offsets[0];
    if (m && !edges) return ANS_E_ARG;
    std::vector<uint64_t> S;
    dataset_space(num_graphs, num_nodes, directed, loops, S);
    ans_gpu* gp = gt->g;
    HIP_TRY(hipSetDevice(gp->device));
    const hipStream_t s = gp->stream;
    std::vector<uint64_t> eo(edge_offsets, edge_offsets + num_graphs + 1);
    for (auto& v : eo) v -= edge_offsets[0];
    Buf d_dense, d_edges, d_nn, d_S, d_eo, d_status;
    if (!d_dense.alloc(S[num_graphs] + 16) || !d_edges.alloc(8 * m) || !d_nn.alloc(4 * num_graphs) ||
        !d_S.alloc(8 * (num_graphs + 1)) || !d_eo.alloc(8 * (num_graphs + 1)) || !d_status.alloc(16))
        return ANS_E_DEVICE;
    if (m) HIP_TRY(hipMemcpyAsync(d_edges.p, edges + 2 * edge_offsets[0], 8 * m, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_nn.p, num_nodes, 4 * num_graphs, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_S.p, S.data(), 8 * (num_graphs + 1), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_eo.p, eo.data(), 8 * (num_graphs + 1), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(d_status.p, 0, 4, s));
    if (S[num_graphs]) HIP_TRY(hipMemsetAsync(d_dense.p, 0, S[num_graphs], s));
    if (m) {
        k_edges_to_dense_multi<<<blocks_for(m, 256), 256, 0, s>>>(directed ? 1u : 0u, loops ? 1u : 0u,
                                                                  d_nn.as<uint32_t>(), d_S.as<uint64_t>(),
                                                                  d_eo.as<uint64_t>(), num_graphs,
                                                                  d_edges.as<uint32_t>(), m, d_dense.as<uint8_t>(),
                                                                  d_status.as<uint32_t>());
        HIP_TRY(hipGetLastError());
    }
    int st = 0;
    int rc = ans_dev_status(gp, d_status.as<uint32_t>(), s, &st);
    if (rc) return rc;
    if (st) return st;
    return ans_encode_var_from_device(gt, d_dense.p, 1, num_graphs, S.data(), out, out_cap, offsets, lens, total);
} ANS_CATCH

int ans_gpu_dense_sets_decode(ans_gpu_table* gt, uint64_t num_graphs, const uint32_t* num_nodes, int directed,
                              int loops, const uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                              const uint64_t* lens, uint32_t* edges, uint64_t cap, uint64_t* edge_offsets) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!gt || !edge_offsets || (num_graphs && (!num_nodes || !offsets || !lens)) || (cap && !edges))
        return ANS_E_ARG;
    if (gt->t.nsym != 2) return ANS_E_ARG;
    edge_offsets[0] = 0;
    if (num_graphs == 0) return ANS_OK;
    std::vector<uint64_t> S;
    dataset_space(num_graphs, num_nodes, directed, loops, S);
    std::vector<uint32_t> l32(num_graphs);
    for (uint64_t g = 0; g < num_graphs; ++g) {
        if (lens[g] > 0xffffffffull || offsets[g] > in_len || lens[g] > in_len - offsets[g]) return ANS_E_LEN;
        l32[g] = static_cast<uint32_t>(lens[g]);
    }
    if (in_len && !in) return ANS_E_ARG;
    const uint64_t len = S[num_graphs];
    ans_gpu* gp = gt->g;
    HIP_TRY(hipSetDevice(gp->device));
    const hipStream_t s = gp->stream;
    const uint64_t ntiles = (len + kTileSlots - 1) / kTileSlots;
    Buf d_in, d_offs, d_lens, d_S, d_nn, d_dense, d_status, d_edges, d_scan, d_eo;
    if (!d_in.alloc(in_len + 128) || !d_offs.alloc(8 * num_graphs) || !d_lens.alloc(4 * num_graphs) ||
        !d_S.alloc(8 * (num_graphs + 1)) || !d_nn.alloc(4 * num_graphs) || !d_dense.alloc(len + 16) ||
        !d_status.alloc(16) || !d_edges.alloc(8 * cap) || !d_scan.alloc(12 * ntiles + 16) ||
        !d_eo.alloc(8 * (num_graphs + 1)))
        return ANS_E_DEVICE;
    if (in_len) HIP_TRY(hipMemcpyAsync(d_in.p, in, in_len, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_offs.p, offsets, 8 * num_graphs, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_lens.p, l32.data(), 4 * num_graphs, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_S.p, S.data(), 8 * (num_graphs + 1), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_nn.p, num_nodes, 4 * num_graphs, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(d_status.p, 0, 16, s));
    uint64_t maxlen = 0;  // the longest graph's slot count: the staged fast decoder (ans_ctx.hpp)
    for (uint64_t g = 0; g < num_graphs; ++g) maxlen = std::max(maxlen, S[g + 1] - S[g]);
    int rc = dev_decode_var(gt, d_in.as<uint8_t>(), d_offs.as<uint64_t>(), 0, d_lens.as<uint32_t>(), num_graphs,
                            d_S.as<uint64_t>(), ANS_GEN_ZEROS, 0, d_dense.p, 1, d_status.as<uint32_t>(), s,
                            staged_lmax(num_graphs, maxlen, len, 1));
    if (rc) return rc;
    auto* base = d_scan.as<uint64_t>();
    auto* counts = reinterpret_cast<uint32_t*>(base + ntiles);
    uint64_t* d_total = d_status.as<uint64_t>() + 1;  // second 8 bytes of the status block
    if (ntiles) {
        k_tile_count<<<static_cast<unsigned>(ntiles), kTileThreads, 0, s>>>(d_dense.as<uint8_t>(), len, counts);
        HIP_TRY(hipGetLastError());
        k_tile_scan<<<1, 1024, 0, s>>>(counts, ntiles, base, d_total);
        HIP_TRY(hipGetLastError());
        k_tile_emit_multi<<<static_cast<unsigned>(ntiles), kTileThreads, 0, s>>>(
            directed ? 1u : 0u, loops ? 1u : 0u, d_nn.as<uint32_t>(), d_S.as<uint64_t>(), num_graphs,
            d_dense.as<uint8_t>(), len, base, d_edges.as<uint32_t>(), cap, d_status.as<uint32_t>());
        HIP_TRY(hipGetLastError());
        k_graph_edge_offsets<<<blocks_for(num_graphs + 1, 256), 256, 0, s>>>(d_dense.as<uint8_t>(), d_S.as<uint64_t>(),
                                                                           num_graphs, base, d_total,
                                                                           d_eo.as<uint64_t>());
        HIP_TRY(hipGetLastError());
    }
    int st = 0;
    if ((rc = ans_dev_status(gp, d_status.as<uint32_t>(), s, &st))) return rc;
    if (st && st != ANS_E_LEN) return st;
    if (ntiles) HIP_TRY(hipMemcpy(edge_offsets, d_eo.p, 8 * (num_graphs + 1), hipMemcpyDeviceToHost));
    else std::fill(edge_offsets, edge_offsets + num_graphs + 1, 0);
    const uint64_t count = edge_offsets[num_graphs];
    const uint64_t got = std::min(count, cap);
    if (got) HIP_TRY(hipMemcpy(edges, d_edges.p, 8 * got, hipMemcpyDeviceToHost));
    return count > cap ? ANS_E_LEN : ANS_OK;
} ANS_CATCH

// ---- GraphIID<NodeC, EdgeC, ErdosRenyi> over a dataset, one message per graph (include/ans_capi.h
// section 5b; src/graph_codec.rs:19-94, the --er models of src/benchmark.rs:308-358)
static bool graph_kind_ok(int k) { return k == ANS_GEN_ZEROS || k == ANS_GEN_EMPTY || k == ANS_GEN_RANDOM; }

// node-label and slot offsets of every graph; ANS_E_ARG for a node count of 2^32 or more
static int graph_offsets(uint64_t num_graphs, const uint32_t* num_nodes, int directed, int loops,
                         std::vector<uint64_t>& NO, std::vector<uint64_t>& S) {
    NO.assign(num_graphs + 1, 0);
    for (uint64_t g = 0; g < num_graphs; ++g) NO[g + 1] = NO[g] + num_nodes[g];
    return dataset_space(num_graphs, num_nodes, directed, loops, S);
}

int ans_gpu_graphs_encode(ans_gpu_tableset* ts, uint32_t node_table, uint32_t edge_table, uint32_t edge_indicator_table,
                          int directed, int loops, uint64_t num_graphs, const uint32_t* num_nodes,
                          const uint32_t* node_labels, const uint32_t* edges, const uint32_t* edge_labels,
                          const uint64_t* edge_offsets, int gen_kind, uint64_t seed, uint8_t* out, uint64_t out_cap,
                          uint64_t* offsets, uint64_t* lens, uint64_t* total) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!ts || !total || !graph_kind_ok(gen_kind) || (num_graphs && (!num_nodes || !edge_offsets))) return ANS_E_ARG;
    *total = 0;
    if (num_graphs == 0) return ANS_OK;
    if (out && (!offsets || !lens)) return ANS_E_ARG;
    const bool nl = node_table != ANS_NO_TABLE, el = edge_table != ANS_NO_TABLE;
    for (uint64_t g = 0; g < num_graphs; ++g)
        if (edge_offsets[g + 1] < edge_offsets[g]) return ANS_E_ARG;
    const uint64_t m = edge_offsets[num_graphs] - edge_offsets[0];
    if (m && (!edges || (el && !edge_labels))) return ANS_E_ARG;
    std::vector<uint64_t> NO, S;
    graph_offsets(num_graphs, num_nodes, directed, loops, NO, S);
    if (nl && NO[num_graphs] && !node_labels) return ANS_E_ARG;
    std::vector<uint64_t> eo(edge_offsets, edge_offsets + num_graphs + 1);
    for (auto& v : eo) v -= edge_offsets[0];
    uint64_t maxlen = 1;  // the longest message in pops: node labels, slots, edge labels
    for (uint64_t g = 0; g < num_graphs; ++g)
        maxlen = std::max(maxlen, (nl ? NO[g + 1] - NO[g] : 0) + (S[g + 1] - S[g]) + (el ? eo[g + 1] - eo[g] : 0));
    const uint64_t slot_cap = ans_tableset_slot_bytes(ts, maxlen), len = S[num_graphs];
    const uint64_t ntiles = (len + kTileSlots - 1) / kTileSlots;
    ans_gpu* gp = ans_tableset_gpu(ts);
    HIP_TRY(hipSetDevice(gp->device));
    const hipStream_t s = gp->stream;
    Buf d_nn, d_NO, d_S, d_eo, d_nl, d_edges, d_el, d_dense, d_rdense, d_rid, d_sorted, d_scan, d_status, d_slots,
        d_lens, d_offs, d_out;
    if (!d_nn.alloc(4 * num_graphs) || !d_NO.alloc(8 * (num_graphs + 1)) || !d_S.alloc(8 * (num_graphs + 1)) ||
        !d_eo.alloc(8 * (num_graphs + 1)) || !d_nl.alloc(nl ? 4 * NO[num_graphs] : 0) || !d_edges.alloc(8 * m) ||
        !d_el.alloc(el ? 4 * m : 0) || !d_dense.alloc(len + 16) || !d_rdense.alloc(el ? len + 16 : 0) ||
        !d_rid.alloc(el ? 4 * len : 0) || !d_sorted.alloc(el ? 4 * m : 0) || !d_scan.alloc(12 * ntiles + 16) ||
        !d_status.alloc(16) || !d_slots.alloc(num_graphs * slot_cap) || !d_lens.alloc(4 * num_graphs) ||
        !d_offs.alloc(8 * num_graphs))
        return ANS_E_DEVICE;
    HIP_TRY(hipMemcpyAsync(d_nn.p, num_nodes, 4 * num_graphs, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_NO.p, NO.data(), 8 * (num_graphs + 1), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_S.p, S.data(), 8 * (num_graphs + 1), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_eo.p, eo.data(), 8 * (num_graphs + 1), hipMemcpyHostToDevice, s));
    if (nl && NO[num_graphs])
        HIP_TRY(hipMemcpyAsync(d_nl.p, node_labels, 4 * NO[num_graphs], hipMemcpyHostToDevice, s));
    if (m) {
        HIP_TRY(hipMemcpyAsync(d_edges.p, edges + 2 * edge_offsets[0], 8 * m, hipMemcpyHostToDevice, s));
        if (el) HIP_TRY(hipMemcpyAsync(d_el.p, edge_labels + edge_offsets[0], 4 * m, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(hipMemsetAsync(d_status.p, 0, 16, s));
    if (len) {
        HIP_TRY(hipMemsetAsync(d_dense.p, 0, len, s));
        if (el) {
            HIP_TRY(hipMemsetAsync(d_rdense.p, 0, len, s));
            HIP_TRY(hipMemsetAsync(d_rid.p, 0, 4 * len, s));
        }
    }
    if (m) {  // DenseSetIID::dense and, for labelled edges, the row-major rank of every edge
        k_graph_edges_in<<<blocks_for(m, 256), 256, 0, s>>>(
            directed ? 1u : 0u, loops ? 1u : 0u, d_nn.as<uint32_t>(), d_S.as<uint64_t>(), d_eo.as<uint64_t>(),
            num_graphs, d_edges.as<uint32_t>(), m, d_dense.as<uint8_t>(), el ? d_rdense.as<uint8_t>() : nullptr,
            d_rid.as<uint32_t>(), d_status.as<uint32_t>());
        HIP_TRY(hipGetLastError());
        if (el && ntiles) {  // EdgesIID::split: the labels sorted by edge index
            auto* base = d_scan.as<uint64_t>();
            auto* counts = reinterpret_cast<uint32_t*>(base + ntiles);
            k_tile_count<<<static_cast<unsigned>(ntiles), kTileThreads, 0, s>>>(d_rdense.as<uint8_t>(), len, counts);
            HIP_TRY(hipGetLastError());
            k_tile_scan<<<1, 1024, 0, s>>>(counts, ntiles, base, d_status.as<uint64_t>() + 1);
            HIP_TRY(hipGetLastError());
            k_graph_sort_labels<<<static_cast<unsigned>(ntiles), kTileThreads, 0, s>>>(
                d_rdense.as<uint8_t>(), len, base, d_rid.as<uint32_t>(), d_el.as<uint32_t>(), m, d_sorted.as<uint32_t>());
            HIP_TRY(hipGetLastError());
        }
    }
    int st = 0;
    int rc = ans_dev_status(gp, d_status.as<uint32_t>(), s, &st);
    if (rc) return rc;
    if (st) return st;
    const GraphLayout gl{d_NO.as<uint64_t>(), d_S.as<uint64_t>(), d_eo.as<uint64_t>(), nl ? node_table : kNoTable,
                         el ? edge_table : kNoTable, edge_indicator_table};
    rc = ans_tableset_graph_encode(ts, gl, num_graphs, d_nl.as<uint32_t>(), d_dense.as<uint8_t>(),
                                   d_sorted.as<uint32_t>(), gen_kind, seed, d_slots.as<uint8_t>(), slot_cap,
                                   d_lens.as<uint32_t>(), d_status.as<uint32_t>(), s);
    if (rc) return rc;
    if ((rc = ans_dev_status(gp, d_status.as<uint32_t>(), s, &st))) return rc;
    if (st) return st;
    std::vector<uint32_t> hl(num_graphs);
    HIP_TRY(hipMemcpy(hl.data(), d_lens.p, 4 * num_graphs, hipMemcpyDeviceToHost));
    std::vector<uint64_t> off(num_graphs);
    uint64_t acc = 0;
    for (uint64_t g = 0; g < num_graphs; ++g) {
        off[g] = acc;
        acc += hl[g];
    }
    *total = acc;
    if (!out) return ANS_OK;
    if (out_cap < acc) return ANS_E_LEN;
    for (uint64_t g = 0; g < num_graphs; ++g) {
        offsets[g] = off[g];
        lens[g] = hl[g];
    }
    if (!d_out.alloc(acc + 16)) return ANS_E_DEVICE;
    HIP_TRY(hipMemcpyAsync(d_offs.p, off.data(), 8 * num_graphs, hipMemcpyHostToDevice, s));
    if ((rc = ans_dev_compact(gp, d_slots.as<uint8_t>(), slot_cap, d_lens.as<uint32_t>(), d_offs.as<uint64_t>(),
                              num_graphs, d_out.as<uint8_t>(), s)))
        return rc;
    HIP_TRY(hipMemcpyAsync(out, d_out.p, acc, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return ANS_OK;
} ANS_CATCH

int ans_gpu_graphs_decode(ans_gpu_tableset* ts, uint32_t node_table, uint32_t edge_table, uint32_t edge_indicator_table,
                          int directed, int loops, uint64_t num_graphs, const uint32_t* num_nodes, const uint8_t* in,
                          uint64_t in_len, const uint64_t* offsets, const uint64_t* lens, int gen_kind, uint64_t seed,
                          uint32_t* node_labels, uint32_t* edges, uint32_t* edge_labels, uint64_t cap,
                          uint64_t* edge_offsets) try {
    (void)hipGetLastError();  // drop a stale error another caller left on this thread
    if (!ts || !edge_offsets || !graph_kind_ok(gen_kind) || (num_graphs && (!num_nodes || !offsets || !lens)))
        return ANS_E_ARG;
    const bool nl = node_table != ANS_NO_TABLE, el = edge_table != ANS_NO_TABLE;
    if (cap && (!edges || (el && !edge_labels))) return ANS_E_ARG;
    edge_offsets[0] = 0;
    if (num_graphs == 0) return ANS_OK;
    if (in_len && !in) return ANS_E_ARG;
    std::vector<uint32_t> l32(num_graphs);
    for (uint64_t g = 0; g < num_graphs; ++g) {
        if (lens[g] > 0xffffffffull || offsets[g] > in_len || lens[g] > in_len - offsets[g]) return ANS_E_LEN;
        l32[g] = static_cast<uint32_t>(lens[g]);
    }
    std::vector<uint64_t> NO, S;
    graph_offsets(num_graphs, num_nodes, directed, loops, NO, S);
    if (nl && NO[num_graphs] && !node_labels) return ANS_E_ARG;
    const uint64_t len = S[num_graphs], ntiles = (len + kTileSlots - 1) / kTileSlots;
    ans_gpu* gp = ans_tableset_gpu(ts);
    HIP_TRY(hipSetDevice(gp->device));
    const hipStream_t s = gp->stream;
    Buf d_in, d_offs, d_lens, d_nn, d_NO, d_S, d_nl, d_dense, d_rdense, d_escr, d_ecnt, d_scan, d_status, d_eo,
        d_edges, d_el;
    if (!d_in.alloc(in_len + 16) || !d_offs.alloc(8 * num_graphs) || !d_lens.alloc(4 * num_graphs) ||
        !d_nn.alloc(4 * num_graphs) || !d_NO.alloc(8 * (num_graphs + 1)) || !d_S.alloc(8 * (num_graphs + 1)) ||
        !d_nl.alloc(nl ? 4 * NO[num_graphs] : 0) || !d_dense.alloc(len + 16) || !d_rdense.alloc(len + 16) ||
        !d_escr.alloc(el ? 4 * len : 0) || !d_ecnt.alloc(8 * num_graphs) || !d_scan.alloc(12 * ntiles + 16) ||
        !d_status.alloc(16) || !d_eo.alloc(8 * (num_graphs + 1)) || !d_edges.alloc(8 * cap) ||
        !d_el.alloc(el ? 4 * cap : 0))
        return ANS_E_DEVICE;
    if (in_len) HIP_TRY(hipMemcpyAsync(d_in.p, in, in_len, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_offs.p, offsets, 8 * num_graphs, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_lens.p, l32.data(), 4 * num_graphs, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_nn.p, num_nodes, 4 * num_graphs, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_NO.p, NO.data(), 8 * (num_graphs + 1), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_S.p, S.data(), 8 * (num_graphs + 1), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(d_status.p, 0, 16, s));
    if (len) HIP_TRY(hipMemsetAsync(d_rdense.p, 0, len, s));
    const GraphLayout gl{d_NO.as<uint64_t>(), d_S.as<uint64_t>(), nullptr, nl ? node_table : kNoTable,
                         el ? edge_table : kNoTable, edge_indicator_table};
    int rc = ans_tableset_graph_decode(ts, gl, num_graphs, d_in.as<uint8_t>(), d_offs.as<uint64_t>(),
                                       d_lens.as<uint32_t>(), gen_kind, seed, d_nl.as<uint32_t>(), d_dense.as<uint8_t>(),
                                       d_escr.as<uint32_t>(), d_ecnt.as<uint64_t>(), d_status.as<uint32_t>(), s);
    if (rc) return rc;
    uint64_t* d_total = d_status.as<uint64_t>() + 1;
    if (ntiles) {  // EdgesIID::pop: the edges sorted by index (row-major rank), labels beside them
        auto* base = d_scan.as<uint64_t>();
        auto* counts = reinterpret_cast<uint32_t*>(base + ntiles);
        k_graph_slots_to_rows<<<blocks_for(len, 256), 256, 0, s>>>(directed ? 1u : 0u, loops ? 1u : 0u,
                                                                   d_nn.as<uint32_t>(), d_S.as<uint64_t>(), num_graphs,
                                                                   d_dense.as<uint8_t>(), len, d_rdense.as<uint8_t>());
        HIP_TRY(hipGetLastError());
        k_tile_count<<<static_cast<unsigned>(ntiles), kTileThreads, 0, s>>>(d_rdense.as<uint8_t>(), len, counts);
        HIP_TRY(hipGetLastError());
        k_tile_scan<<<1, 1024, 0, s>>>(counts, ntiles, base, d_total);
        HIP_TRY(hipGetLastError());
        k_graph_edge_offsets<<<blocks_for(num_graphs + 1, 256), 256, 0, s>>>(
            d_rdense.as<uint8_t>(), d_S.as<uint64_t>(), num_graphs, base, d_total, d_eo.as<uint64_t>());
        HIP_TRY(hipGetLastError());
        k_graph_emit_rows<<<static_cast<unsigned>(ntiles), kTileThreads, 0, s>>>(
            directed ? 1u : 0u, loops ? 1u : 0u, d_nn.as<uint32_t>(), d_S.as<uint64_t>(), num_graphs,
            d_rdense.as<uint8_t>(), len, base, d_eo.as<uint64_t>(), d_escr.as<uint32_t>(), d_edges.as<uint32_t>(),
            el ? d_el.as<uint32_t>() : nullptr, cap, d_status.as<uint32_t>());
        HIP_TRY(hipGetLastError());
    }
    int st = 0;
    if ((rc = ans_dev_status(gp, d_status.as<uint32_t>(), s, &st))) return rc;
    if (st && st != ANS_E_LEN) return st;
    if (ntiles) HIP_TRY(hipMemcpy(edge_offsets, d_eo.p, 8 * (num_graphs + 1), hipMemcpyDeviceToHost));
    else std::fill(edge_offsets, edge_offsets + num_graphs + 1, 0);
    if (nl && NO[num_graphs]) HIP_TRY(hipMemcpy(node_labels, d_nl.p, 4 * NO[num_graphs], hipMemcpyDeviceToHost));
    const uint64_t count = edge_offsets[num_graphs], got = std::min(count, cap);
    if (got) {
        HIP_TRY(hipMemcpy(edges, d_edges.p, 8 * got, hipMemcpyDeviceToHost));
        if (el) HIP_TRY(hipMemcpy(edge_labels, d_el.p, 4 * got, hipMemcpyDeviceToHost));
    }
    return count > cap ? ANS_E_LEN : ANS_OK;
} ANS_CATCH

}  // extern "C"
