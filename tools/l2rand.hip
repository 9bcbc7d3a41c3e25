// tools/l2rand.hip — random-gather rate of a global table (the C4 kernels' row / bucket
// lookups): loads per second chip-wide for table sizes from L1- to L2-resident, 4/8/16-B
// loads, independent (throughput) or dependent (latency chain) addresses.
// Build: hipcc --offload-arch=gfx950 -O3 tools/l2rand.hip -o tools/l2rand
// Usage: tools/l2rand [blocks_per_cu=2] (512-thread blocks)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kIters = 512;
constexpr int kIndep = 8;

// cache-policy variants of a 16-B gather: buffer loads with the gfx950 cache-policy bits
// (aux 1 = sc0, 2 = nt, 16 = sc1, 17 = sc0 sc1)
typedef unsigned v4u __attribute__((ext_vector_type(4)));
template <int kAux>
__global__ __launch_bounds__(512) void k_gather_pol(const uint4* __restrict__ tab, uint32_t mask, unsigned* out) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(tab), 0, 0x7fffffff, 0x00020000);
    uint32_t x[kIndep];
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int j = 0; j < kIndep; ++j) x[j] = (tid * 2654435761u) ^ (j * 0x9E3779B9u);
    uint32_t acc = 0;
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int j = 0; j < kIndep; ++j) {
            const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>((x[j] & mask) * 16), 0, kAux);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
            x[j] = x[j] * 1664525u + 1013904223u;
        }
    }
    out[tid] = acc ^ x[0];
}

template <typename T, bool kDep>
__global__ __launch_bounds__(512) void k_gather(const T* __restrict__ tab, uint32_t mask, unsigned* out) {
    uint32_t x[kIndep];
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int j = 0; j < kIndep; ++j) x[j] = (tid * 2654435761u) ^ (j * 0x9E3779B9u);
    uint32_t acc = 0;
    for (int it = 0; it < kIters; ++it) {
        if constexpr (kDep) {
            // one chain: the next address depends on the loaded value
            const T v = tab[x[0] & mask];
            uint32_t w;
            if constexpr (sizeof(T) == 16) w = reinterpret_cast<const uint4&>(v).x;
            else w = static_cast<uint32_t>(v);
            x[0] = x[0] * 1664525u + 1013904223u + w;
        } else {
#pragma unroll
            for (int j = 0; j < kIndep; ++j) {
                const T v = tab[x[j] & mask];
                uint32_t w;
                if constexpr (sizeof(T) == 16) w = reinterpret_cast<const uint4&>(v).x;
                else w = static_cast<uint32_t>(v);
                acc ^= w;
                x[j] = x[j] * 1664525u + 1013904223u;
            }
        }
    }
    out[tid] = acc ^ x[0];
}

template <typename T, bool kDep>
void run(const char* name, void* tab, size_t bytes, unsigned* out, int blocks) {
    const uint32_t n = static_cast<uint32_t>(bytes / sizeof(T));
    const uint32_t mask = n - 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_gather<T, kDep><<<blocks, 512>>>(static_cast<const T*>(tab), mask, out);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) k_gather<T, kDep><<<blocks, 512>>>(static_cast<const T*>(tab), mask, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double loads = static_cast<double>(reps) * blocks * 512.0 * kIters * (kDep ? 1 : kIndep);
    printf("%-6s %-5s table %8zu KiB: %8.3f ms  %7.2f G lane-loads/s  (%6.1f ns per dependent step)\n", name,
           kDep ? "dep" : "indep", bytes >> 10, ms / reps, loads / (ms * 1e-3) / 1e9,
           kDep ? ms * 1e6 / reps / kIters : 0.0);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

template <int kPol>
void run_pol(const char* name, void* tab, size_t bytes, unsigned* out, int blocks) {
    const uint32_t mask = static_cast<uint32_t>(bytes / 16) - 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_gather_pol<kPol><<<blocks, 512>>>(static_cast<const uint4*>(tab), mask, out);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) k_gather_pol<kPol><<<blocks, 512>>>(static_cast<const uint4*>(tab), mask, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double loads = static_cast<double>(reps) * blocks * 512.0 * kIters * kIndep;
    printf("16B %-9s table %8zu KiB: %8.3f ms  %7.2f G lane-loads/s\n", name, bytes >> 10, ms / reps,
           loads / (ms * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
    const int per_cu = argc > 1 ? atoi(argv[1]) : 2;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int blocks = prop.multiProcessorCount * per_cu;
    printf("CUs %d, %d blocks of 512 (%d waves/SIMD)\n", prop.multiProcessorCount, blocks, per_cu * 2);
    const size_t max_bytes = 4u << 20;
    void* tab = nullptr;
    unsigned* out = nullptr;
    if (hipMalloc(&tab, max_bytes) != hipSuccess || hipMalloc(&out, sizeof(unsigned) * blocks * 512) != hipSuccess) return 1;
    std::vector<uint32_t> h(max_bytes / 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint32_t>(i * 2654435761u);
    if (hipMemcpy(tab, h.data(), max_bytes, hipMemcpyHostToDevice) != hipSuccess) return 1;
    for (size_t kb : {64, 256, 1024, 2048}) {
        const size_t b = kb << 10;
        run_pol<0>("plain", tab, b, out, blocks);
        run_pol<1>("sc0", tab, b, out, blocks);
        run_pol<16>("sc1", tab, b, out, blocks);
        run_pol<17>("sc0sc1", tab, b, out, blocks);
        run_pol<2>("nt", tab, b, out, blocks);
        run_pol<18>("sc1nt", tab, b, out, blocks);
    }
    if (argc > 2) return 0;
    for (size_t kb : {16, 64, 256, 1024, 2048, 4096}) {
        const size_t b = kb << 10;
        run<uint4, false>("16B", tab, b, out, blocks);
        run<uint64_t, false>("8B", tab, b, out, blocks);
        run<uint32_t, false>("4B", tab, b, out, blocks);
        run<uint4, true>("16B", tab, b, out, blocks);
    }
    return 0;
}
