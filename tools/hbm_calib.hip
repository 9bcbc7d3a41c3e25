// tools/hbm_calib.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE for the fast kernels'
// access pattern (MI355X_MICROARCH.md §HBM: "other access widths are uncalibrated: calibrate on a
// known byte count in your own access pattern").
//
// One lane per 4096-byte chunk; each lane moves its chunk in 64-byte groups (four dwordx4) with
// `gap` x s_sleep(127) (~8k cycles each) between groups, as k_encode / k_decode do between
// points.  Exactly 2^30 bytes are read (rd) or written (wr); a 4-byte sink per lane is written by rd.
// Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_calib.hip -o tools/hbm_calib
// Run under: rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./tools/hbm_calib <gap>   (and WRITE_SIZE)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr unsigned long long kBytes = 1ull << 30;
constexpr int kChunk = 4096;

__global__ __launch_bounds__(512) void rd(const uint4* __restrict__ src, unsigned* __restrict__ sink, int gap) {
    const unsigned long long c = static_cast<unsigned long long>(blockIdx.x) * 512 + threadIdx.x;
    const uint4* p = src + c * (kChunk / 16);
    unsigned acc = 0;
    for (int g = kChunk / 64 - 1; g >= 0; --g) {
        const uint4 a = p[4 * g], b = p[4 * g + 1], d = p[4 * g + 2], e = p[4 * g + 3];
        acc += a.x ^ b.y ^ d.z ^ e.w;
        for (int s = 0; s < gap; ++s) __builtin_amdgcn_s_sleep(127);
    }
    sink[c] = acc;
}

__global__ __launch_bounds__(512) void wr(uint4* __restrict__ dst, int gap) {
    const unsigned long long c = static_cast<unsigned long long>(blockIdx.x) * 512 + threadIdx.x;
    uint4* p = dst + c * (kChunk / 16);
    for (int g = 0; g < kChunk / 64; ++g) {
        const uint4 v = make_uint4(g, c, g ^ 7, 1);
        p[4 * g] = v;
        p[4 * g + 1] = v;
        p[4 * g + 2] = v;
        p[4 * g + 3] = v;
        for (int s = 0; s < gap; ++s) __builtin_amdgcn_s_sleep(127);
    }
}

int main(int argc, char** argv) {
    const int gap = argc > 1 ? atoi(argv[1]) : 0;
    void *a = nullptr, *b = nullptr, *sink = nullptr;
    const unsigned nlanes = kBytes / kChunk;
    if (hipMalloc(&a, kBytes) != hipSuccess || hipMalloc(&b, kBytes) != hipSuccess ||
        hipMalloc(&sink, 4ull * nlanes) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    (void)hipMemset(a, 1, kBytes);
    hipEvent_t e0, e1, e2;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventCreate(&e2);
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0, nullptr);
        rd<<<nlanes / 512, 512>>>(static_cast<const uint4*>(a), static_cast<unsigned*>(sink), gap);
        (void)hipEventRecord(e1, nullptr);
        wr<<<nlanes / 512, 512>>>(static_cast<uint4*>(b), gap);
        (void)hipEventRecord(e2, nullptr);
        (void)hipEventSynchronize(e2);
        float t1 = 0, t2 = 0;
        (void)hipEventElapsedTime(&t1, e0, e1);
        (void)hipEventElapsedTime(&t2, e1, e2);
        printf("gap %d rep %d: rd %.3f ms (%.0f GB/s)  wr %.3f ms (%.0f GB/s)\n", gap, rep, t1, kBytes / t1 / 1e6, t2,
               kBytes / t2 / 1e6);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    return 0;
}
