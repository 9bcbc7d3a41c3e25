// tools/unaligned_probe.hip — do 8-byte global loads at 4-byte-aligned (not 8-aligned) addresses
// return the right words on gfx950, and at what random-gather rate (the wide encoder reads
// (cum[s], cum[s+1]) pairs from a u32 cdf array)?
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512) void k_pairs(const uint32_t* __restrict__ cum, uint32_t mask, uint32_t* bad,
                                               unsigned* out, int iters) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x[8], acc = 0, nbad = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (tid * 2654435761u) ^ (j * 0x9E3779B9u);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t s = x[j] & mask;
            typedef unsigned v2u __attribute__((ext_vector_type(2)));
            typedef __attribute__((address_space(1))) const v2u gu2;
            const v2u v = *reinterpret_cast<gu2*>(reinterpret_cast<uintptr_t>(cum + s));  // 4-aligned only
            nbad += (v.x != s * 3u || v.y != (s + 1) * 3u) ? 1u : 0u;
            acc ^= v.x + v.y;
            x[j] = x[j] * 1664525u + 1013904223u;
        }
    }
    out[tid] = acc;
    if (nbad) atomicAdd(bad, nbad);
}

int main() {
    const uint32_t n = 1u << 16;
    std::vector<uint32_t> h(n + 2);
    for (uint32_t i = 0; i < n + 2; ++i) h[i] = 3u * i;
    uint32_t *d, *bad;
    unsigned* out;
    const int blocks = 512;
    if (hipMalloc(&d, 4 * (n + 2)) != hipSuccess || hipMalloc(&bad, 4) != hipSuccess ||
        hipMalloc(&out, 4 * blocks * 512) != hipSuccess)
        return 1;
    (void)hipMemcpy(d, h.data(), 4 * (n + 2), hipMemcpyHostToDevice);
    (void)hipMemset(bad, 0, 4);
    k_pairs<<<blocks, 512>>>(d, n - 1, bad, out, 4);
    if (hipDeviceSynchronize() != hipSuccess) { printf("fault\n"); return 1; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_pairs<<<blocks, 512>>>(d, n - 1, bad, out, 256);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint32_t hb = 0;
    (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("4-aligned 8-B loads: %u wrong pairs; %.2f G lane-loads/s from a 256 KiB table\n", hb,
           blocks * 512.0 * 256 * 8 / (ms * 1e-3) / 1e9);
    return 0;
}
