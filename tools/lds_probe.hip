// tools/lds_probe.hip — does gfx950 LDS honour unaligned ds_write_b32 / ds_read_b32 / b64,
// and what does a per-lane byte-ring write pattern cost?
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__global__ void k_unaligned(unsigned* out) {
    __shared__ __align__(16) unsigned char buf[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) buf[i] = 0;
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned addr = static_cast<unsigned>(reinterpret_cast<uintptr_t>(buf)) + 64 * threadIdx.x + threadIdx.x;  // offset 0,65,130,195
        unsigned v = 0x44332211u + threadIdx.x;
        asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(addr), "v"(v) : "memory");
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned addr = static_cast<unsigned>(reinterpret_cast<uintptr_t>(buf)) + 64 * threadIdx.x + threadIdx.x;
        unsigned r;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr) : "memory");
        out[threadIdx.x] = r;
        unsigned long long r64;
        unsigned a2 = addr + 1;  // unaligned b64 read spanning the written dword
        asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r64) : "v"(a2) : "memory");
        out[8 + 2 * threadIdx.x] = static_cast<unsigned>(r64);
        out[9 + 2 * threadIdx.x] = static_cast<unsigned>(r64 >> 32);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += blockDim.x) out[32 + i] = buf[i];
}

// Cost of each lane writing 4 bytes at a random byte offset into its own 128-B ring
// (rows contiguous, stride S), vs the aligned pattern.
template <int S, bool kAligned>
__global__ __launch_bounds__(256) void k_ring(unsigned* out, int iters) {
    __shared__ __align__(16) unsigned char ring[256 * S + 16];
    unsigned base = static_cast<unsigned>(reinterpret_cast<uintptr_t>(ring)) + threadIdx.x * S;
    unsigned pos = threadIdx.x * 7u;
    unsigned v = threadIdx.x;
    for (int it = 0; it < iters; ++it) {
        pos += (v & 3u);  // 0..3 bytes per step, per-lane
        unsigned off = (pos & 127u);
        if (kAligned) off &= ~3u;
        else off = off > 124u ? 124u : off;
        unsigned a = base + off;
        asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
        v = v * 1664525u + 1013904223u;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    out[blockIdx.x * 256 + threadIdx.x] = ring[threadIdx.x * S];
}

int main() {
    unsigned* d;
    hipMalloc(&d, 4 << 20);
    hipMemset(d, 0, 4 << 20);
    k_unaligned<<<1, 64>>>(d);
    unsigned h[288];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("unaligned ds_read_b32 back: %08x %08x %08x %08x (expect 44332211..44332214)\n", h[0], h[1], h[2], h[3]);
    printf("unaligned ds_read_b64 (+1): ");
    for (int i = 0; i < 4; ++i) printf("%08x%08x ", h[9 + 2 * i], h[8 + 2 * i]);
    printf("\nbytes around offsets 0,65,130,195:\n");
    for (int t = 0; t < 4; ++t) {
        int o = 64 * t + t;
        printf("  off %3d:", o);
        for (int k = -1; k < 5; ++k) printf(" %02x", h[32 + o + k] & 0xff);
        printf("\n");
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, const char* name) {
        const int blocks = 256 * 4, iters = 4096;
        kern<<<blocks, 256>>>(d, iters);
        hipEventRecord(e0);
        kern<<<blocks, 256>>>(d, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double wave_instr = double(blocks) * 4 * iters;
        printf("%-28s %.3f ms  %.2f LDS-cycles(@2.4GHz) per wave-write per CU\n", name, ms,
               ms * 1e-3 * 2.4e9 * 256 / wave_instr);
    };
    run(k_ring<128, true>, "ring S=128 aligned");
    run(k_ring<128, false>, "ring S=128 unaligned");
    run(k_ring<132, false>, "ring S=132 unaligned");
    run(k_ring<136, false>, "ring S=136 unaligned");
    return 0;
}
