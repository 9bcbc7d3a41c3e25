// tools/b16_probe.hip — does a 16-bit VALU shift on gfx950 clear the destination's upper half,
// and what does its SDWA form (byte source, zero-padded word destination) cost per wave64
// instruction?  (A candidate for the 4-cycle v_lshlrev_b32 in the kernels' LDS addresses.)
// Build: hipcc --offload-arch=gfx950 -O3 tools/b16_probe.hip -o tools/b16_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_sem(unsigned* out, unsigned x) {
    unsigned r0, r1, r2;
    asm volatile("v_mov_b32 %0, -1\n\ts_nop 1\n\tv_lshlrev_b16 %0, 3, %1" : "=&v"(r0) : "v"(x));
    asm volatile("v_mov_b32 %0, -1\n\ts_nop 1\n\tv_lshlrev_b16_sdwa %0, 3, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
                 : "=&v"(r1) : "v"(x));
    asm volatile("v_mov_b32 %0, -1\n\ts_nop 1\n\tv_lshlrev_b16_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
                 : "=&v"(r2) : "v"(x));
    if (threadIdx.x == 0) {
        out[0] = r0;
        out[1] = r1;
        out[2] = r2;
    }
}

#define ITERS 2048
#define CH(INS, D, S) asm volatile(INS : "+v"(D) : "v"(S))
#define KERNEL(NAME, INS)                                                                     \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed) {               \
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                       \
        for (int it = 0; it < ITERS; ++it) {                                                  \
            CH(INS, a0, a1); CH(INS, a1, a2); CH(INS, a2, a3); CH(INS, a3, a4);               \
            CH(INS, a4, a5); CH(INS, a5, a6); CH(INS, a6, a7); CH(INS, a7, a0);               \
        }                                                                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;   \
    }
KERNEL(k_lshl32, "v_lshlrev_b32 %0, 3, %1")
KERNEL(k_lshl16, "v_lshlrev_b16 %0, 3, %1")
KERNEL(k_lshl16_sdwa, "v_lshlrev_b16_sdwa %0, 3, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1")
KERNEL(k_lshl32_sdwa, "v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1")
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %1, 3, %0")
KERNEL(k_mul24, "v_mul_u32_u24 %0, 8, %1")
KERNEL(k_add32, "v_add_u32 %0, %0, %1")

int main() {
    unsigned* out;
    hipMalloc(&out, sizeof(unsigned) * 256 * 8 * 256);
    unsigned h[3];
    hipLaunchKernelGGL(k_sem, dim3(1), dim3(64), 0, 0, out, 0x12345678u);
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    printf("v_lshlrev_b16 (dst preset ~0, x=0x12345678): %08x\n", h[0]);
    printf("v_lshlrev_b16_sdwa WORD_0 UNUSED_PAD byte1:   %08x\n", h[1]);
    printf("v_lshlrev_b16_sdwa DWORD UNUSED_PAD byte1:    %08x\n", h[2]);
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const double clk = prop.clockRate * 1e3;
    struct K { const char* name; void (*fn)(unsigned*, unsigned); } ks[] = {
        {"v_lshlrev_b32", k_lshl32}, {"v_lshlrev_b16", k_lshl16}, {"v_lshlrev_b16_sdwa", k_lshl16_sdwa},
        {"v_lshlrev_b32_sdwa", k_lshl32_sdwa}, {"v_lshl_add_u32", k_lshl_add}, {"v_mul_u32_u24", k_mul24},
        {"v_add_u32", k_add32}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 8, threads = 256;
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, out, 1u);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, out, 1u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double wi = 5.0 * blocks * (threads / 64.0) * ITERS * 8;
        const double per = wi / (ms * 1e-3) / prop.multiProcessorCount / clk;
        printf("%-22s %7.3f ms  %.2f cycles per wave-instr per SIMD\n", k.name, ms, 4.0 / per);
    }
    return 0;
}
