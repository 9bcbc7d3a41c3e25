// tools/microbench.hip — issue-rate microbenchmark of the VALU instructions the rANS
// inner loops are built from (64-bit integer multiply, FP64, 64-bit shifts/compares).
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench.hip -o tools/microbench
// Prints wave-instructions per cycle per CU for 8 independent chains per lane.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define ITERS 2048

#define KERNEL(NAME, DECL, INIT, BODY, SINK)                                       \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed) {     \
        DECL;                                                                       \
        INIT;                                                                       \
        for (int it = 0; it < ITERS; ++it) {                                        \
            BODY;                                                                   \
        }                                                                           \
        SINK;                                                                       \
    }

// 32-bit ops: 8 chains a0..a7
#define DECL32 unsigned a0, a1, a2, a3, a4, a5, a6, a7
#define INIT32                                                                         \
    a0 = threadIdx.x ^ seed; a1 = a0 + 1; a2 = a0 + 2; a3 = a0 + 3; a4 = a0 + 4;       \
    a5 = a0 + 5; a6 = a0 + 6; a7 = a0 + 7
#define SINK32 out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7
#define OP32(INS)                                                                        \
    asm volatile(INS " %0, %0, %1" : "+v"(a0) : "v"(a1));                                \
    asm volatile(INS " %0, %0, %1" : "+v"(a1) : "v"(a2));                                \
    asm volatile(INS " %0, %0, %1" : "+v"(a2) : "v"(a3));                                \
    asm volatile(INS " %0, %0, %1" : "+v"(a3) : "v"(a4));                                \
    asm volatile(INS " %0, %0, %1" : "+v"(a4) : "v"(a5));                                \
    asm volatile(INS " %0, %0, %1" : "+v"(a5) : "v"(a6));                                \
    asm volatile(INS " %0, %0, %1" : "+v"(a6) : "v"(a7));                                \
    asm volatile(INS " %0, %0, %1" : "+v"(a7) : "v"(a0))

KERNEL(k_add_u32, DECL32, INIT32, OP32("v_add_u32"), SINK32)
KERNEL(k_mul_lo_u32, DECL32, INIT32, OP32("v_mul_lo_u32"), SINK32)
KERNEL(k_mul_hi_u32, DECL32, INIT32, OP32("v_mul_hi_u32"), SINK32)
KERNEL(k_mul_u32_u24, DECL32, INIT32, OP32("v_mul_u32_u24"), SINK32)
KERNEL(k_mul_hi_u32_u24, DECL32, INIT32, OP32("v_mul_hi_u32_u24"), SINK32)
KERNEL(k_xor_b32, DECL32, INIT32, OP32("v_xor_b32"), SINK32)

// 64-bit ops on pairs
#define DECL64 unsigned long long b0, b1, b2, b3, b4, b5, b6, b7
#define INIT64                                                                          \
    b0 = (threadIdx.x ^ seed) * 0x9E3779B97F4A7C15ull; b1 = b0 + 1; b2 = b0 + 2;        \
    b3 = b0 + 3; b4 = b0 + 4; b5 = b0 + 5; b6 = b0 + 6; b7 = b0 + 7
#define SINK64 out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7)
#define MAD64(D, S)                                                                       \
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(D) : "v"((unsigned)S), "v"((unsigned)(S >> 32)) : "vcc")
#define OPMAD MAD64(b0, b1); MAD64(b1, b2); MAD64(b2, b3); MAD64(b3, b4); MAD64(b4, b5); MAD64(b5, b6); MAD64(b6, b7); MAD64(b7, b0)
KERNEL(k_mad_u64_u32, DECL64, INIT64, OPMAD, SINK64)

#define SH64(D, S) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(D) : "v"((unsigned)S))
#define OPSH SH64(b0, b1); SH64(b1, b2); SH64(b2, b3); SH64(b3, b4); SH64(b4, b5); SH64(b5, b6); SH64(b6, b7); SH64(b7, b0)
KERNEL(k_lshrrev_b64, DECL64, INIT64, OPSH, SINK64)

#define LA64(D, S) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(D) : "v"(S))
#define OPLA LA64(b0, b1); LA64(b1, b2); LA64(b2, b3); LA64(b3, b4); LA64(b4, b5); LA64(b5, b6); LA64(b6, b7); LA64(b7, b0)
KERNEL(k_lshl_add_u64, DECL64, INIT64, OPLA, SINK64)

#define DECLF double d0, d1, d2, d3, d4, d5, d6, d7
#define INITF                                                                              \
    d0 = (threadIdx.x ^ seed) * 1e-3; d1 = d0 + 1; d2 = d0 + 2; d3 = d0 + 3; d4 = d0 + 4; \
    d5 = d0 + 5; d6 = d0 + 6; d7 = d0 + 7
#define SINKF out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7)
#define FMA64(D, S) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(D) : "v"(S))
#define OPFMA FMA64(d0, d1); FMA64(d1, d2); FMA64(d2, d3); FMA64(d3, d4); FMA64(d4, d5); FMA64(d5, d6); FMA64(d6, d7); FMA64(d7, d0)
KERNEL(k_fma_f64, DECLF, INITF, OPFMA, SINKF)

#define CVT(D, S) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(D) : "v"((unsigned)__double_as_longlong(S)))
#define OPCVT CVT(d0, d1); CVT(d1, d2); CVT(d2, d3); CVT(d3, d4); CVT(d4, d5); CVT(d5, d6); CVT(d6, d7); CVT(d7, d0)
KERNEL(k_cvt_f64_u32, DECLF, INITF, OPCVT, SINKF)

#define DECLS float f0, f1, f2, f3, f4, f5, f6, f7
#define INITS                                                                              \
    f0 = (threadIdx.x ^ seed) * 1e-3f; f1 = f0 + 1; f2 = f0 + 2; f3 = f0 + 3; f4 = f0 + 4; \
    f5 = f0 + 5; f6 = f0 + 6; f7 = f0 + 7
#define SINKS out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7)
#define FMA32(D, S) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(D) : "v"(S))
#define OPFMA32 FMA32(f0, f1); FMA32(f1, f2); FMA32(f2, f3); FMA32(f3, f4); FMA32(f4, f5); FMA32(f5, f6); FMA32(f6, f7); FMA32(f7, f0)
KERNEL(k_fma_f32, DECLS, INITS, OPFMA32, SINKS)

#define CMP64(D, S) asm volatile("v_cmp_ge_u64 vcc, %0, %1\n\tv_cndmask_b32 %2, %2, 0, vcc" : "+v"(D) : "v"(S), "v"(a0) : "vcc")
KERNEL(k_cmp_u64_cnd, DECL64; unsigned a0 = threadIdx.x, INIT64,
       CMP64(b0, b1); CMP64(b1, b2); CMP64(b2, b3); CMP64(b3, b4); CMP64(b4, b5); CMP64(b5, b6); CMP64(b6, b7); CMP64(b7, b0),
       SINK64 + a0)


#define OP3(INS)                                                                        \
    asm volatile(INS " %0, %0, %1, %2" : "+v"(a0) : "v"(a1), "v"(a2));                   \
    asm volatile(INS " %0, %0, %1, %2" : "+v"(a1) : "v"(a2), "v"(a3));                   \
    asm volatile(INS " %0, %0, %1, %2" : "+v"(a2) : "v"(a3), "v"(a4));                   \
    asm volatile(INS " %0, %0, %1, %2" : "+v"(a3) : "v"(a4), "v"(a5));                   \
    asm volatile(INS " %0, %0, %1, %2" : "+v"(a4) : "v"(a5), "v"(a6));                   \
    asm volatile(INS " %0, %0, %1, %2" : "+v"(a5) : "v"(a6), "v"(a7));                   \
    asm volatile(INS " %0, %0, %1, %2" : "+v"(a6) : "v"(a7), "v"(a0));                   \
    asm volatile(INS " %0, %0, %1, %2" : "+v"(a7) : "v"(a0), "v"(a1))
#define OP1(INS)                                                                        \
    asm volatile(INS " %0, %1" : "=v"(a0) : "v"(a1));                                    \
    asm volatile(INS " %0, %1" : "=v"(a1) : "v"(a2));                                    \
    asm volatile(INS " %0, %1" : "=v"(a2) : "v"(a3));                                    \
    asm volatile(INS " %0, %1" : "=v"(a3) : "v"(a4));                                    \
    asm volatile(INS " %0, %1" : "=v"(a4) : "v"(a5));                                    \
    asm volatile(INS " %0, %1" : "=v"(a5) : "v"(a6));                                    \
    asm volatile(INS " %0, %1" : "=v"(a6) : "v"(a7));                                    \
    asm volatile(INS " %0, %1" : "=v"(a7) : "v"(a0))
#define CMP32(D, S) asm volatile("v_cmp_ge_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(D) : "v"(S) : "vcc")
#define OPCMP32 CMP32(a0, a1); CMP32(a1, a2); CMP32(a2, a3); CMP32(a3, a4); CMP32(a4, a5); CMP32(a5, a6); CMP32(a6, a7); CMP32(a7, a0)
#define MULF(D, S) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(D) : "v"(S))
#define OPMULF MULF(d0, d1); MULF(d1, d2); MULF(d2, d3); MULF(d3, d4); MULF(d4, d5); MULF(d5, d6); MULF(d6, d7); MULF(d7, d0)
#define ADDF(D, S) asm volatile("v_add_f64 %0, %0, %1" : "+v"(D) : "v"(S))
#define OPADDF ADDF(d0, d1); ADDF(d1, d2); ADDF(d2, d3); ADDF(d3, d4); ADDF(d4, d5); ADDF(d5, d6); ADDF(d6, d7); ADDF(d7, d0)
typedef float f2v __attribute__((ext_vector_type(2)));
#define DECLP f2v p0, p1, p2, p3, p4, p5, p6, p7
#define INITP p0 = f2v{(float)threadIdx.x, 1.f}; p1 = p0 + 1; p2 = p0 + 2; p3 = p0 + 3; p4 = p0 + 4; p5 = p0 + 5; p6 = p0 + 6; p7 = p0 + 7
#define SINKP out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7).x
#define PK(D, S) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(D) : "v"(S))
#define OPPK PK(p0, p1); PK(p1, p2); PK(p2, p3); PK(p3, p4); PK(p4, p5); PK(p5, p6); PK(p6, p7); PK(p7, p0)

KERNEL(k_alignbyte, DECL32, INIT32, OP3("v_alignbyte_b32"), SINK32)
KERNEL(k_perm_b32, DECL32, INIT32, OP3("v_perm_b32"), SINK32)
KERNEL(k_add3_u32, DECL32, INIT32, OP3("v_add3_u32"), SINK32)
KERNEL(k_lshl_or_b32, DECL32, INIT32, OP3("v_lshl_or_b32"), SINK32)
KERNEL(k_bfe_u32, DECL32, INIT32, OP3("v_bfe_u32"), SINK32)
KERNEL(k_mad_u32_u24, DECL32, INIT32, OP3("v_mad_u32_u24"), SINK32)
KERNEL(k_ffbh_u32, DECL32, INIT32, OP1("v_ffbh_u32"), SINK32)
KERNEL(k_cvt_f32_u32, DECL32, INIT32, OP1("v_cvt_f32_u32"), SINK32)
KERNEL(k_cvt_u32_f32, DECL32, INIT32, OP1("v_cvt_u32_f32"), SINK32)
KERNEL(k_rcp_f32, DECL32, INIT32, OP1("v_rcp_f32"), SINK32)
KERNEL(k_mul_f32, DECL32, INIT32, OP32("v_mul_f32"), SINK32)
KERNEL(k_min_u32, DECL32, INIT32, OP32("v_min_u32"), SINK32)
KERNEL(k_lshrrev_b32, DECL32, INIT32, OP32("v_lshrrev_b32"), SINK32)
KERNEL(k_cmp_u32_cnd, DECL32, INIT32, OPCMP32, SINK32)
KERNEL(k_mul_f64, DECLF, INITF, OPMULF, SINKF)
KERNEL(k_add_f64, DECLF, INITF, OPADDF, SINKF)
KERNEL(k_pk_fma_f32, DECLP, INITP, OPPK, SINKP)

#define CND(D, S) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(D) : "v"(S))
#define OPCND asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(a0), "v"(a1) : "vcc"); CND(a0, a1); CND(a1, a2); CND(a2, a3); CND(a3, a4); CND(a4, a5); CND(a5, a6); CND(a6, a7); CND(a7, a0)
#define CND64(D, S) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[10:11]" : "+v"(D) : "v"(S))
#define OPCND64 asm volatile("v_cmp_gt_u32_e64 s[10:11], %0, %1" :: "v"(a0), "v"(a1) : "s10", "s11"); CND64(a0, a1); CND64(a1, a2); CND64(a2, a3); CND64(a3, a4); CND64(a4, a5); CND64(a5, a6); CND64(a6, a7); CND64(a7, a0)
#define CMPO(D, S) asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(D), "v"(S) : "vcc")
#define OPCMPONLY CMPO(a0, a1); CMPO(a1, a2); CMPO(a2, a3); CMPO(a3, a4); CMPO(a4, a5); CMPO(a5, a6); CMPO(a6, a7); CMPO(a7, a0); asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a0) : "v"(a1))
#define ADDCO(D, S) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(D) : "v"(S) : "vcc")
#define OPADDCO ADDCO(a0, a1); ADDCO(a1, a2); ADDCO(a2, a3); ADDCO(a3, a4); ADDCO(a4, a5); ADDCO(a5, a6); ADDCO(a6, a7); ADDCO(a7, a0)
#define ADDC(D, S) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(D) : "v"(S) : "vcc")
#define OPADDC ADDC(a0, a1); ADDC(a1, a2); ADDC(a2, a3); ADDC(a3, a4); ADDC(a4, a5); ADDC(a5, a6); ADDC(a6, a7); ADDC(a7, a0)
#define FMADEP(D) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(D))
#define OPFMA32DEP FMADEP(f0); FMADEP(f0); FMADEP(f0); FMADEP(f0); FMADEP(f0); FMADEP(f0); FMADEP(f0); FMADEP(f0)
#define ADDDEP(D) asm volatile("v_add_u32 %0, %0, %0" : "+v"(D))
#define OPADDDEP ADDDEP(a0); ADDDEP(a0); ADDDEP(a0); ADDDEP(a0); ADDDEP(a0); ADDDEP(a0); ADDDEP(a0); ADDDEP(a0)
#define MADDEP(D) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(D) : "v"((unsigned)D) : "vcc")
#define OPMADDEP MADDEP(b0); MADDEP(b0); MADDEP(b0); MADDEP(b0); MADDEP(b0); MADDEP(b0); MADDEP(b0); MADDEP(b0)
#define FMAFDEP(D) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(D))
#define OPFMAFDEP FMAFDEP(d0); FMAFDEP(d0); FMAFDEP(d0); FMAFDEP(d0); FMAFDEP(d0); FMAFDEP(d0); FMAFDEP(d0); FMAFDEP(d0)
#define PERMDEP(D) asm volatile("v_perm_b32 %0, %0, %0, %0" : "+v"(D))
#define OPPERMDEP PERMDEP(a0); PERMDEP(a0); PERMDEP(a0); PERMDEP(a0); PERMDEP(a0); PERMDEP(a0); PERMDEP(a0); PERMDEP(a0)

KERNEL(k_sub_u32, DECL32, INIT32, OP32("v_sub_u32"), SINK32)
KERNEL(k_and_b32, DECL32, INIT32, OP32("v_and_b32"), SINK32)
KERNEL(k_or_b32, DECL32, INIT32, OP32("v_or_b32"), SINK32)
KERNEL(k_lshlrev_b32, DECL32, INIT32, OP32("v_lshlrev_b32"), SINK32)
KERNEL(k_ashrrev_i32, DECL32, INIT32, OP32("v_ashrrev_i32"), SINK32)
KERNEL(k_max_u32, DECL32, INIT32, OP32("v_max_u32"), SINK32)
KERNEL(k_add_f32, DECL32, INIT32, OP32("v_add_f32"), SINK32)
KERNEL(k_cndmask_e32, DECL32, INIT32, OPCND, SINK32)
KERNEL(k_cndmask_e64, DECL32, INIT32, OPCND64, SINK32)
KERNEL(k_cmp_e32, DECL32, INIT32, OPCMPONLY, SINK32)
KERNEL(k_add_co, DECL32, INIT32, OPADDCO, SINK32)
KERNEL(k_addc_co, DECL32, INIT32, OPADDC, SINK32)
KERNEL(k_sub_f32_e64, DECL32, INIT32, OP32("v_sub_f32_e64"), SINK32)
KERNEL(k_add_u32_e64, DECL32, INIT32, OP32("v_add_u32_e64"), SINK32)
KERNEL(k_and_or_b32, DECL32, INIT32, OP3("v_and_or_b32"), SINK32)
KERNEL(k_or3_b32, DECL32, INIT32, OP3("v_or3_b32"), SINK32)
KERNEL(k_bfi_b32, DECL32, INIT32, OP3("v_bfi_b32"), SINK32)
KERNEL(k_lshl_add_u32, DECL32, INIT32, OP3("v_lshl_add_u32"), SINK32)
KERNEL(k_fma_f32_dep, DECLS, INITS, OPFMA32DEP, SINKS)
KERNEL(k_add_u32_dep, DECL32, INIT32, OPADDDEP, SINK32)
KERNEL(k_mad64_dep, DECL64, INIT64, OPMADDEP, SINK64)
KERNEL(k_fma_f64_dep, DECLF, INITF, OPFMAFDEP, SINKF)
KERNEL(k_perm_dep, DECL32, INIT32, OPPERMDEP, SINK32)

#define RCPF(D, S) asm volatile("v_rcp_f64 %0, %1" : "=v"(D) : "v"(S))
#define OPRCPF RCPF(d0, d1); RCPF(d1, d2); RCPF(d2, d3); RCPF(d3, d4); RCPF(d4, d5); RCPF(d5, d6); RCPF(d6, d7); RCPF(d7, d0)
KERNEL(k_rcp_f64, DECLF, INITF, OPRCPF, SINKF)
#define FRX(D, S) asm volatile("v_frexp_exp_i32_f64 %0, %1" : "=v"(D) : "v"(S))
KERNEL(k_frexp, DECLF; unsigned e0 = 0, INITF, FRX(e0, d1); FRX(e0, d2); FRX(e0, d3); FRX(e0, d4); FRX(e0, d5); FRX(e0, d6); FRX(e0, d7); FRX(e0, d0), SINKF + e0)
#define SUBB(D, S) asm volatile("v_sub_co_u32 %0, vcc, %0, %1" : "+v"(D) : "v"(S) : "vcc")
KERNEL(k_sub_co, DECL32, INIT32, SUBB(a0, a1); SUBB(a1, a2); SUBB(a2, a3); SUBB(a3, a4); SUBB(a4, a5); SUBB(a5, a6); SUBB(a6, a7); SUBB(a7, a0), SINK32)
KERNEL(k_mul_u32_u24_dep, DECL32, INIT32, OP32("v_mul_u32_u24"), SINK32)
KERNEL(k_lshlrev_b16, DECL32, INIT32, OP32("v_lshlrev_b16"), SINK32)
KERNEL(k_add_u16, DECL32, INIT32, OP32("v_add_u16"), SINK32)
KERNEL(k_cvt_f64_i32, DECLF, INITF, OPCVT, SINKF)
#define CVTF(D, S) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(D) : "v"(S))
KERNEL(k_cvt_f32_f64, DECLF; float g0 = 0, INITF, CVTF(g0, d1); CVTF(g0, d2); CVTF(g0, d3); CVTF(g0, d4); CVTF(g0, d5); CVTF(g0, d6); CVTF(g0, d7); CVTF(g0, d0), SINKF + (unsigned)g0)

int main(int argc, char** argv) {
    const int blocks = 256 * (argc > 1 ? atoi(argv[1]) : 8), threads = 256;
    unsigned* out;
    hipMalloc(&out, sizeof(unsigned) * blocks * threads);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const double clk_hz = prop.clockRate * 1e3;  // kHz -> Hz (max clock)
    struct K { const char* name; void (*fn)(unsigned*, unsigned); int instr_per_op; };
    K ks[] = {
        {"v_add_u32", k_add_u32, 1},        {"v_xor_b32", k_xor_b32, 1},
        {"v_mul_lo_u32", k_mul_lo_u32, 1},  {"v_mul_hi_u32", k_mul_hi_u32, 1},
        {"v_mul_u32_u24", k_mul_u32_u24, 1}, {"v_mul_hi_u32_u24", k_mul_hi_u32_u24, 1},
        {"v_mad_u64_u32", k_mad_u64_u32, 1}, {"v_lshrrev_b64", k_lshrrev_b64, 1},
        {"v_lshl_add_u64", k_lshl_add_u64, 1}, {"v_fma_f64", k_fma_f64, 1},
        {"v_cvt_f64_u32", k_cvt_f64_u32, 1}, {"v_fma_f32", k_fma_f32, 1},
        {"v_cmp_ge_u64+v_cndmask", k_cmp_u64_cnd, 2},
        {"v_alignbyte_b32", k_alignbyte, 1}, {"v_perm_b32", k_perm_b32, 1}, {"v_add3_u32", k_add3_u32, 1},
        {"v_lshl_or_b32", k_lshl_or_b32, 1}, {"v_bfe_u32", k_bfe_u32, 1}, {"v_mad_u32_u24", k_mad_u32_u24, 1},
        {"v_ffbh_u32", k_ffbh_u32, 1}, {"v_cvt_f32_u32", k_cvt_f32_u32, 1}, {"v_cvt_u32_f32", k_cvt_u32_f32, 1},
        {"v_rcp_f32", k_rcp_f32, 1}, {"v_mul_f32", k_mul_f32, 1}, {"v_min_u32", k_min_u32, 1},
        {"v_lshrrev_b32", k_lshrrev_b32, 1}, {"v_cmp_ge_u32+v_cndmask", k_cmp_u32_cnd, 2},
        {"v_mul_f64", k_mul_f64, 1}, {"v_add_f64", k_add_f64, 1}, {"v_pk_fma_f32", k_pk_fma_f32, 1},
        {"v_sub_u32", k_sub_u32, 1}, {"v_and_b32", k_and_b32, 1}, {"v_or_b32", k_or_b32, 1},
        {"v_lshlrev_b32", k_lshlrev_b32, 1}, {"v_ashrrev_i32", k_ashrrev_i32, 1}, {"v_max_u32", k_max_u32, 1},
        {"v_add_f32", k_add_f32, 1}, {"v_cndmask_e32", k_cndmask_e32, 1}, {"v_cndmask_e64", k_cndmask_e64, 1},
        {"v_cmp_gt_u32_e32", k_cmp_e32, 1}, {"v_add_co_u32", k_add_co, 1}, {"v_addc_co_u32", k_addc_co, 1},
        {"v_sub_f32_e64", k_sub_f32_e64, 1}, {"v_add_u32_e64", k_add_u32_e64, 1}, {"v_and_or_b32", k_and_or_b32, 1},
        {"v_or3_b32", k_or3_b32, 1}, {"v_bfi_b32", k_bfi_b32, 1}, {"v_lshl_add_u32", k_lshl_add_u32, 1},
        {"DEP v_fma_f32", k_fma_f32_dep, 1}, {"DEP v_add_u32", k_add_u32_dep, 1}, {"DEP v_mad_u64_u32", k_mad64_dep, 1},
        {"DEP v_fma_f64", k_fma_f64_dep, 1}, {"DEP v_perm_b32", k_perm_dep, 1},
        {"v_rcp_f64", k_rcp_f64, 1}, {"v_frexp_exp_i32_f64", k_frexp, 1}, {"v_sub_co_u32", k_sub_co, 1},
        {"v_lshlrev_b16", k_lshlrev_b16, 1}, {"v_add_u16", k_add_u16, 1}, {"v_cvt_f32_f64", k_cvt_f32_f64, 1},
    };
    printf("clock(max) %.0f MHz, CUs %d\n", clk_hz / 1e6, prop.multiProcessorCount);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, out, 1u);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, out, 1u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double wave_instr = 5.0 * blocks * (threads / 64.0) * ITERS * 8 * k.instr_per_op;
        const double per_cu_per_clk = wave_instr / (ms * 1e-3) / prop.multiProcessorCount / clk_hz;
        printf("%-24s %8.3f ms  %6.3f wave-instr/clk/CU  (%.2f cycles per wave-instr per SIMD)\n", k.name, ms,
               per_cu_per_clk, 4.0 / per_cu_per_clk);
    }
    return 0;
}
