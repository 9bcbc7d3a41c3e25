// Host-side cost of hipMemcpyAsync per 16 MiB batch, by host buffer kind (hipHostMalloc with
// default / coherent / non-coherent flags, hipHostRegister'ed malloc, plain pageable malloc),
// H2D and D2H on two streams at once.  Prints per-call enqueue time and overall GB/s.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

__global__ void k_copy(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

static void run_kernel(const char* name, unsigned char* hin, unsigned char* hout, size_t total, size_t batch, void* din,
                       void* dout, hipStream_t s1, hipStream_t s2, int grid) {
    CK(hipDeviceSynchronize());
    const double t0 = now();
    for (size_t off = 0; off < total; off += batch) {
        k_copy<<<grid, 256, 0, s1>>>(reinterpret_cast<uint4*>(static_cast<char*>(din) + off), reinterpret_cast<const uint4*>(hin + off), batch / 16);
        k_copy<<<grid, 256, 0, s2>>>(reinterpret_cast<uint4*>(hout + off), reinterpret_cast<const uint4*>(static_cast<char*>(dout) + off), batch / 16);
    }
    CK(hipStreamSynchronize(s1));
    CK(hipStreamSynchronize(s2));
    const double t = now() - t0;
    printf("%-28s grid %4d: total %.2f ms = %.1f GB/s each way\n", name, grid, t, total / t / 1e6);
    CK(hipDeviceSynchronize());
    double t1 = now();
    for (size_t off = 0; off < total; off += batch)
        k_copy<<<grid, 256, 0, s1>>>(reinterpret_cast<uint4*>(static_cast<char*>(din) + off), reinterpret_cast<const uint4*>(hin + off), batch / 16);
    CK(hipStreamSynchronize(s1));
    double t2 = now();
    for (size_t off = 0; off < total; off += batch)
        k_copy<<<grid, 256, 0, s2>>>(reinterpret_cast<uint4*>(hout + off), reinterpret_cast<const uint4*>(static_cast<char*>(dout) + off), batch / 16);
    CK(hipStreamSynchronize(s2));
    double t3 = now();
    printf("%-28s grid %4d: h2d alone %.1f GB/s, d2h alone %.1f GB/s\n", name, grid, total / (t2 - t1) / 1e6, total / (t3 - t2) / 1e6);
}

static void run(const char* name, unsigned char* hin, unsigned char* hout, size_t total, size_t batch, void* din, void* dout,
                hipStream_t s1, hipStream_t s2) {
    double worst = 0, sum = 0;
    CK(hipDeviceSynchronize());
    const double t0 = now();
    for (size_t off = 0; off < total; off += batch) {
        const double a = now();
        CK(hipMemcpyAsync(static_cast<char*>(din) + off, hin + off, batch, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(hout + off, static_cast<char*>(dout) + off, batch, hipMemcpyDeviceToHost, s2));
        const double d = now() - a;
        sum += d;
        if (d > worst) worst = d;
    }
    CK(hipStreamSynchronize(s1));
    CK(hipStreamSynchronize(s2));
    const double t = now() - t0;
    printf("%-28s enqueue avg %.3f ms worst %.3f ms; total %.2f ms = %.1f GB/s each way\n", name, sum / (total / batch), worst,
           t, total / t / 1e6);
}

int main() {
    const size_t total = 1ull << 30, batch = 16ull << 20;
    void *din, *dout;
    CK(hipMalloc(&din, total));
    CK(hipMalloc(&dout, total));
    CK(hipMemset(dout, 1, total));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const unsigned flags[3] = {hipHostMallocDefault, hipHostMallocCoherent, hipHostMallocNonCoherent};
    const char* names[3] = {"hipHostMalloc default", "hipHostMalloc coherent", "hipHostMalloc noncoherent"};
    for (int k = 0; k < 3; ++k) {
        unsigned char *a, *b;
        CK(hipHostMalloc(reinterpret_cast<void**>(&a), total, flags[k]));
        CK(hipHostMalloc(reinterpret_cast<void**>(&b), total, flags[k]));
        memset(a, 3, total);
        memset(b, 0, total);
        for (int r = 0; r < 2; ++r) run(names[k], a, b, total, batch, din, dout, s1, s2);
        for (int grid : {64, 256, 1024}) run_kernel(names[k], a, b, total, batch, din, dout, s1, s2, grid);
        CK(hipHostFree(a));
        CK(hipHostFree(b));
    }
    {
        auto* a = static_cast<unsigned char*>(aligned_alloc(4096, total));
        auto* b = static_cast<unsigned char*>(aligned_alloc(4096, total));
        memset(a, 3, total);
        memset(b, 0, total);
        for (int r = 0; r < 2; ++r) run("pageable malloc", a, b, total, batch, din, dout, s1, s2);
        const double t0 = now();
        CK(hipHostRegister(a, total, hipHostRegisterDefault));
        CK(hipHostRegister(b, total, hipHostRegisterDefault));
        printf("hipHostRegister 2 x 1 GiB: %.1f ms\n", now() - t0);
        for (int r = 0; r < 2; ++r) run("hipHostRegister'ed malloc", a, b, total, batch, din, dout, s1, s2);
        CK(hipHostUnregister(a));
        CK(hipHostUnregister(b));
        free(a);
        free(b);
    }
    return 0;
}
