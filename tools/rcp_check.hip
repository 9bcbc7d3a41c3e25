// tools/rcp_check.hip — accuracy of v_rcp_f64 against the correctly rounded 1.0/d (the fast
// encoder's quotient estimate needs |rcp - 1/d| <= a few ulp): every d in
// [1, 2^24] and 2^26 random d up to 2^32.  Prints the largest error in ulps of 1/d.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_check(unsigned long long base, unsigned long long count, int random, unsigned* worst,
                        unsigned long long* bad) {
    const unsigned long long i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= count) return;
    unsigned long long d = base + i;
    if (random) {
        unsigned long long z = i * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
        z = (z ^ (z >> 31)) * 0xBF58476D1CE4E5B9ull;
        d = 1 + ((z ^ (z >> 29)) & 0xFFFFFFFFull);
    }
    const double dd = static_cast<double>(d);
    double r;
    asm volatile("v_rcp_f64 %0, %1" : "=v"(r) : "v"(dd));
    const double exact = 1.0 / dd;  // IEEE division (correctly rounded)
    const long long diff = __double_as_longlong(r) - __double_as_longlong(exact);
    const unsigned ad = static_cast<unsigned>(diff < 0 ? -diff : diff);
    atomicMax(worst, ad);
    if (ad > 1) atomicAdd(bad, 1ull);
}

int main() {
    unsigned* w;
    unsigned long long* b;
    if (hipMalloc(&w, 4) != hipSuccess || hipMalloc(&b, 8) != hipSuccess) return 1;
    (void)hipMemset(w, 0, 4);
    (void)hipMemset(b, 0, 8);
    const unsigned long long n1 = 1ull << 24;
    k_check<<<(n1 + 255) / 256, 256>>>(1, n1, 0, w, b);
    const unsigned long long n2 = 1ull << 26;
    k_check<<<(n2 + 255) / 256, 256>>>(0, n2, 1, w, b);
    unsigned hw = 0;
    unsigned long long hb = 0;
    (void)hipMemcpy(&hw, w, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&hb, b, 8, hipMemcpyDeviceToHost);
    printf("v_rcp_f64 vs 1.0/d: max |error| = %u ulp; %llu of %llu divisors beyond 1 ulp\n", hw, hb, n1 + n2);
    return 0;
}
