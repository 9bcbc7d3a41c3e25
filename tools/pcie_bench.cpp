// Host-memory (PCIe-inclusive) rate of the bulk path through the C ABI alone, as a C/Rust
// caller sees it (no torch in the process): C3 symbols in host memory,
// ans_gpu_encode_chunks into a host container, ans_gpu_decode_chunks back into host memory.
// Page-locked buffers (ans_host_alloc) and pageable ones (malloc).  Prints one JSON line.
// usage: pcie_bench [log2n=30] [reps=3] [batch_mib=0 (library default)]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/ans_capi.h"

#define CK(x) do { int rc_ = (x); if (rc_) { fprintf(stderr, "%s -> %d\n", #x, rc_); exit(1); } } while (0)

static double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Rate { double enc, dec; };

static Rate run(ans_gpu_table* gt, const uint8_t* syms, uint64_t n, uint64_t L, uint8_t* out, uint64_t cap, uint8_t* back,
                int reps) {
    const uint64_t nch = (n + L - 1) / L;
    std::vector<uint64_t> offs(nch), lens(nch);
    double te = 1e30, td = 1e30;
    for (int r = 0; r < reps; ++r) {
        uint64_t total = 0;
        double t0 = now_s();
        CK(ans_gpu_encode_chunks(gt, syms, 1, n, L, out, cap, offs.data(), lens.data(), &total));
        double t1 = now_s();
        CK(ans_gpu_decode_chunks(gt, out, total, offs.data(), lens.data(), n, L, ANS_GEN_ZEROS, back, 1));
        double t2 = now_s();
        te = std::min(te, t1 - t0);
        td = std::min(td, t2 - t1);
    }
    if (memcmp(back, syms, n)) { fprintf(stderr, "round trip mismatch\n"); exit(1); }
    return {n / te / (1u << 30), n / td / (1u << 30)};
}

int main(int argc, char** argv) {
    const int log2n = argc > 1 ? atoi(argv[1]) : 30;
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    const uint64_t batch_mib = argc > 3 ? strtoull(argv[3], nullptr, 10) : 0;
    const uint64_t n = 1ull << log2n, L = 4096;
    std::vector<uint64_t> masses(256);
    for (uint64_t s = 0; s < 256; ++s) masses[s] = 1 + (splitmix64(0x5EEDull ^ s) & ((1ull << 20) - 1));
    ans_table* t = nullptr;
    CK(ans_table_create(masses.data(), 256, &t));
    ans_gpu* g = nullptr;
    CK(ans_gpu_create(0, &g));
    CK(ans_gpu_set_batch_bytes(g, batch_mib << 20));
    ans_gpu_table* gt = nullptr;
    CK(ans_gpu_table_create(g, t, &gt));
    uint64_t slot = 0;
    CK(ans_gpu_slot_capacity(gt, L, &slot));
    const uint64_t cap = (n / L) * slot;
    void* d = nullptr;
    if (hipMalloc(&d, n) != hipSuccess) return 1;
    CK(ans_dev_gen_iid(gt, 1, 0, n, d, 1, nullptr));
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    // page-locked
    uint8_t *ps, *po, *pb;
    CK(ans_host_alloc(n, reinterpret_cast<void**>(&ps)));
    CK(ans_host_alloc(cap, reinterpret_cast<void**>(&po)));
    CK(ans_host_alloc(n, reinterpret_cast<void**>(&pb)));
    if (hipMemcpy(ps, d, n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    memset(po, 0, cap);
    memset(pb, 0, n);
    const Rate pin = run(gt, ps, n, L, po, cap, pb, reps);
    // pageable
    auto* qs = static_cast<uint8_t*>(malloc(n));
    auto* qo = static_cast<uint8_t*>(malloc(cap));
    auto* qb = static_cast<uint8_t*>(malloc(n));
    memcpy(qs, ps, n);
    memset(qo, 0, cap);
    memset(qb, 0, n);
    const Rate pag = run(gt, qs, n, L, qo, cap, qb, reps);
    printf("{\"workload\": \"C3 2^%d u8 symbols, chunk %lu\", \"caller\": \"C ABI only (tools/pcie_bench.cpp)\", "
           "\"reps\": %d, \"batch_mib\": %lu, "
           "\"pinned\": {\"encode_gib_s\": %.2f, \"decode_gib_s\": %.2f, \"round_trip_gib_s\": %.2f}, "
           "\"pageable\": {\"encode_gib_s\": %.2f, \"decode_gib_s\": %.2f, \"round_trip_gib_s\": %.2f}}\n",
           log2n, (unsigned long)L, reps, (unsigned long)(batch_mib ? batch_mib : 256), pin.enc, pin.dec,
           1.0 / (1.0 / pin.enc + 1.0 / pin.dec), pag.enc, pag.dec, 1.0 / (1.0 / pag.enc + 1.0 / pag.dec));
    ans_host_free(ps);
    ans_host_free(po);
    ans_host_free(pb);
    free(qs);
    free(qo);
    free(qb);
    (void)hipFree(d);
    ans_gpu_table_free(gt);
    ans_gpu_free(g);
    ans_table_free(t);
    return 0;
}
