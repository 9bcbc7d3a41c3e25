// ans_launch.hpp — the per-symbol-width launchers of the bulk kernels (ans_launch_impl.hpp),
// explicitly instantiated for u8 / u16 / u32 symbols in ans_launch_{enc,dec}_u*.hip so the
// kernel instantiations compile in parallel translation units; called by ans_kernels.hip.
#pragma once

#include "ans_ctx.hpp"

namespace shuffle_coding {
namespace launch {

template <typename Sym>
int launch_encode(ans_gpu_table* gt, const void* d_syms, uint64_t n, uint64_t chunk_len, uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens, uint32_t* d_status, hipStream_t s, fast::ChunkInit ini = {});
template <typename Sym>
int launch_decode(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap, const uint32_t* d_lens, uint64_t n, uint64_t chunk_len, int gen_kind, void* d_syms, uint32_t* d_status, hipStream_t s, fast::ChunkInit ini = {});
template <typename Sym>
int launch_gen(ans_gpu_table* gt, uint64_t seed, uint64_t start, uint64_t n, void* d_syms, hipStream_t s);
template <typename Sym>
int launch_encode_var(ans_gpu_table* gt, const void* d_syms, uint64_t nchunks, const uint64_t* d_starts, uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens, uint32_t* d_status, hipStream_t s, fast::ChunkInit ini = {}, uint64_t lmax = 0);
template <typename Sym>
int launch_decode_var(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap, const uint32_t* d_lens, uint64_t nchunks, const uint64_t* d_starts, int gen_kind, void* d_syms, uint32_t* d_status, hipStream_t s, fast::ChunkInit ini = {}, uint64_t lmax = 0);
template <typename Sym>
int launch_sample(ans_gpu_table* gt, uint64_t seed, uint64_t n, uint64_t chunk_len, void* d_syms, hipStream_t s);

}  // namespace launch
}  // namespace shuffle_coding
