// ans_launch_dec_u32.hip — decode-side launchers for u32 symbols (ans_launch_impl.hpp): one of six units
// that compile the kernel instantiations in parallel.
#include "ans_launch_impl.hpp"

namespace shuffle_coding {
namespace launch {

template int launch_decode<uint32_t>(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap, const uint32_t* d_lens, uint64_t n, uint64_t chunk_len, int gen_kind, void* d_syms, uint32_t* d_status, hipStream_t s, fast::ChunkInit ini);
template int launch_decode_var<uint32_t>(ans_gpu_table* gt, const uint8_t* d_in, const uint64_t* d_offsets, uint64_t slot_cap, const uint32_t* d_lens, uint64_t nchunks, const uint64_t* d_starts, int gen_kind, void* d_syms, uint32_t* d_status, hipStream_t s, fast::ChunkInit ini, uint64_t lmax);

}  // namespace launch
}  // namespace shuffle_coding
