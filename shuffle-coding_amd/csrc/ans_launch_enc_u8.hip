// ans_launch_enc_u8.hip — encode-side launchers for u8 symbols (ans_launch_impl.hpp): one of six units
// that compile the kernel instantiations in parallel.
#include "ans_launch_impl.hpp"

namespace shuffle_coding {
namespace launch {

template int launch_encode<uint8_t>(ans_gpu_table* gt, const void* d_syms, uint64_t n, uint64_t chunk_len, uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens, uint32_t* d_status, hipStream_t s, fast::ChunkInit ini);
template int launch_gen<uint8_t>(ans_gpu_table* gt, uint64_t seed, uint64_t start, uint64_t n, void* d_syms, hipStream_t s);
template int launch_encode_var<uint8_t>(ans_gpu_table* gt, const void* d_syms, uint64_t nchunks, const uint64_t* d_starts, uint8_t* d_slots, uint64_t slot_cap, uint32_t* d_lens, uint32_t* d_status, hipStream_t s, fast::ChunkInit ini, uint64_t lmax);
template int launch_sample<uint8_t>(ans_gpu_table* gt, uint64_t seed, uint64_t n, uint64_t chunk_len, void* d_syms, hipStream_t s);

}  // namespace launch
}  // namespace shuffle_coding
