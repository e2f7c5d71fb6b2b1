// flood_host.hpp -- host-side interfaces between the flood*.hip translation units.
#pragma once
#include <cstddef>
#include <cstdint>

#include "flood_dev.hpp"

namespace ldpc {

constexpr int kStreamMaxDeg = 32;  // register windows of stream_check_kernel / stream_var_kernel
inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }

// flood.hip: fold per-workgroup counter rows (counters_reduce_kernel)
int reduce_counter_rows(const uint32_t *partials, int64_t nwg, uint64_t *counters, int32_t *batch_iters,
                        const int32_t *gate, hipStream_t s);

// flood_fixed_ms.hip / flood_fixed_bp.hip: flood_fixed_kernel<code, ALGO, es> for fixed_id 1 (BG2 Z=4)
// or 2 (BG2 Z=32), es one of LDPC_ES_OFF / LDPC_ES_FRAME / LDPC_ES_BATCH / ES_P1 / ES_P2
int launch_fixed_minsum(int fixed_id, int es, dim3 grid, dim3 block, size_t lds, hipStream_t s, const FloodTables &T,
                        const float *llr, int64_t B, int max_iter, float alpha, int out_dtype, void *bits,
                        const Outs &O, const EsWs &W);
int launch_fixed_bp(int fixed_id, int es, dim3 grid, dim3 block, size_t lds, hipStream_t s, const FloodTables &T,
                    const float *llr, int64_t B, int max_iter, float alpha, int out_dtype, void *bits, const Outs &O,
                    const EsWs &W);

// flood_stream.hip: the streaming decoders (messages in HBM, any graph)
int64_t stream_ws_bytes(const ldpc_graph *g, int64_t B, int max_iter);
int run_stream_decode(int algo, const ldpc_graph *g, const float *llr, int64_t B, int max_iter, float alpha, int es,
                      int out_dtype, void *bits, int32_t *iters_out, uint64_t *counters, int32_t *batch_iters,
                      void *work, hipStream_t s);
int64_t custom_ws_bytes(const ldpc_graph *g, int64_t B);
int run_custom_minsum(const ldpc_graph *g, const float *llr, int64_t B, int iterations, float *probs, void *work,
                      hipStream_t s);

}  // namespace ldpc
