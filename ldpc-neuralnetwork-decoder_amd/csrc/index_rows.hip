// index_rows.hip -- the hybrid layers' public per-message updates on the reference's index rows.
//
// Replaces:
//   CustomCheckMessageGNNLayer.check_layer_update     message_gnn_decoder.py:976-1044
//   CustomVariableMessageGNNLayer.variable_layer_update message_gnn_decoder.py:611-670
// Both walk an index tensor row by row: row m = [node, incoming message ids..., -1 padding].  For
// every listed id i the reference overwrites output m with the update that leaves position i out,
// so output m is the update that excludes the row's LAST valid entry (the loop's last assignment).
//   check:    out[b, m] = prod_{others} sign(x[b, id]) * min_{others} |x[b, id]|
//             torch.sign semantics (sign(+-0) = +0, sign(NaN) = 0), torch.min propagates NaN; the
//             product of the +-1 / 0 signs is exact in any order (its sign is the xor of the
//             factors' sign bits); no valid entry or no other entry -> +0.0.
//   variable: out[b, m] = (llr[b, node] + sum_{valid} c[b, id]) - c[b, last id], the sum ascending
//             (this build's definition of torch's .sum for these rows, as in the hybrid decoders);
//             no valid entry -> llr[b, node]; iteration > 0: 0.5 * out + 0.5 * c[b, m] (:659-663).
//             The reference's total_sum broadcasts (B, 1) + (B,) to (B, B) and only runs at B = 1;
//             this is its per-frame meaning.
// One thread per (row, frame), rows fastest.  Ids are validated on the host (the reference raises
// IndexError); the kernels trust them.
#include <cmath>
#include <cstdint>

#include "common.hpp"

namespace ldpc {
namespace {

__device__ __forceinline__ float torch_sign(float v) { return v > 0.0f ? 1.0f : (v < 0.0f ? -1.0f : 0.0f); }

__global__ __launch_bounds__(256) void index_rows_minsum_kernel(const float *__restrict__ x, int64_t B, int64_t Ein,
                                                                const int64_t *__restrict__ rows, int64_t R, int W,
                                                                float *__restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const int64_t *row = rows + r * W;
    int last = -1, nvalid = 0;
    for (int j = 1; j < W; ++j)
        if (row[j] >= 0) {
            last = j;
            ++nvalid;
        }
    for (int64_t b = blockIdx.y; b < B; b += gridDim.y) {
        float res = 0.0f;
        if (nvalid >= 2) {
            const float *xb = x + b * Ein;
            float sgn = 1.0f, mn = 0.0f;
            bool first = true;
            for (int j = 1; j < W; ++j) {
                const int64_t id = row[j];
                if (id < 0 || j == last) continue;
                const float v = xb[id];
                sgn = sgn * torch_sign(v);
                const float a = fabsf(v);
                mn = first ? a : ((mn != mn || a != a) ? __builtin_nanf("") : fminf(mn, a));
                first = false;
            }
            res = sgn * mn;
        }
        out[b * R + r] = res;
    }
}

__global__ __launch_bounds__(256) void index_rows_varsum_kernel(const float *__restrict__ llr, int64_t B, int64_t Nv,
                                                                const float *__restrict__ c2v, int64_t Ein,
                                                                const int64_t *__restrict__ rows, int64_t R, int W,
                                                                int damp, float *__restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const int64_t *row = rows + r * W;
    const int64_t node = row[0];
    int last = -1;
    for (int j = 1; j < W; ++j)
        if (row[j] >= 0) last = j;
    for (int64_t b = blockIdx.y; b < B; b += gridDim.y) {
        const float *cb = c2v + b * Ein;
        float v = llr[b * Nv + node];
        if (last > 0) {
            float sum = 0.0f;
            bool first = true;
            for (int j = 1; j < W; ++j) {
                const int64_t id = row[j];
                if (id < 0) continue;
                sum = first ? cb[id] : sum + cb[id];
                first = false;
            }
            v = (v + sum) - cb[row[last]];
        }
        if (damp) v = 0.5f * v + 0.5f * cb[r];
        out[b * R + r] = v;
    }
}

dim3 rows_grid(int64_t R, int64_t B) {
    const unsigned gx = (unsigned)((R + 255) / 256);
    const unsigned gy = (unsigned)(B < 65535 ? (B > 0 ? B : 1) : 65535);
    return dim3(gx, gy);
}

}  // namespace
}  // namespace ldpc

using namespace ldpc;

extern "C" int ldpc_index_rows_minsum(const float *d_x, int64_t B, int64_t E_in, const int64_t *d_rows, int64_t R,
                                      int W, float *d_out, void *stream) {
    if (B < 0 || E_in < 0 || R < 0 || W < 1) return fail(LDPC_EINVAL, "bad dimensions");
    if (B == 0 || R == 0) return LDPC_OK;
    if (!d_x || !d_rows || !d_out) return fail(LDPC_EINVAL, "NULL tensor");
    if ((R + 255) / 256 > 0x7fffffffLL) return fail(LDPC_EUNSUPPORTED, "too many rows");
    hipLaunchKernelGGL(index_rows_minsum_kernel, rows_grid(R, B), dim3(256), 0, static_cast<hipStream_t>(stream),
                       d_x, B, E_in, d_rows, R, W, d_out);
    LDPC_CHECK_LAUNCH("index_rows_minsum_kernel");
    return LDPC_OK;
}

extern "C" int ldpc_index_rows_varsum(const float *d_llr, int64_t B, int64_t N_var, const float *d_c2v, int64_t E_in,
                                      const int64_t *d_rows, int64_t R, int W, int damp, float *d_out, void *stream) {
    if (B < 0 || N_var < 0 || E_in < 0 || R < 0 || W < 1) return fail(LDPC_EINVAL, "bad dimensions");
    if (damp && R != E_in) return fail(LDPC_EINVAL, "damping mixes output m with input message m: rows must equal E_in");
    if (B == 0 || R == 0) return LDPC_OK;
    if (!d_llr || !d_c2v || !d_rows || !d_out) return fail(LDPC_EINVAL, "NULL tensor");
    if ((R + 255) / 256 > 0x7fffffffLL) return fail(LDPC_EUNSUPPORTED, "too many rows");
    hipLaunchKernelGGL(index_rows_varsum_kernel, rows_grid(R, B), dim3(256), 0, static_cast<hipStream_t>(stream),
                       d_llr, B, N_var, d_c2v, E_in, d_rows, R, W, damp, d_out);
    LDPC_CHECK_LAUNCH("index_rows_varsum_kernel");
    return LDPC_OK;
}
