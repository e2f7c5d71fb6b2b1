// gnn_train.hip -- backward pass of the message-GNN decoder (fp32), for training on the device.
//
// The reference trains with torch autograd through MessageGNNDecoder.forward + the BCE of
// message_gnn_decoder.py:314 (loss.backward(), then SGD: trainer.py:70-102).  This file is that
// backward, written out by hand.  The forward (gnn.hip, fp32) saves every layer's output features
// x_{l+1}; the backward walks the layers in reverse and recomputes what it needs.
//
// Forward of layer l (message_gnn_decoder.py:51-129, :261), per message m of frame b:
//   c = x_l + emb[t]          a = mean_{var group of m} c       q = mean_{check group of m} c
//   u_v = W1v [c; a] + b1v    h_v = relu(u_v)    (same with W1c, [c; q] -> u_c, h_c)
//   x_{l+1} = W2v h_v + b2v + W2c h_c + b2c (+ x_l if l > 0)
// Head (:270-307): out_m = wo . x_L + bo,  z_v = llr_v + sum_{m -> v} out_m,  p = sigmoid(z).
//
// Backward, given G = dLoss/dp (from torch's BCE):
//   dz = G p (1 - p);  dout_m = dz[var(m)];  dX_L = dout (x) wo;  dwo = sum dout x_L;  dbo = sum dout
//   per layer, with dX = dLoss/dx_{l+1}:
//     dW2s += dX (x) h_s, db2s += dX;  dh_s = (W2s^T dX) * [u_s > 0]
//     dW1s += dh_s (x) [c; g_s], db1s += dh_s;  dz_s = W1s^T dh_s   (s = v, c;  g_v = a, g_c = q)
//     dc = dz_v[:H] + dz_c[:H] + mean_{var group}(dz_v[H:]) + mean_{check group}(dz_c[H:])
//          (the group-mean operator is symmetric, so its transpose is itself)
//     demb[t] += dc;  dx_l = dc (+ dX if l > 0);   layer 0: dw_in += dc llr, db_in += dc
//
// Kernels (lanes = hidden units, looping over units past 64; VALU fp32 -- a training batch is small
// next to the decode batches, and every product is an exact fp32 fma chain):
//   train_group_mean_kernel  group means of c (or of any (B, E, H) array), one wave per group
//   train_mlp_bwd_kernel     recompute u, h; dh, dz; writes c, h_v, h_c, dh_v, dh_c, dz parts
//   train_mlp_bwd_wide_kernel  the same for H > 64 (weights read through the caches, not LDS)
//   train_mlp_bwd_mfma_kernel  the same for H = 64 on fp32 MFMA (default; bit-for-bit fmaf chains
//                            in a different summation order than the VALU kernel)
//   train_combine_kernel     dc and dx_l
//   train_outer_kernel       weight gradients sum_r A_r (x) Z_r (+ bias sums), split over rows
//   train_colsum_kernel + train_vecfinal_kernel  emb / input-embedding / output-projection gradients
#include <cstdint>
#include <cstdlib>
#include <string>

#include "common.hpp"
#include "gnn.hpp"

namespace ldpc {
namespace {

constexpr int kMaxH = 64;         // widest H of the LDS-image kernels (train_mlp_bwd_kernel, train_outer_kernel)
// widest H trained: the training forward runs gnn_mlp_tiled_kernel (fma chains in k order) at every
// H != 64 up to 1024 -- never the wide MFMA path (gnn.hip carve(train)) -- and the wide backward
// recomputes exactly those products, so hv and the ReLU masks it rebuilds are the forward's bit for bit
constexpr int kMaxTrainH = 1024;

struct TW {  // one layer's weights in the blob (see ldpc_amd.h)
    const float *emb, *w1v, *b1v, *w2v, *b2v, *w1c, *b1c, *w2c, *b2c, *wo, *bo;
};
__host__ __device__ inline int64_t tl_floats(int H, int T) {
    return (int64_t)T * H + 2 * (2LL * H * H + H + (int64_t)H * H + H) + H + 1;
}
template <typename P>
__host__ __device__ inline void t_layer(P blob, int H, int T, int l, P *out) {  // 11 section pointers
    P e = blob + 2 * H + (int64_t)l * tl_floats(H, T);
    out[0] = e;                           // emb
    out[1] = out[0] + (int64_t)T * H;     // w1v
    out[2] = out[1] + 2LL * H * H;        // b1v
    out[3] = out[2] + H;                  // w2v
    out[4] = out[3] + (int64_t)H * H;     // b2v
    out[5] = out[4] + H;                  // w1c
    out[6] = out[5] + 2LL * H * H;        // b1c
    out[7] = out[6] + H;                  // w2c
    out[8] = out[7] + (int64_t)H * H;     // b2c
    out[9] = out[8] + H;                  // wo
    out[10] = out[9] + H;                 // bo
}

// ------------------------------------------------------------------------ head
__global__ void train_head_kernel(const float *__restrict__ p, const float *__restrict__ g, int64_t n,
                                  float *__restrict__ dz) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dz[i] = g[i] * (p[i] * (1.0f - p[i]));  // d sigmoid
}

// dX_L[r][u] = dz[b][var(m)] * wo[u]   (acc: dX[r][u] += that -- a deep-supervision head on an
// intermediate layer's output, added to the gradient that arrives from the layers above)
__global__ void train_dx_last_kernel(const float *__restrict__ dz, const int32_t *__restrict__ msg_var,
                                     const float *__restrict__ wo, int H, int64_t E, int N, int64_t n,
                                     float *__restrict__ dX, int acc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = i / H;
    const int u = (int)(i - r * H);
    const int64_t b = r / E, m = r - b * E;
    const float d = dz[b * N + msg_var[m]] * wo[u];
    dX[i] = acc ? dX[i] + d : d;
}

// Deep-supervision head (training only, no reference counterpart): out_m = wo . x_m + bo for every
// message row of one layer's saved output features (16 lanes per row, H <= 64); the variable sums
// and the sigmoid are the decoder's own output stage (gnn_output)
__global__ __launch_bounds__(256) void train_msg_head_kernel(const float *__restrict__ x, int H, int64_t R,
                                                             const float *__restrict__ wo, const float *__restrict__ bo,
                                                             float *__restrict__ msg_out) {
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const int q = threadIdx.x & 15;
    if (r >= R) return;  // whole 16-lane groups leave together
    const float *xr = x + r * H;
    float part = 0.0f;
    for (int u = q; u < H; u += 16) part = fmaf(xr[u], wo[u], part);
    for (int off = 8; off > 0; off >>= 1) part += __shfl_xor(part, off, 16);
    if (q == 0) msg_out[r] = part + bo[0];
}

// ------------------------------------------------------------------------ group means
// src_mode 0: src is the (B, E, H) array itself; 1: c = src + emb[type]; 2: c = w_in llr + b_in + emb
struct GmT {
    const float *src, *emb, *llr, *w_in, *b_in;
    const int32_t *msg_type, *msg_var, *ptr, *mem;
    const float *inv;
    float *dst;  // (B, G, H)
    int src_mode, G, H, N;
    int sum_only = 0;  // 1: plain group sums (inv ignored)
    int64_t E, B;
    const float *w = nullptr;  // weighted plan: member weights (s += w c, gnn_group_mean_kernel's expression)
};

__device__ __forceinline__ float c_value(const GmT &A, int64_t b, int64_t m, int u) {
    float v;
    if (A.src_mode == 2) v = A.w_in[u] * A.llr[b * A.N + A.msg_var[m]] + A.b_in[u];
    else v = A.src[(b * A.E + m) * A.H + u];
    if (A.src_mode != 0) v += A.emb[A.msg_type[m] * A.H + u];
    return v;
}

__global__ __launch_bounds__(256) void train_group_mean_kernel(GmT A) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= A.B * A.G) return;
    const int64_t b = w / A.G;
    const int g = (int)(w - b * A.G);
    for (int u = threadIdx.x & 63; u < A.H; u += 64) {
        float s = 0.0f;
        for (int q = A.ptr[g]; q < A.ptr[g + 1]; ++q) {
            if (A.w)
                s += A.w[q] * c_value(A, b, A.mem[q], u);
            else
                s += c_value(A, b, A.mem[q], u);
        }
        A.dst[w * A.H + u] = A.sum_only ? s : s * A.inv[g];
    }
}

// H = 64: 16 lanes per group (float4 each), 4 groups per wave, members unrolled by 4 (the
// kernel above keeps one 256-B row in flight per wave and is latency-bound)
__device__ __forceinline__ float4 c_value4(const GmT &A, int64_t b, int64_t m, int q) {
    float4 v;
    if (A.src_mode == 2) {
        const float l = A.llr[b * A.N + A.msg_var[m]];
        const float4 w = reinterpret_cast<const float4 *>(A.w_in)[q], bi = reinterpret_cast<const float4 *>(A.b_in)[q];
        v = make_float4(w.x * l + bi.x, w.y * l + bi.y, w.z * l + bi.z, w.w * l + bi.w);
    } else {
        v = reinterpret_cast<const float4 *>(A.src + (b * A.E + m) * 64)[q];
    }
    if (A.src_mode != 0) {
        const float4 e = reinterpret_cast<const float4 *>(A.emb + A.msg_type[m] * 64)[q];
        v = make_float4(v.x + e.x, v.y + e.y, v.z + e.z, v.w + e.w);
    }
    return v;
}

__global__ __launch_bounds__(256) void train_group_mean_h64_kernel(GmT A) {
    const int lane = threadIdx.x & 63, q = lane & 15;
    const int64_t gid = (xcd_block(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6)) * 4 + (lane >> 4);
    if (gid >= A.B * A.G) return;
    const int64_t b = gid / A.G;
    const int g = (int)(gid - b * A.G);
    const int p0 = A.ptr[g], p1 = A.ptr[g + 1];
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    int p = p0;
    for (; p + 4 <= p1; p += 4) {  // loads first; the adds keep the member order of the kernel above
        const float4 v0 = c_value4(A, b, A.mem[p], q), v1 = c_value4(A, b, A.mem[p + 1], q);
        const float4 v2 = c_value4(A, b, A.mem[p + 2], q), v3 = c_value4(A, b, A.mem[p + 3], q);
        acc.x += v0.x; acc.y += v0.y; acc.z += v0.z; acc.w += v0.w;
        acc.x += v1.x; acc.y += v1.y; acc.z += v1.z; acc.w += v1.w;
        acc.x += v2.x; acc.y += v2.y; acc.z += v2.z; acc.w += v2.w;
        acc.x += v3.x; acc.y += v3.y; acc.z += v3.z; acc.w += v3.w;
    }
    for (; p < p1; ++p) {
        const float4 v = c_value4(A, b, A.mem[p], q);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (!A.sum_only) {
        const float inv = A.inv[g];
        acc = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
    }
    reinterpret_cast<float4 *>(A.dst + gid * 64)[q] = acc;
}

int launch_group_mean(const GmT &g, hipStream_t s) {
    const int64_t n = g.B * g.G;
    if (g.H == 64 && !g.w)
        hipLaunchKernelGGL(train_group_mean_h64_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, s, g);
    else
        hipLaunchKernelGGL(train_group_mean_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, g);
    LDPC_CHECK_LAUNCH("train_group_mean_kernel");
    return LDPC_OK;
}

// ------------------------------------------------------------------------ MLP backward
constexpr int kNM = 4;  // rows per wave and step (share every weight read from LDS)

struct MlpT {
    const float *x, *llr, *w_in, *b_in;  // x = x_l (null at layer 0)
    const float *Mv, *Mc, *dX;
    const int32_t *msg_type, *msg_var, *vgroup, *cgroup;
    const float *emb, *w1v, *b1v, *w2v, *w1c, *b1c, *w2c;
    float *cbuf, *hv, *hc, *dhv, *dhc, *dco, *da, *db;
    int H, N, Gv, Gc;
    int64_t E, R;  // R = B E rows
};

// LDS (floats): W1v, W1c [H][2H + 1]; W2v, W2c [H][H + 1]; b1v, b1c [H];
// per wave: z [kNM][3H] (c | a | q), dX [kNM][H], dh [kNM][2][H]
inline size_t mlp_bwd_lds(int H) {
    return ((size_t)2 * H * (2 * H + 1) + 2 * H * (H + 1) + 2 * H + 4 * (size_t)kNM * (3 * H + H + 2 * H)) * 4;
}

__global__ __launch_bounds__(256) void train_mlp_bwd_kernel(MlpT A) {
    extern __shared__ float sm[];
    const int H = A.H, H2 = 2 * H, S1 = H2 + 1, S2 = H + 1;
    float *W1v = sm, *W1c = W1v + H * S1, *W2v = W1c + H * S1, *W2c = W2v + H * S2;
    float *b1v = W2c + H * S2, *b1c = b1v + H;
    const int wave = threadIdx.x >> 6, u = threadIdx.x & 63;
    float *z = b1c + H + wave * kNM * 6 * H, *dXs = z + kNM * 3 * H, *dh = dXs + kNM * H;
    for (int i = threadIdx.x; i < H * H2; i += 256) {
        const int o = i / H2, k = i - o * H2;
        W1v[o * S1 + k] = A.w1v[i];
        W1c[o * S1 + k] = A.w1c[i];
    }
    for (int i = threadIdx.x; i < H * H; i += 256) {
        const int o = i / H, k = i - o * H;
        W2v[o * S2 + k] = A.w2v[i];
        W2c[o * S2 + k] = A.w2c[i];
    }
    if (threadIdx.x < H) {
        b1v[threadIdx.x] = A.b1v[threadIdx.x];
        b1c[threadIdx.x] = A.b1c[threadIdx.x];
    }
    __syncthreads();
    const bool lane_on = u < H;
    const int64_t step = (int64_t)gridDim.x * 4 * kNM;
    for (int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * kNM; r0 - wave * kNM < A.R; r0 += step) {
        // stage c | a | q and dX of this wave's kNM rows
        float uv[kNM], uc[kNM];
#pragma unroll
        for (int i = 0; i < kNM; ++i) {
            const int64_t r = r0 + i;
            if (lane_on && r < A.R) {
                const int64_t b = r / A.E, m = r - b * A.E;
                const float c = (A.x ? A.x[r * H + u] : A.w_in[u] * A.llr[b * A.N + A.msg_var[m]] + A.b_in[u]) +
                                A.emb[A.msg_type[m] * H + u];
                z[i * 3 * H + u] = c;
                z[i * 3 * H + H + u] = A.Mv[(b * A.Gv + A.vgroup[m]) * H + u];
                z[i * 3 * H + H2 + u] = A.Mc[(b * A.Gc + A.cgroup[m]) * H + u];
                dXs[i * H + u] = A.dX[r * H + u];
                A.cbuf[r * H + u] = c;
            } else if (lane_on) {
                z[i * 3 * H + u] = z[i * 3 * H + H + u] = z[i * 3 * H + H2 + u] = 0.0f;
                dXs[i * H + u] = 0.0f;
            }
        }
        __syncthreads();
        if (lane_on) {
            // u_s = W1s [c; g_s] + b1s   (row u of W1, lanes on rows: stride 2H + 1, conflict-free)
#pragma unroll
            for (int i = 0; i < kNM; ++i) { uv[i] = b1v[u]; uc[i] = b1c[u]; }
            for (int k = 0; k < H; ++k) {  // c part, shared by both sides
                const float wv = W1v[u * S1 + k], wc = W1c[u * S1 + k];
#pragma unroll
                for (int i = 0; i < kNM; ++i) {
                    const float c = z[i * 3 * H + k];
                    uv[i] = fmaf(wv, c, uv[i]);
                    uc[i] = fmaf(wc, c, uc[i]);
                }
            }
            for (int k = 0; k < H; ++k) {
                const float wv = W1v[u * S1 + H + k], wc = W1c[u * S1 + H + k];
#pragma unroll
                for (int i = 0; i < kNM; ++i) {
                    uv[i] = fmaf(wv, z[i * 3 * H + H + k], uv[i]);
                    uc[i] = fmaf(wc, z[i * 3 * H + H2 + k], uc[i]);
                }
            }
            // dh_s = (W2s^T dX) * [u_s > 0]   (column u of W2: lanes on columns)
            float gv[kNM], gc[kNM];
#pragma unroll
            for (int i = 0; i < kNM; ++i) gv[i] = gc[i] = 0.0f;
            for (int o = 0; o < H; ++o) {
                const float wv = W2v[o * S2 + u], wc = W2c[o * S2 + u];
#pragma unroll
                for (int i = 0; i < kNM; ++i) {
                    const float d = dXs[i * H + o];
                    gv[i] = fmaf(wv, d, gv[i]);
                    gc[i] = fmaf(wc, d, gc[i]);
                }
            }
#pragma unroll
            for (int i = 0; i < kNM; ++i) {
                const int64_t r = r0 + i;
                const float dv = uv[i] > 0.0f ? gv[i] : 0.0f, dc = uc[i] > 0.0f ? gc[i] : 0.0f;
                dh[(i * 2) * H + u] = dv;
                dh[(i * 2 + 1) * H + u] = dc;
                if (r < A.R) {
                    A.hv[r * H + u] = relu_nan(uv[i]);
                    A.hc[r * H + u] = relu_nan(uc[i]);
                    A.dhv[r * H + u] = dv;
                    A.dhc[r * H + u] = dc;
                }
            }
        }
        __syncthreads();
        if (lane_on) {
            // dz_s[k] = sum_u W1s[u][k] dh_s[u] for k = u (c part) and k = H + u (group part)
            float zc0[kNM], zv1[kNM], zc1[kNM];
#pragma unroll
            for (int i = 0; i < kNM; ++i) zc0[i] = zv1[i] = zc1[i] = 0.0f;
            float zv0[kNM];
#pragma unroll
            for (int i = 0; i < kNM; ++i) zv0[i] = 0.0f;
            for (int q = 0; q < H; ++q) {
                const float wv0 = W1v[q * S1 + u], wv1 = W1v[q * S1 + H + u];
                const float wc0 = W1c[q * S1 + u], wc1 = W1c[q * S1 + H + u];
#pragma unroll
                for (int i = 0; i < kNM; ++i) {
                    const float dv = dh[(i * 2) * H + q], dc = dh[(i * 2 + 1) * H + q];
                    zv0[i] = fmaf(wv0, dv, zv0[i]);
                    zv1[i] = fmaf(wv1, dv, zv1[i]);
                    zc0[i] = fmaf(wc0, dc, zc0[i]);
                    zc1[i] = fmaf(wc1, dc, zc1[i]);
                }
            }
#pragma unroll
            for (int i = 0; i < kNM; ++i) {
                const int64_t r = r0 + i;
                if (r < A.R) {
                    A.dco[r * H + u] = zv0[i] + zc0[i];
                    A.da[r * H + u] = zv1[i];
                    A.db[r * H + u] = zc1[i];
                }
            }
        }
        __syncthreads();
    }
}

// H > 64: the same products and fma order as train_mlp_bwd_kernel (lanes = units, each lane
// looping over units lane, lane + 64, ...), with the weights read from global memory -- the
// [H][2H + 1] LDS image stops fitting past H = 64 -- and only the per-wave rows in LDS: c | a | q,
// dX and dh of kNM rows (24 H floats per wave).  GEMM2' and GEMM3' read W rows across the lanes
// (coalesced); GEMM1 walks each lane's own W1 row (one cache line per lane per 32 k).
inline size_t mlp_bwd_wide_lds(int H, int waves) { return (size_t)waves * kNM * 6 * H * 4; }

__global__ __launch_bounds__(256) void train_mlp_bwd_wide_kernel(MlpT A) {
    extern __shared__ float sm[];
    const int H = A.H, H2 = 2 * H, nw = blockDim.x >> 6;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float *z = sm + wave * kNM * 6 * H, *dXs = z + kNM * 3 * H, *dh = dXs + kNM * H;
    const int64_t step = (int64_t)gridDim.x * nw * kNM;
    for (int64_t r0 = ((int64_t)blockIdx.x * nw + wave) * kNM; r0 - wave * kNM < A.R; r0 += step) {
        for (int u = lane; u < H; u += 64) {
#pragma unroll
            for (int i = 0; i < kNM; ++i) {
                const int64_t r = r0 + i;
                if (r < A.R) {
                    const int64_t b = r / A.E, m = r - b * A.E;
                    const float c = (A.x ? A.x[r * H + u] : A.w_in[u] * A.llr[b * A.N + A.msg_var[m]] + A.b_in[u]) +
                                    A.emb[A.msg_type[m] * H + u];
                    z[i * 3 * H + u] = c;
                    z[i * 3 * H + H + u] = A.Mv[(b * A.Gv + A.vgroup[m]) * H + u];
                    z[i * 3 * H + H2 + u] = A.Mc[(b * A.Gc + A.cgroup[m]) * H + u];
                    dXs[i * H + u] = A.dX[r * H + u];
                    A.cbuf[r * H + u] = c;
                } else {
                    z[i * 3 * H + u] = z[i * 3 * H + H + u] = z[i * 3 * H + H2 + u] = 0.0f;
                    dXs[i * H + u] = 0.0f;
                }
            }
        }
        __syncthreads();
        for (int u = lane; u < H; u += 64) {
            // u_s = W1s [c; g_s] + b1s (row u of W1s)
            float uv[kNM], uc[kNM];
#pragma unroll
            for (int i = 0; i < kNM; ++i) { uv[i] = A.b1v[u]; uc[i] = A.b1c[u]; }
            const float *w1v = A.w1v + (int64_t)u * H2, *w1c = A.w1c + (int64_t)u * H2;
            for (int k = 0; k < H; ++k) {
                const float wv = w1v[k], wc = w1c[k];
#pragma unroll
                for (int i = 0; i < kNM; ++i) {
                    const float c = z[i * 3 * H + k];
                    uv[i] = fmaf(wv, c, uv[i]);
                    uc[i] = fmaf(wc, c, uc[i]);
                }
            }
            for (int k = 0; k < H; ++k) {
                const float wv = w1v[H + k], wc = w1c[H + k];
#pragma unroll
                for (int i = 0; i < kNM; ++i) {
                    uv[i] = fmaf(wv, z[i * 3 * H + H + k], uv[i]);
                    uc[i] = fmaf(wc, z[i * 3 * H + H2 + k], uc[i]);
                }
            }
            // dh_s = (W2s^T dX) * [u_s > 0] (column u of W2s)
            float gv[kNM], gc[kNM];
#pragma unroll
            for (int i = 0; i < kNM; ++i) gv[i] = gc[i] = 0.0f;
            for (int o = 0; o < H; ++o) {
                const float wv = A.w2v[(int64_t)o * H + u], wc = A.w2c[(int64_t)o * H + u];
#pragma unroll
                for (int i = 0; i < kNM; ++i) {
                    const float d = dXs[i * H + o];
                    gv[i] = fmaf(wv, d, gv[i]);
                    gc[i] = fmaf(wc, d, gc[i]);
                }
            }
#pragma unroll
            for (int i = 0; i < kNM; ++i) {
                const int64_t r = r0 + i;
                const float dv = uv[i] > 0.0f ? gv[i] : 0.0f, dc = uc[i] > 0.0f ? gc[i] : 0.0f;
                dh[(i * 2) * H + u] = dv;
                dh[(i * 2 + 1) * H + u] = dc;
                if (r < A.R) {
                    A.hv[r * H + u] = relu_nan(uv[i]);
                    A.hc[r * H + u] = relu_nan(uc[i]);
                    A.dhv[r * H + u] = dv;
                    A.dhc[r * H + u] = dc;
                }
            }
        }
        __syncthreads();
        for (int u = lane; u < H; u += 64) {
            // dz_s[k] = sum_q W1s[q][k] dh_s[q] for k = u (c part) and k = H + u (group part)
            float zv0[kNM], zv1[kNM], zc0[kNM], zc1[kNM];
#pragma unroll
            for (int i = 0; i < kNM; ++i) zv0[i] = zv1[i] = zc0[i] = zc1[i] = 0.0f;
            for (int q = 0; q < H; ++q) {
                const float *rv = A.w1v + (int64_t)q * H2, *rc = A.w1c + (int64_t)q * H2;
                const float wv0 = rv[u], wv1 = rv[H + u], wc0 = rc[u], wc1 = rc[H + u];
#pragma unroll
                for (int i = 0; i < kNM; ++i) {
                    const float dv = dh[(i * 2) * H + q], dc = dh[(i * 2 + 1) * H + q];
                    zv0[i] = fmaf(wv0, dv, zv0[i]);
                    zv1[i] = fmaf(wv1, dv, zv1[i]);
                    zc0[i] = fmaf(wc0, dc, zc0[i]);
                    zc1[i] = fmaf(wc1, dc, zc1[i]);
                }
            }
#pragma unroll
            for (int i = 0; i < kNM; ++i) {
                const int64_t r = r0 + i;
                if (r < A.R) {
                    A.dco[r * H + u] = zv0[i] + zc0[i];
                    A.da[r * H + u] = zv1[i];
                    A.db[r * H + u] = zc1[i];
                }
            }
        }
        __syncthreads();
    }
}

// ---- H = 64 on v_mfma_f32_32x32x2_f32: the same three products per message as the kernel above,
// in the forward's transposed orientation (hidden units / input features on the MFMA rows,
// 32 messages of a tile on the columns; lane (j, h) = message j, half h):
//   GEMM1  u = W1 [c; g]       A = W1[u][k]   B = in[k]: half 0 lanes carry c, half 1 lanes g
//                               (k-step kk pairs input k = kk with k = 64 + kk)
//   GEMM2' d = W2^T dX         A = W2[o][u]   B = dX[o]: half h carries o = 32 h + kk
//   GEMM3' dz = W1^T dh        A = W1[u][k]   B = dh straight from GEMM2's accumulators (step
//                               (rt, r) pairs unit 32 rt + crow(r, 0) with 32 rt + crow(r, 1))
// One padded row-major copy of each W1 ([64][129]) serves GEMM1 (lanes walk u: stride 129 words,
// conflict-free within each 32-lane ds_read_b32 group) and GEMM3' (lanes walk k: consecutive
// words); W2 is [64][65].  The dz of the c part of both sides accumulates in one register tile
// (dco); the group parts go out per side.
constexpr int kS1 = 129, kS2 = 65;
inline size_t mlp_bwd_mfma_lds() { return ((size_t)2 * 64 * kS1 + 2 * 64 * kS2 + 128) * 4; }

typedef float f32x16 __attribute__((ext_vector_type(16)));
struct F64 {
    float v[64];
    __device__ __forceinline__ float &operator[](int i) { return v[i]; }
    __device__ __forceinline__ float operator[](int i) const { return v[i]; }
};
__device__ __forceinline__ int crow_t(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// PJ (projected groups, the default): Mv / Mc hold the side's projected group rows W1_right g + b1
// (gnn_project_groups), so GEMM1 runs over c alone (lane half h carries c[32 h + kk]) from that
// row, and GEMM3' computes only the c part of dz: the group part's mean over a group is
// W1_right^T (mean of dh over the group), formed per group afterwards (train_group_back_kernel).
// Per side 64 + 64 + 64 MFMAs instead of 64 + 128 + 128.
template <int NT, bool PJ = false>
__global__ __launch_bounds__(NT, NT / 256 > 1 ? NT / 256 : 1) void train_mlp_bwd_mfma_kernel(MlpT A) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    constexpr int H = 64;
    float *W1v = sm, *W1c = W1v + H * kS1, *W2v = W1c + H * kS1, *W2c = W2v + H * kS2;
    float *b1 = W2c + H * kS2;  // b1v [64], b1c [64]
    for (int i = threadIdx.x; i < H * 2 * H; i += NT) {
        const int o = i >> 7, k = i & 127;
        W1v[o * kS1 + k] = A.w1v[i];
        W1c[o * kS1 + k] = A.w1c[i];
    }
    for (int i = threadIdx.x; i < H * H; i += NT) {
        const int o = i >> 6, k = i & 63;
        W2v[o * kS2 + k] = A.w2v[i];
        W2c[o * kS2 + k] = A.w2c[i];
    }
    if (threadIdx.x < H) {
        b1[threadIdx.x] = A.b1v[threadIdx.x];
        b1[H + threadIdx.x] = A.b1c[threadIdx.x];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 31, half = lane >> 5, wave = threadIdx.x >> 6;
    const int64_t ntiles = (A.R + 31) / 32;
    const TileWalk tw = xcd_tiles(ntiles, NT / 64, wave);
    for (int64_t t = tw.first; t < tw.end; t += tw.stride) {
        const int64_t row = t * 32 + j;
        const bool ok = row < A.R;
        const int64_t rr = ok ? row : A.R - 1;
        const int64_t b = rr / A.E, m = rr - b * A.E;
        // B operand of GEMM1, rebuilt per side so it is not live across GEMM3': half 0 lanes c =
        // x (or w_in llr + b_in) + emb[type] (written to cbuf on side 0 for the weight gradients),
        // half 1 lanes the side's group mean
        auto load_in = [&](int side) {
            F64 in;
            if (PJ) {  // c[32 half + kk], kk < 32
                const float4 *e = reinterpret_cast<const float4 *>(A.emb + A.msg_type[m] * H + 32 * half);
                if (A.x) {
                    const float4 *xr = reinterpret_cast<const float4 *>(A.x + rr * H + 32 * half);
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const float4 v = xr[q], ev = e[q];
                        in[4 * q] = v.x + ev.x; in[4 * q + 1] = v.y + ev.y;
                        in[4 * q + 2] = v.z + ev.z; in[4 * q + 3] = v.w + ev.w;
                    }
                } else {
                    const float l = A.llr[b * A.N + A.msg_var[m]];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const float4 ev = e[q];
                        const float4 w = reinterpret_cast<const float4 *>(A.w_in + 32 * half)[q];
                        const float4 bi = reinterpret_cast<const float4 *>(A.b_in + 32 * half)[q];
                        in[4 * q] = (w.x * l + bi.x) + ev.x; in[4 * q + 1] = (w.y * l + bi.y) + ev.y;
                        in[4 * q + 2] = (w.z * l + bi.z) + ev.z; in[4 * q + 3] = (w.w * l + bi.w) + ev.w;
                    }
                }
                if (side == 0 && ok && A.cbuf) {
                    float4 *cb = reinterpret_cast<float4 *>(A.cbuf + row * H + 32 * half);
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        cb[q] = make_float4(in[4 * q], in[4 * q + 1], in[4 * q + 2], in[4 * q + 3]);
                }
                return in;
            }
            if (half == 0) {
                const float4 *e = reinterpret_cast<const float4 *>(A.emb + A.msg_type[m] * H);
                if (A.x) {
                    const float4 *xr = reinterpret_cast<const float4 *>(A.x + rr * H);
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const float4 v = xr[q], ev = e[q];
                        in[4 * q] = v.x + ev.x; in[4 * q + 1] = v.y + ev.y;
                        in[4 * q + 2] = v.z + ev.z; in[4 * q + 3] = v.w + ev.w;
                    }
                } else {
                    const float l = A.llr[b * A.N + A.msg_var[m]];
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const float4 ev = e[q];
                        const float4 w = reinterpret_cast<const float4 *>(A.w_in)[q];
                        const float4 bi = reinterpret_cast<const float4 *>(A.b_in)[q];
                        in[4 * q] = (w.x * l + bi.x) + ev.x; in[4 * q + 1] = (w.y * l + bi.y) + ev.y;
                        in[4 * q + 2] = (w.z * l + bi.z) + ev.z; in[4 * q + 3] = (w.w * l + bi.w) + ev.w;
                    }
                }
                if (side == 0 && ok) {
                    float4 *cb = reinterpret_cast<float4 *>(A.cbuf + row * H);
#pragma unroll
                    for (int q = 0; q < 16; ++q)
                        cb[q] = make_float4(in[4 * q], in[4 * q + 1], in[4 * q + 2], in[4 * q + 3]);
                }
            } else {
                const float4 *g = reinterpret_cast<const float4 *>(
                    side == 0 ? A.Mv + (b * A.Gv + A.vgroup[m]) * H : A.Mc + (b * A.Gc + A.cgroup[m]) * H);
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const float4 v = g[q];
                    in[4 * q] = v.x; in[4 * q + 1] = v.y; in[4 * q + 2] = v.z; in[4 * q + 3] = v.w;
                }
            }
            return in;
        };
        f32x16 dco0 = {}, dco1 = {};
        int l1 = j * kS1 + 64 * half, l2 = (32 * half) * kS2 + j, l3 = j;  // per-lane LDS bases
        asm volatile("" : "+v"(l1), "+v"(l2), "+v"(l3));
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const float *W1 = side == 0 ? W1v : W1c, *W2 = side == 0 ? W2v : W2c, *bs = b1 + 64 * side;
            // GEMM2' first (dX is re-read per side, L2-hot, so it is not live across GEMM1):
            // d[u][msg] = sum_o W2[o][u] dX[o]; A = W2[32 half + kk][32 rt + j]
            f32x16 d0 = {}, d1 = {};
            {
                float dx[32];
                const float4 *dp = reinterpret_cast<const float4 *>(A.dX + rr * H + 32 * half);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const float4 v = dp[q];
                    dx[4 * q] = v.x; dx[4 * q + 1] = v.y; dx[4 * q + 2] = v.z; dx[4 * q + 3] = v.w;
                }
#pragma unroll
                for (int kk = 0; kk < 32; ++kk) {
                    const float *wr = W2 + l2 + kk * kS2;
                    d0 = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[0], dx[kk], d0, 0, 0, 0);
                    d1 = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[32], dx[kk], d1, 0, 0, 0);
                }
            }
            // GEMM1: u[32 rt + i][msg]; A = W1[32 rt + j][64 half + kk]
            f32x16 u0 = {}, u1 = {};
            if constexpr (PJ) {  // from the projected row (b1 included); A = W1[32 rt + j][32 half + kk]
                const float *pr = side == 0 ? A.Mv + (b * A.Gv + A.vgroup[m]) * H : A.Mc + (b * A.Gc + A.cgroup[m]) * H;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 p0 = *reinterpret_cast<const float4 *>(pr + 8 * q + 4 * half);
                    const float4 p1 = *reinterpret_cast<const float4 *>(pr + 32 + 8 * q + 4 * half);
                    u0[4 * q] = p0.x; u0[4 * q + 1] = p0.y; u0[4 * q + 2] = p0.z; u0[4 * q + 3] = p0.w;
                    u1[4 * q] = p1.x; u1[4 * q + 1] = p1.y; u1[4 * q + 2] = p1.z; u1[4 * q + 3] = p1.w;
                }
                const F64 in = load_in(side);
                const int lp = j * kS1 + 32 * half;
#pragma unroll
                for (int kk = 0; kk < 32; ++kk) {
                    const float *wr = W1 + lp + kk;
                    u0 = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[0], in[kk], u0, 0, 0, 0);
                    u1 = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[32 * kS1], in[kk], u1, 0, 0, 0);
                }
            } else {
                const F64 in = load_in(side);
#pragma unroll
                for (int kk = 0; kk < 64; ++kk) {
                    const float *wr = W1 + l1 + kk;
                    u0 = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[0], in[kk], u0, 0, 0, 0);
                    u1 = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[32 * kS1], in[kk], u1, 0, 0, 0);
                }
            }
            // bias, relu, mask: lane holds units 32 rt + crow(r, half)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float a0 = PJ ? u0[r] : u0[r] + bs[crow_t(r, half)];
                const float a1 = PJ ? u1[r] : u1[r] + bs[32 + crow_t(r, half)];
                u0[r] = relu_nan(a0);
                u1[r] = relu_nan(a1);
                d0[r] = a0 > 0.0f ? d0[r] : 0.0f;
                d1[r] = a1 > 0.0f ? d1[r] : 0.0f;
            }
            if (ok) {
                float *ho = (side == 0 ? A.hv : A.hc) + row * H, *dho = (side == 0 ? A.dhv : A.dhc) + row * H;
#pragma unroll
                for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const f32x16 &uu = rt ? u1 : u0, &dd = rt ? d1 : d0;
                        const int o0 = 32 * rt + 8 * q + 4 * half;
                        *reinterpret_cast<float4 *>(ho + o0) =
                            make_float4(uu[4 * q], uu[4 * q + 1], uu[4 * q + 2], uu[4 * q + 3]);
                        *reinterpret_cast<float4 *>(dho + o0) =
                            make_float4(dd[4 * q], dd[4 * q + 1], dd[4 * q + 2], dd[4 * q + 3]);
                    }
            }
            // GEMM3': dz[k][msg] = sum_u W1[u][k] dh[u]; A = W1[32 rt + crow(r, half)][32 kt + j]
#pragma unroll
            for (int kt = 0; kt < (PJ ? 2 : 4); ++kt) {
                f32x16 acc = kt == 0 ? dco0 : kt == 1 ? dco1 : f32x16{};
#pragma unroll
                for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float w = W1[l3 + (32 * rt + crow_t(r, half)) * kS1 + 32 * kt];
                        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w, rt ? d1[r] : d0[r], acc, 0, 0, 0);
                    }
                __builtin_amdgcn_sched_barrier(0);  // keep each kt's 32 A reads next to their MFMAs
                if (kt == 0) dco0 = acc;
                else if (kt == 1) dco1 = acc;
                else if (ok) {  // group part: k = 64 + 32 (kt - 2) + unit
                    float *go = (side == 0 ? A.da : A.db) + row * H + 32 * (kt - 2);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        *reinterpret_cast<float4 *>(go + 8 * q + 4 * half) =
                            make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
                }
            }
        }
        if (ok) {
            float *co = A.dco + row * H;
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const f32x16 &cc = rt ? dco1 : dco0;
                    *reinterpret_cast<float4 *>(co + 32 * rt + 8 * q + 4 * half) =
                        make_float4(cc[4 * q], cc[4 * q + 1], cc[4 * q + 2], cc[4 * q + 3]);
                }
        }
    }
}

// ---- H = 64, projected groups, every fp32 product as bf16x6 splits on v_mfma_f32_32x32x16_bf16
// (gnn_mlp2s_kernel's scheme: the results are fp32 GEMMs up to summation order, at 6 x 32 instead
// of 8 x 64 MFMA cycles per K = 16).  Same outputs as train_mlp_bwd_mfma_kernel<.., true>; hidden
// units / input features on the MFMA rows, the tile's 32 messages on the columns, per side:
//   GEMM2'  d  = W2^T dX     A[u][o] = W2[o][u]            B: dX, natural K order
//   GEMM1   u  = W1_left c   A[u][p] = W1[u][pi16(p)]      B: c in pi16 K order (x loaded as the
//                             + P (the projected row)       forward loads it)
//   GEMM3'  dz = W1_left^T dh A[k][p] = W1[pi16(p)][k]      B: dh's accumulator registers as they
//                             (both sides into one tile)    stand (k-step t = registers 8 (t&1) ..
//                                                           of tile t >> 1)
// Six A images (2 sides x 3 matrices) x 3 bf16 splits in 147 KB of LDS: 64-element rows with the
// 16-byte chunks XOR-swizzled by (row >> 1) & 7, so a ds_read_b128 of 16 rows hits 16 bank groups.
constexpr int kB6Img = 64 * 64;  // bf16 per split image
__device__ __forceinline__ int b6_at(int row, int k) { return row * 64 + (((k >> 3) ^ ((row >> 1) & 7)) << 3) + (k & 7); }
inline size_t mlp_bwd_s6_lds() { return (size_t)18 * kB6Img * 2; }
// acc += A B over k-step chunk pair (lane half h reads chunk 2 s + h of row r): A from the three
// split images at img + off (off = b6_at(r, 16 s + 8 h)), B the three splits of the lane's operand
__device__ __forceinline__ f32x16 mfma6o(const __bf16 *img, int off, const bf16x8_t &b0, const bf16x8_t &b1,
                                         const bf16x8_t &b2, f32x16 acc) {
    return mfma6(img + off, b0, b1, b2, acc, kB6Img);
}

__global__ __launch_bounds__(512, 1) void train_mlp_bwd_s6_kernel(MlpT A) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    __bf16 *img = reinterpret_cast<__bf16 *>(sm);  // image m (G2T_v, G1_v, G3_v, G2T_c, G1_c, G3_c), split q: 3 m + q
    constexpr int H = 64;
    for (int i = threadIdx.x; i < H * H; i += 512) {
        const int r = i >> 6, p = i & 63, up = pi16(p);
        const float w[6] = {A.w2v[p * H + r], A.w1v[r * 2 * H + up], A.w1v[up * 2 * H + r],
                            A.w2c[p * H + r], A.w1c[r * 2 * H + up], A.w1c[up * 2 * H + r]};
#pragma unroll
        for (int q = 0; q < 6; ++q) split_store(w[q], img + 3 * q * kB6Img + b6_at(r, p), kB6Img);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 31, half = lane >> 5,
              wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // A fragment offsets    // A fragment offsets of row j per k-step (row j + 32: + 32 * 64, the same swizzle)
    int aoff[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) aoff[s] = b6_at(j, 16 * s + 8 * half);
    const __bf16 *G2[2] = {img, img + 9 * kB6Img}, *G1[2] = {img + 3 * kB6Img, img + 12 * kB6Img},
                 *G3[2] = {img + 6 * kB6Img, img + 15 * kB6Img};
    const int64_t ntiles = (A.R + 31) / 32;
    const TileWalk tw = xcd_tiles(ntiles, 8, wave);
    // this tile's dX (k-step s: o = 16 s + 8 h + i) and x (feature pi16(16 s + 8 h + i)) rows; the
    // next tile's load under this tile's GEMM3' (layer 0 forms its x from the LLR at the tile)
    float dxr[4][8], xr[4][8];
    auto load_rows = [&](int64_t rq) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const float4 v = *reinterpret_cast<const float4 *>(A.dX + rq * H + 16 * s + 8 * half + 4 * q);
                dxr[s][4 * q] = v.x; dxr[s][4 * q + 1] = v.y; dxr[s][4 * q + 2] = v.z; dxr[s][4 * q + 3] = v.w;
                if (A.x) {
                    const float4 w = *reinterpret_cast<const float4 *>(A.x + rq * H + 32 * (s >> 1) + 16 * (s & 1) + 8 * q + 4 * half);
                    xr[s][4 * q] = w.x; xr[s][4 * q + 1] = w.y; xr[s][4 * q + 2] = w.z; xr[s][4 * q + 3] = w.w;
                }
            }
    };
    if (tw.first < tw.end) load_rows(std::min<int64_t>(tw.first * 32 + j, A.R - 1));
    for (int64_t t = tw.first; t < tw.end; t += tw.stride) {
        const int64_t row = t * 32 + j;
        const bool ok = row < A.R;
        const int64_t rr = ok ? row : A.R - 1;
        const int64_t b = rr / A.E, m = rr - b * A.E;
        const int64_t rn = std::min<int64_t>((t + tw.stride < tw.end ? t + tw.stride : t) * 32 + j, A.R - 1);
        // GEMM2' of both sides over one split of dX per k-step
        f32x16 d[2][2] = {};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            bf16x8_t b0, b1, b2;
            split3(dxr[s], b0, b1, b2);
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                d[side][0] = mfma6o(G2[side], aoff[s], b0, b1, b2, d[side][0]);
                d[side][1] = mfma6o(G2[side], aoff[s] + 32 * 64, b0, b1, b2, d[side][1]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // GEMM1 of both sides over one split of c, each from its projected row W1_right g + b1
        f32x16 u[2][2];
        {
            const float *pv = A.Mv + (b * A.Gv + A.vgroup[m]) * H + 4 * half;
            const float *pc = A.Mc + (b * A.Gc + A.cgroup[m]) * H + 4 * half;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int side = 0; side < 2; ++side) {
                    const float *pr = side ? pc : pv;
                    const float4 a = *reinterpret_cast<const float4 *>(pr + 8 * q);
                    const float4 c = *reinterpret_cast<const float4 *>(pr + 32 + 8 * q);
                    u[side][0][4 * q] = a.x; u[side][0][4 * q + 1] = a.y; u[side][0][4 * q + 2] = a.z; u[side][0][4 * q + 3] = a.w;
                    u[side][1][4 * q] = c.x; u[side][1][4 * q + 1] = c.y; u[side][1][4 * q + 2] = c.z; u[side][1][4 * q + 3] = c.w;
                }
            }
        }
        const float *e = A.emb + A.msg_type[m] * H;
        const float l = A.x ? 0.0f : A.llr[b * A.N + A.msg_var[m]];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            // c[i] = feature pi16(16 s + 8 h + i) = 32 (s >> 1) + 16 (s & 1) + 8 (i >> 2) + 4 h + (i & 3)
            float c[8];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int u0 = 32 * (s >> 1) + 16 * (s & 1) + 8 * q + 4 * half;
                const float4 ev = *reinterpret_cast<const float4 *>(e + u0);
                float4 xv;
                if (A.x) {
                    xv = make_float4(xr[s][4 * q], xr[s][4 * q + 1], xr[s][4 * q + 2], xr[s][4 * q + 3]);
                } else {
                    const float4 w = *reinterpret_cast<const float4 *>(A.w_in + u0);
                    const float4 bi = *reinterpret_cast<const float4 *>(A.b_in + u0);
                    xv = make_float4(w.x * l + bi.x, w.y * l + bi.y, w.z * l + bi.z, w.w * l + bi.w);
                }
                c[4 * q] = xv.x + ev.x; c[4 * q + 1] = xv.y + ev.y; c[4 * q + 2] = xv.z + ev.z; c[4 * q + 3] = xv.w + ev.w;
                if (ok && A.cbuf)
                    *reinterpret_cast<float4 *>(A.cbuf + row * H + u0) = make_float4(c[4 * q], c[4 * q + 1], c[4 * q + 2], c[4 * q + 3]);
            }
            bf16x8_t c0, c1, c2;
            split3(c, c0, c1, c2);
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                u[side][0] = mfma6o(G1[side], aoff[s], c0, c1, c2, u[side][0]);
                u[side][1] = mfma6o(G1[side], aoff[s] + 32 * 64, c0, c1, c2, u[side][1]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // h = relu(u), dh = d masked by u > 0; lane holds units 32 rt + 8 q + 4 half + i (register 4 q + i)
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            float *ho = (side == 0 ? A.hv : A.hc) + row * H, *dho = (side == 0 ? A.dhv : A.dhc) + row * H;
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float a = u[side][rt][r];
                    u[side][rt][r] = relu_nan(a);
                    d[side][rt][r] = a > 0.0f ? d[side][rt][r] : 0.0f;
                }
                if (ok)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int o0 = 32 * rt + 8 * q + 4 * half;
                        const f32x16 &uu = u[side][rt], &dd = d[side][rt];
                        *reinterpret_cast<float4 *>(ho + o0) = make_float4(uu[4 * q], uu[4 * q + 1], uu[4 * q + 2], uu[4 * q + 3]);
                        *reinterpret_cast<float4 *>(dho + o0) = make_float4(dd[4 * q], dd[4 * q + 1], dd[4 * q + 2], dd[4 * q + 3]);
                    }
            }
        }
        load_rows(rn);
        // GEMM3' of both sides into one tile pair: dz_c[k][msg]
        f32x16 z0 = {}, z1 = {};
#pragma unroll
        for (int side = 0; side < 2; ++side)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                float hv[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) hv[i] = d[side][s >> 1][8 * (s & 1) + i];
                bf16x8_t r0, r1, r2;
                split3(hv, r0, r1, r2);
                z0 = mfma6o(G3[side], aoff[s], r0, r1, r2, z0);
                z1 = mfma6o(G3[side], aoff[s] + 32 * 64, r0, r1, r2, z1);
                __builtin_amdgcn_sched_barrier(0);
            }
        if (ok) {
            float *co = A.dco + row * H;
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const f32x16 &cc = rt ? z1 : z0;
                    *reinterpret_cast<float4 *>(co + 32 * rt + 8 * q + 4 * half) =
                        make_float4(cc[4 * q], cc[4 * q + 1], cc[4 * q + 2], cc[4 * q + 3]);
                }
        }
    }
}

// PJ backward: the group part of dz averaged over a group, formed per group --
// Mda[b][g][k] = inv[g] sum_u W1v[u][64 + k] S_v[b][g][u] with S the group sums of dh (Mdb: the
// check side with W1c).  32-row tiles of a side on v_mfma_f32_32x32x2_f32, C[row][k] =
// sum_u S[row][u] W1_right[u][k]: the A fragment of step s is S[row j][32 half + s] (each lane
// reads 128 contiguous bytes of its row), the B fragments W1_right[32 half + s][32 kt + j] stay in
// registers for the whole side.  (A lane-per-unit VALU form with readlane broadcasts ran at
// 1.3 TB/s: half-rate SGPR-operand FMAs.)
__global__ __launch_bounds__(256) void train_group_back_kernel(const float *__restrict__ Sv, const float *__restrict__ Sc,
                                                               const float *__restrict__ w1v, const float *__restrict__ w1c,
                                                               const float *__restrict__ inv_v,
                                                               const float *__restrict__ inv_c, int Gv, int Gc, int64_t B,
                                                               float *__restrict__ Mda, float *__restrict__ Mdb) {
    const int lane = threadIdx.x & 63, j = lane & 31, half = lane >> 5, wave = threadIdx.x >> 6;
    for (int side = 0; side < 2; ++side) {
        const int G = side ? Gc : Gv;
        const int64_t rows = B * G;
        const float *S = side ? Sc : Sv, *inv = side ? inv_c : inv_v, *w1 = side ? w1c : w1v;
        float *out = side ? Mdb : Mda;
        float wr[2][32];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int s = 0; s < 32; ++s) wr[kt][s] = w1[(32 * half + s) * 128 + 64 + 32 * kt + j];
        const TileWalk tw = xcd_tiles((rows + 31) / 32, 4, wave);
        for (int64_t t = tw.first; t < tw.end; t += tw.stride) {
            const int64_t ra = t * 32 + j < rows ? t * 32 + j : rows - 1;
            float a[32];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const float4 v = *reinterpret_cast<const float4 *>(S + ra * 64 + 32 * half + 4 * q);
                a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
            }
            f32x16 c0 = {}, c1 = {};
#pragma unroll
            for (int s = 0; s < 32; ++s) {
                c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], wr[0][s], c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], wr[1][s], c1, 0, 0, 0);
            }
            // register r: row t * 32 + crow(r, half), unit j (+ 32)
            int g0 = (int)((t * 32) % G);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t row = t * 32 + crow_t(r, half);
                int g = g0 + crow_t(r, half);
                while (g >= G) g -= G;
                if (row < rows) {
                    const float iv = inv[g];
                    out[row * 64 + j] = c0[r] * iv;
                    out[row * 64 + 32 + j] = c1[r] * iv;
                }
            }
        }
    }
}

// dc = dco + mean_var(da) + mean_chk(db) -> dco (kept for demb); dx_l = dc (+ dX)
__global__ void train_combine_kernel(float *__restrict__ dco, const float *__restrict__ Mda,
                                     const float *__restrict__ Mdb, const float *__restrict__ dX,
                                     const int32_t *__restrict__ vgroup, const int32_t *__restrict__ cgroup, int H,
                                     int Gv, int Gc, int64_t E, int64_t n, int residual, float *__restrict__ dx_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = i / H;
    const int u = (int)(i - r * H);
    const int64_t b = r / E, m = r - b * E;
    const float dc = (dco[i] + Mda[(b * Gv + vgroup[m]) * H + u]) + Mdb[(b * Gc + cgroup[m]) * H + u];
    dco[i] = dc;
    dx_out[i] = residual ? dc + dX[i] : dc;
}

// same, H % 4 == 0: one float4 of a row per thread (a float4 never crosses a message row);
// identical operation order, so identical results
__global__ void train_combine4_kernel(float4 *__restrict__ dco, const float4 *__restrict__ Mda,
                                      const float4 *__restrict__ Mdb, const float4 *__restrict__ dX,
                                      const int32_t *__restrict__ vgroup, const int32_t *__restrict__ cgroup, int H4,
                                      int Gv, int Gc, int64_t E, int64_t n4, int residual, float4 *__restrict__ dx_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const int64_t r = i / H4;
    const int u = (int)(i - r * H4);
    const int64_t b = r / E, m = r - b * E;
    const float4 c = dco[i], a = Mda[(b * Gv + vgroup[m]) * H4 + u], bb = Mdb[(b * Gc + cgroup[m]) * H4 + u];
    const float4 dc = make_float4((c.x + a.x) + bb.x, (c.y + a.y) + bb.y, (c.z + a.z) + bb.z, (c.w + a.w) + bb.w);
    dco[i] = dc;
    if (residual) {
        const float4 x = dX[i];
        dx_out[i] = make_float4(dc.x + x.x, dc.y + x.y, dc.z + x.z, dc.w + x.w);
    } else {
        dx_out[i] = dc;
    }
}

// The combine step fused with the first pass of the embedding gradients (projected-group backward):
// one thread per (message, unit) walks the frames in order, forms dc as train_combine4_kernel does
// (the same float sequence), writes dx_l and sums dc over the frames (demb's first pass,
// train_colsum_kernel<0>: the same order, so the same sums), and at layer 0 also sum dc * llr
// (train_colsum_kernel<1>).  dc itself is never stored: 2 of the step's 6 passes over (B, E, H).
template <bool L0>
__global__ void train_combine_sum_kernel(const float *__restrict__ dco, const float *__restrict__ Mda,
                                         const float *__restrict__ Mdb, const float *__restrict__ dX,
                                         const int32_t *__restrict__ vgroup, const int32_t *__restrict__ cgroup,
                                         const int32_t *__restrict__ msg_var, const float *__restrict__ llr, int H,
                                         int Gv, int Gc, int N, int64_t E, int64_t B, int residual,
                                         float *__restrict__ dx_out, float *__restrict__ Sdc, float *__restrict__ Sdl) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t EH = E * H;
    if (t >= EH) return;
    const int64_t m = t / H;
    const int u = (int)(t - m * H);
    const int64_t vg = vgroup[m], cg = cgroup[m];
    const int var = L0 ? msg_var[m] : 0;
    float s0 = 0.0f, s1 = 0.0f;
#pragma unroll 4
    for (int64_t b = 0; b < B; ++b) {
        const int64_t i = b * EH + t;
        const float dc = (dco[i] + Mda[(b * Gv + vg) * H + u]) + Mdb[(b * Gc + cg) * H + u];
        dx_out[i] = residual ? dc + dX[i] : dc;
        s0 += dc;
        if (L0) s1 = fmaf(dc, llr[b * N + var], s1);
    }
    Sdc[t] = s0;
    if (L0) Sdl[t] = s1;
}

// ------------------------------------------------------------------------ weight gradients
// out[i][j] += sum_r A[r][i] Z_r[j] (i < H, j < J), bias[i] += sum_r A[r][i];
// Z_r = zsrc[r] (J = H), or [zsrc[r]; G[b][grp(m)]] (J = 2H, the concatenated MLP input)
struct OuterT {
    const float *A, *zsrc, *G;
    const int32_t *grp;
    float *out, *bias;
    int H, J, Gn;
    int ld = 0, col0 = 0;  // out[i * ld + col0 + j] (ld 0 = J): one half of a [H][2H] gradient
    int64_t E, R;
    // one output tile (H > 64 or J > 128, see launch_outer): rows i0 .. i0 + ni of the gradient,
    // columns j0 .. j0 + nj of Z (ni / nj 0: all H / J)
    int i0 = 0, j0 = 0, ni = 0, nj = 0;
};
constexpr int kRB = 16;  // rows staged per step

__global__ __launch_bounds__(256) void train_outer_kernel(OuterT P) {
    __shared__ float As[kRB][kMaxH];
    __shared__ float Zs[kRB][2 * kMaxH];
    const int t = threadIdx.x, i = t >> 2, jq = t & 3;
    const int H = P.H, J = P.J, JW = J / 4;
    float acc[32], bacc = 0.0f;
#pragma unroll
    for (int k = 0; k < 32; ++k) acc[k] = 0.0f;
    const int64_t per = (P.R + gridDim.x - 1) / gridDim.x;
    const int64_t r_begin = (int64_t)blockIdx.x * per, r_end = r_begin + per < P.R ? r_begin + per : P.R;
    for (int64_t r0 = r_begin; r0 < r_end; r0 += kRB) {
        for (int e = t; e < kRB * H; e += 256) {
            const int rr = e / H, k = e - rr * H;
            const int64_t r = r0 + rr;
            As[rr][k] = r < r_end ? P.A[r * H + k] : 0.0f;
        }
        for (int e = t; e < kRB * J; e += 256) {
            const int rr = e / J, k = e - rr * J;
            const int64_t r = r0 + rr;
            float v = 0.0f;
            if (r < r_end) {
                if (k < H) {
                    v = P.zsrc[r * H + k];
                } else {
                    const int64_t b = r / P.E, m = r - b * P.E;
                    v = P.G[(b * P.Gn + P.grp[m]) * H + (k - H)];
                }
            }
            Zs[rr][k] = v;
        }
        __syncthreads();
        if (i < H) {
            for (int rr = 0; rr < kRB; ++rr) {
                const float a = As[rr][i];
                bacc += a;
#pragma unroll
                for (int k = 0; k < 32; ++k)
                    if (k < JW) acc[k] = fmaf(a, Zs[rr][jq * JW + k], acc[k]);
            }
        }
        __syncthreads();
    }
    if (i < H) {
#pragma unroll
        for (int k = 0; k < 32; ++k)
            if (k < JW) atomicAdd(&P.out[i * (P.ld ? P.ld : J) + P.col0 + jq * JW + k], acc[k]);
        if (jq == 0 && P.bias) atomicAdd(&P.bias[i], bacc);
    }
}

// Same reduction on fp32 MFMA: dW (i < H, j < J) = A^T Z with the rows as the K dimension.
// v_mfma_f32_32x32x2_f32 takes K = 2 rows per instruction; its A fragment (lane l: row i = l & 31
// of the 32 x 2 block, k = l >> 5) is A[r0 + k][32 it + i] and its B fragment is
// Z[r0 + k][32 jt + (l & 31)] -- both straight from global memory, two 128-B row segments per
// load, no LDS.  Every wave owns a contiguous range of rows and keeps the whole (up to) 64 x 128
// tile in 8 accumulators; at the end it adds them into the gradient with float atomics (a 32 x 32
// accumulator register is two 128-B row segments: the full-rate atomic shape).
typedef float f32x16 __attribute__((ext_vector_type(16)));


// H64: H = J = 64 from zsrc: no per-load bounds or source checks, software-pipelined
template <int NIT, int NJT, bool H64 = false>
__global__ __launch_bounds__(256) void train_outer_mfma_kernel(OuterT P) {
    const int lane = threadIdx.x & 63, col = lane & 31, k = lane >> 5;
    const int H = H64 ? 64 : P.H, J = H64 ? 32 * NJT : P.J;
    const int NI = H64 ? 64 : P.ni ? P.ni : H, NJ = H64 ? J : P.nj ? P.nj : J;  // this tile's extent
    const int i0 = H64 ? 0 : P.i0, j0 = H64 ? 0 : P.j0;
    const int64_t nw = (int64_t)gridDim.x * 4, w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t per = ((P.R + nw - 1) / nw + 1) & ~1LL;  // even: whole k-steps
    const int64_t r_begin = w * per, r_end = r_begin + per < P.R ? r_begin + per : P.R;
    f32x16 acc[NIT][NJT];
#pragma unroll
    for (int it = 0; it < NIT; ++it)
#pragma unroll
        for (int jt = 0; jt < NJT; ++jt) acc[it][jt] = f32x16{};
    float bsum[NIT] = {};
    auto zval = [&](int64_t r, int64_t b, int64_t m, int j) -> float {
        if constexpr (H64) return P.zsrc[r * 64 + j];
        if (j >= NJ) return 0.0f;
        j += j0;
        if (j < H) return P.zsrc[r * H + j];
        return P.G[(b * P.Gn + P.grp[m]) * H + (j - H)];
    };
    // (frame, message) of row r0 + k, stepped along with r0 (no 64-bit division per row)
    int64_t bb = (r_begin + k) / P.E, mm = r_begin + k - bb * P.E;
    // KU k-steps (2 KU rows) of fragments are loaded before their MFMAs, so each wave keeps
    // 2 KU (NIT + NJT) independent loads in flight instead of waiting on one k-step at a time
    constexpr int KU = 8;
    struct Batch { float a[KU][NIT], z[KU][NJT]; };
    auto load_batch = [&](int64_t r0, Batch &B) {
#pragma unroll
        for (int u = 0; u < KU; ++u) {
            const int64_t r = r0 + 2 * u + k;
            const bool ok = r < r_end;
            int64_t bu = bb, mu = mm + 2 * u;
            if constexpr (!H64)
                while (mu >= P.E) { mu -= P.E; ++bu; }
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int i = 32 * it + col;
                B.a[u][it] = ok && (H64 || i < NI) ? P.A[r * H + i0 + i] : 0.0f;
            }
#pragma unroll
            for (int jt = 0; jt < NJT; ++jt) B.z[u][jt] = ok ? zval(r, bu, mu, 32 * jt + col) : 0.0f;
        }
        if constexpr (!H64) {
            mm += 2 * KU;
            while (mm >= P.E) { mm -= P.E; ++bb; }
        }
    };
    auto mfma_batch = [&](const Batch &B) {
#pragma unroll
        for (int u = 0; u < KU; ++u)
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                bsum[it] += B.a[u][it];
#pragma unroll
                for (int jt = 0; jt < NJT; ++jt)
                    acc[it][jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(B.a[u][it], B.z[u][jt], acc[it][jt], 0, 0, 0);
            }
    };
    if constexpr (H64) {
        // software-pipelined: the next batch's rows load while this batch's MFMAs run.  Branch-free
        // loads (rows clamped to the range, the rows past it zeroed at use) and two batch buffers
        // used alternately: a load under a branch, or a batch copied register to register, makes
        // the compiler wait for the next batch's loads before this batch's MFMAs.
        if (r_begin < r_end) {
            const int64_t rlast = r_end - 1;
            auto load_h = [&](int64_t r0, Batch &B) {
#pragma unroll
                for (int u = 0; u < KU; ++u) {
                    const int64_t r = r0 + 2 * u + k < rlast ? r0 + 2 * u + k : rlast;
#pragma unroll
                    for (int it = 0; it < NIT; ++it) B.a[u][it] = P.A[r * 64 + 32 * it + col];
#pragma unroll
                    for (int jt = 0; jt < NJT; ++jt) B.z[u][jt] = zval(r, 0, 0, 32 * jt + col);
                }
            };
            auto mfma_h = [&](int64_t r0, const Batch &B) {
#pragma unroll
                for (int u = 0; u < KU; ++u) {
                    const bool ok = r0 + 2 * u + k < r_end;
#pragma unroll
                    for (int it = 0; it < NIT; ++it) {
                        const float a = ok ? B.a[u][it] : 0.0f;
                        bsum[it] += a;
#pragma unroll
                        for (int jt = 0; jt < NJT; ++jt)
                            acc[it][jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, B.z[u][jt], acc[it][jt], 0, 0, 0);
                    }
                }
            };
            Batch b0, b1;
            load_h(r_begin, b0);
            // (sched_barrier: the scheduler would otherwise sink each load next to its first use)
            for (int64_t r0 = r_begin;;) {
                load_h(r0 + 2 * KU, b1);
                __builtin_amdgcn_sched_barrier(0);
                mfma_h(r0, b0);
                if ((r0 += 2 * KU) >= r_end) break;
                load_h(r0 + 2 * KU, b0);
                __builtin_amdgcn_sched_barrier(0);
                mfma_h(r0, b1);
                if ((r0 += 2 * KU) >= r_end) break;
            }
        }
    } else {
        for (int64_t r0 = r_begin; r0 < r_end; r0 += 2 * KU) {
            Batch cur;
            load_batch(r0, cur);
            mfma_batch(cur);
        }
    }
    // D[i][j]: register q of lane l holds i = 8 (q >> 2) + 4 k + (q & 3), j = col.  The four waves'
    // tiles are summed in LDS first, so each workgroup issues one global atomic per gradient entry
    // (per-wave atomics put thousands of adds on every address).
    __shared__ float red[NIT * 32 * NJT * 32], bred[NIT * 32];
    for (int e = threadIdx.x; e < NIT * 32 * NJT * 32; e += 256) red[e] = 0.0f;
    if (threadIdx.x < NIT * 32) bred[threadIdx.x] = 0.0f;
    __syncthreads();
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
#pragma unroll
        for (int jt = 0; jt < NJT; ++jt)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int i = 32 * it + 8 * (q >> 2) + 4 * k + (q & 3);
                atomicAdd(&red[i * (NJT * 32) + 32 * jt + col], acc[it][jt][q]);
            }
        const float s = bsum[it] + __shfl_xor(bsum[it], 32, 64);
        if (k == 0) atomicAdd(&bred[32 * it + col], s);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < NIT * 32 * NJT * 32; e += 256) {
        const int i = e / (NJT * 32), j = e - i * (NJT * 32);
        if (i < NI && j < NJ) {
            atomicAdd(&P.out[(i0 + i) * (P.ld ? P.ld : J) + P.col0 + j0 + j], red[e]);
        }
    }
    if (P.bias && threadIdx.x < NI) atomicAdd(&P.bias[i0 + threadIdx.x], bred[threadIdx.x]);
}

// dW1_left of both sides in one pass over the rows (H = 64, projected-group backward):
//   gw1s[i][j] += sum_r dh_s[r][i] c_r[j],  gb1s[i] += sum_r dh_s[r][i]   (s = v, c; j < 64)
// with c_r = x_r + emb[type(m)] (ZM 1; x = the saved features of the layer's input) or
// (w_in llr + b_in) + emb[type(m)] (ZM 2, layer 0) formed here in the MLP backward's float order
// (the same c, bit for bit), so the backward MLP writes no copy of c and c is read once for both
// sides.  Layout and pipelining as train_outer_mfma_kernel<2, 2, true>: lane (col, k) loads rows
// r0 + 2u + k, batches of KU k-steps double-buffered, the type embedding in LDS.
struct Dw1T {
    const float *dhv, *dhc, *x, *emb, *llr, *w_in, *b_in;
    const int32_t *msg_type, *msg_var;
    float *gv, *gc, *bv, *bc;
    int T, N;
    int64_t E, R;
};
inline size_t dw1_lds(int T) { return (size_t)std::max(T * 64, 2 * 64 * 64 + 2 * 64) * 4; }

template <int ZM>
__global__ __launch_bounds__(256, 2) void train_dw1_kernel(Dw1T P) {
    extern __shared__ __attribute__((aligned(16))) float sh[];
    for (int i = threadIdx.x; i < P.T * 64; i += 256) sh[i] = P.emb[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, col = lane & 31, k = lane >> 5;
    const int64_t nw = (int64_t)gridDim.x * 4, w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t per = ((P.R + nw - 1) / nw + 1) & ~1LL;
    const int64_t r_begin = w * per, r_end = r_begin + per < P.R ? r_begin + per : P.R;
    f32x16 acc[2][2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
            for (int jt = 0; jt < 2; ++jt) acc[s][it][jt] = f32x16{};
    float bsum[2][2] = {};
    float win[2] = {}, bin[2] = {};
    if (ZM == 2)
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            win[jt] = P.w_in[32 * jt + col];
            bin[jt] = P.b_in[32 * jt + col];
        }
    constexpr int KU = 4;
    struct Batch { float a[KU][2][2], z[KU][2], l[KU]; int ty[KU]; };
    if (r_begin < r_end) {
        const int64_t rlast = r_end - 1;
        int64_t bq = r_begin / P.E, mq = r_begin - bq * P.E;  // (frame, message) of the batch's first row
        const int64_t bl = rlast / P.E, ml = rlast - bl * P.E;  // ... and of the range's last row
        auto load = [&](int64_t r0, int64_t b0, int64_t m0, Batch &Bt) {
#pragma unroll
            for (int u = 0; u < KU; ++u) {
                // rows past the range read the last row (their A values are zeroed at use)
                const bool in = r0 + 2 * u + k <= rlast;
                const int64_t r = in ? r0 + 2 * u + k : rlast;
                int64_t mu = m0 + 2 * u + k, bu = b0;
                if (mu >= P.E) { mu -= P.E; ++bu; }
                mu = in ? mu : ml;
                bu = in ? bu : bl;
#pragma unroll
                for (int it = 0; it < 2; ++it) {
                    Bt.a[u][0][it] = P.dhv[r * 64 + 32 * it + col];
                    Bt.a[u][1][it] = P.dhc[r * 64 + 32 * it + col];
                }
                Bt.ty[u] = P.msg_type[mu];
                if (ZM == 1) {
#pragma unroll
                    for (int jt = 0; jt < 2; ++jt) Bt.z[u][jt] = P.x[r * 64 + 32 * jt + col];
                } else {
                    Bt.l[u] = P.llr[bu * P.N + P.msg_var[mu]];
                }
            }
        };
        auto mfma = [&](int64_t r0, const Batch &Bt) {
#pragma unroll
            for (int u = 0; u < KU; ++u) {
                const bool ok = r0 + 2 * u + k < r_end;
                float z[2];
#pragma unroll
                for (int jt = 0; jt < 2; ++jt) {
                    const float xv = ZM == 1 ? Bt.z[u][jt] : win[jt] * Bt.l[u] + bin[jt];
                    z[jt] = xv + sh[Bt.ty[u] * 64 + 32 * jt + col];
                }
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int it = 0; it < 2; ++it) {
                        const float a = ok ? Bt.a[u][s][it] : 0.0f;
                        bsum[s][it] += a;
#pragma unroll
                        for (int jt = 0; jt < 2; ++jt)
                            acc[s][it][jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, z[jt], acc[s][it][jt], 0, 0, 0);
                    }
            }
        };
        auto step = [&]() {
            mq += 2 * KU;
            if (mq >= P.E) { mq -= P.E; ++bq; }
        };
        Batch b0, b1;
        load(r_begin, bq, mq, b0);
        for (int64_t r0 = r_begin;;) {
            int64_t nb = bq, nm = mq + 2 * KU;
            if (nm >= P.E) { nm -= P.E; ++nb; }
            load(r0 + 2 * KU, nb, nm, b1);
            __builtin_amdgcn_sched_barrier(0);
            mfma(r0, b0);
            step();
            if ((r0 += 2 * KU) >= r_end) break;
            nb = bq; nm = mq + 2 * KU;
            if (nm >= P.E) { nm -= P.E; ++nb; }
            load(r0 + 2 * KU, nb, nm, b0);
            __builtin_amdgcn_sched_barrier(0);
            mfma(r0, b1);
            step();
            if ((r0 += 2 * KU) >= r_end) break;
        }
    }
    // the four waves' tiles summed in LDS (the embedding image is no longer read), then one
    // global atomic per gradient entry per workgroup; D[i][j]: register q of lane (col, k) holds
    // i = 8 (q >> 2) + 4 k + (q & 3), j = col
    __syncthreads();
    float *red = sh, *bred = sh + 2 * 64 * 64;
    for (int e = threadIdx.x; e < 2 * 64 * 64 + 2 * 64; e += 256) sh[e] = 0.0f;
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int it = 0; it < 2; ++it) {
#pragma unroll
            for (int jt = 0; jt < 2; ++jt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int i = 32 * it + 8 * (q >> 2) + 4 * k + (q & 3);
                    atomicAdd(&red[s * 4096 + i * 64 + 32 * jt + col], acc[s][it][jt][q]);
                }
            const float sm = bsum[s][it] + __shfl_xor(bsum[s][it], 32, 64);
            if (k == 0) atomicAdd(&bred[s * 64 + 32 * it + col], sm);
        }
    __syncthreads();
    for (int e = threadIdx.x; e < 2 * 4096; e += 256) {
        const int s = e >> 12, i = (e >> 6) & 63, j = e & 63;
        atomicAdd(&(s ? P.gc : P.gv)[i * 128 + j], red[e]);
    }
    if (threadIdx.x < 128) {
        const int s = threadIdx.x >> 6, i = threadIdx.x & 63;
        atomicAdd(&(s ? P.bc : P.bv)[i], bred[threadIdx.x]);
    }
}

// dW2 of both sides in one pass over dX (H = 64): gw2s[i][j] += sum_r dX[r][i] h_s[r][j],
// gb2s[i] += sum_r dX[r][i] (the same bias sums for both sides); h_v = hv, h_c = hc.  The layout
// and pipelining of train_dw1_kernel, with one A and two Z sources; dX is read once instead of
// twice.
struct Dw2T {
    const float *dX, *hv, *hc;
    float *gv, *gc, *bv, *bc;
    int64_t R;
};

__global__ __launch_bounds__(256, 2) void train_dw2_kernel(Dw2T P) {
    __shared__ __attribute__((aligned(16))) float sh[2 * 64 * 64 + 64];
    const int lane = threadIdx.x & 63, col = lane & 31, k = lane >> 5;
    const int64_t nw = (int64_t)gridDim.x * 4, w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t per = ((P.R + nw - 1) / nw + 1) & ~1LL;
    const int64_t r_begin = w * per, r_end = r_begin + per < P.R ? r_begin + per : P.R;
    f32x16 acc[2][2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
            for (int jt = 0; jt < 2; ++jt) acc[s][it][jt] = f32x16{};
    float bsum[2] = {};
    constexpr int KU = 4;
    struct Batch { float a[KU][2], z[KU][2][2]; };
    if (r_begin < r_end) {
        const int64_t rlast = r_end - 1;
        auto load = [&](int64_t r0, Batch &Bt) {
#pragma unroll
            for (int u = 0; u < KU; ++u) {
                const int64_t r = r0 + 2 * u + k <= rlast ? r0 + 2 * u + k : rlast;
#pragma unroll
                for (int it = 0; it < 2; ++it) Bt.a[u][it] = P.dX[r * 64 + 32 * it + col];
#pragma unroll
                for (int jt = 0; jt < 2; ++jt) {
                    Bt.z[u][0][jt] = P.hv[r * 64 + 32 * jt + col];
                    Bt.z[u][1][jt] = P.hc[r * 64 + 32 * jt + col];
                }
            }
        };
        auto mfma = [&](int64_t r0, const Batch &Bt) {
#pragma unroll
            for (int u = 0; u < KU; ++u) {
                const bool ok = r0 + 2 * u + k < r_end;
#pragma unroll
                for (int it = 0; it < 2; ++it) {
                    const float a = ok ? Bt.a[u][it] : 0.0f;
                    bsum[it] += a;
#pragma unroll
                    for (int s = 0; s < 2; ++s)
#pragma unroll
                        for (int jt = 0; jt < 2; ++jt)
                            acc[s][it][jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Bt.z[u][s][jt], acc[s][it][jt], 0, 0, 0);
                }
            }
        };
        Batch b0, b1;
        load(r_begin, b0);
        for (int64_t r0 = r_begin;;) {
            load(r0 + 2 * KU, b1);
            __builtin_amdgcn_sched_barrier(0);
            mfma(r0, b0);
            if ((r0 += 2 * KU) >= r_end) break;
            load(r0 + 2 * KU, b0);
            __builtin_amdgcn_sched_barrier(0);
            mfma(r0, b1);
            if ((r0 += 2 * KU) >= r_end) break;
        }
    }
    float *red = sh, *bred = sh + 2 * 64 * 64;
    for (int e = threadIdx.x; e < 2 * 64 * 64 + 64; e += 256) sh[e] = 0.0f;
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 2; ++it) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int jt = 0; jt < 2; ++jt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int i = 32 * it + 8 * (q >> 2) + 4 * k + (q & 3);
                    atomicAdd(&red[s * 4096 + i * 64 + 32 * jt + col], acc[s][it][jt][q]);
                }
        const float sm = bsum[it] + __shfl_xor(bsum[it], 32, 64);
        if (k == 0) atomicAdd(&bred[32 * it + col], sm);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 2 * 4096; e += 256) atomicAdd(&((e >> 12) ? P.gc : P.gv)[e & 4095], red[e]);
    if (threadIdx.x < 64) {
        atomicAdd(&P.bv[threadIdx.x], bred[threadIdx.x]);
        atomicAdd(&P.bc[threadIdx.x], bred[threadIdx.x]);
    }
}

// workgroups per CU of the weight-gradient reductions: 1 (4 waves per CU).  Each wave ends with a
// 64 x 64 (x 2) block of float atomics into the gradient; fewer waves, fewer atomics: 30.5-30.7 ms
// per step against 32.8 at 2 workgroups per CU and 32.2-32.7 at 3 (round 5, profiles/r05/ab_r05o;
// round 4 had measured 2 best among 2, 4 and 8)
constexpr int kOuterWgs = 1;

int launch_outer(const OuterT &o, unsigned grid, hipStream_t s) {
    if (o.H > 64 || o.J > 128) {  // tiles of 64 gradient rows x 128 Z columns, one launch each
        for (int i0 = 0; i0 < o.H; i0 += 64)
            for (int j0 = 0; j0 < o.J; j0 += 128) {
                OuterT t = o;
                t.i0 = i0; t.ni = std::min(64, o.H - i0);
                t.j0 = j0; t.nj = std::min(128, o.J - j0);
                if (j0) t.bias = nullptr;  // the bias sums once per gradient row
                const int nit = (t.ni + 31) / 32, njt = (t.nj + 31) / 32;
                if (nit == 2 && njt == 4) hipLaunchKernelGGL((train_outer_mfma_kernel<2, 4>), dim3(grid), dim3(256), 0, s, t);
                else if (nit == 2 && njt == 3) hipLaunchKernelGGL((train_outer_mfma_kernel<2, 3>), dim3(grid), dim3(256), 0, s, t);
                else if (nit == 2 && njt == 2) hipLaunchKernelGGL((train_outer_mfma_kernel<2, 2>), dim3(grid), dim3(256), 0, s, t);
                else if (nit == 2) hipLaunchKernelGGL((train_outer_mfma_kernel<2, 1>), dim3(grid), dim3(256), 0, s, t);
                else if (njt == 4) hipLaunchKernelGGL((train_outer_mfma_kernel<1, 4>), dim3(grid), dim3(256), 0, s, t);
                else if (njt == 3) hipLaunchKernelGGL((train_outer_mfma_kernel<1, 3>), dim3(grid), dim3(256), 0, s, t);
                else if (njt == 2) hipLaunchKernelGGL((train_outer_mfma_kernel<1, 2>), dim3(grid), dim3(256), 0, s, t);
                else hipLaunchKernelGGL((train_outer_mfma_kernel<1, 1>), dim3(grid), dim3(256), 0, s, t);
                LDPC_CHECK_LAUNCH("train_outer_mfma_kernel (tile)");
            }
        return LDPC_OK;
    }
    const int nit = (o.H + 31) / 32, njt = (o.J + 31) / 32;
    // H = 64 from plain row sources: the specialised kernels (no per-load source / bounds checks)
    const bool h64 = o.H == 64 && !o.G && o.J == 64;
    if (h64 && njt == 2) hipLaunchKernelGGL((train_outer_mfma_kernel<2, 2, true>), dim3(grid), dim3(256), 0, s, o);
    else if (nit == 2 && njt == 4) hipLaunchKernelGGL((train_outer_mfma_kernel<2, 4>), dim3(grid), dim3(256), 0, s, o);
    else if (nit == 2 && njt == 2) hipLaunchKernelGGL((train_outer_mfma_kernel<2, 2>), dim3(grid), dim3(256), 0, s, o);
    else if (nit == 1 && njt == 2) hipLaunchKernelGGL((train_outer_mfma_kernel<1, 2>), dim3(grid), dim3(256), 0, s, o);
    else if (nit == 1 && njt == 1) hipLaunchKernelGGL((train_outer_mfma_kernel<1, 1>), dim3(grid), dim3(256), 0, s, o);
    else hipLaunchKernelGGL(train_outer_kernel, dim3(grid), dim3(256), 0, s, o);
    LDPC_CHECK_LAUNCH("train_outer_kernel");
    return LDPC_OK;
}

// per-row vector gradients, lanes = units:
//   mode 0 (emb):  demb[type(m)][u] += src[r][u]
//   mode 1 (input embedding, layer 0): dw_in[u] += src[r][u] llr[b][var(m)], db_in[u] += src[r][u]
//   mode 2 (head): dwo[u] += dz[b][var(m)] src[r][u], dbo += dz[b][var(m)]
struct VecT {
    const float *src, *llr, *dz;
    const int32_t *msg_type, *msg_var;
    float *g0, *g1;  // mode 0: demb; 1: dw_in, db_in; 2: dwo, dbo
    int H, T, N, mode;
    int64_t E, R;
    float *part = nullptr;  // per-workgroup partial sums (scratch), capacity part_cap floats
    int64_t part_cap = 0;
};

// The same three reductions in two coalesced passes: first over the frames, per (message, unit)
// -- consecutive threads read consecutive words of each frame's (E, H) slab --, then over the
// messages into the gradient (a row walk with a per-type LDS accumulation ran at ~0.8 TB/s).
// The frame loop keeps the sequential order (one sum per thread), unrolled so that eight frames'
// loads are in flight.
template <int MODE>
__global__ void train_colsum_kernel(VecT P, float *__restrict__ S0, float *__restrict__ S1) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t EH = P.E * P.H;
    if (t >= EH) return;
    const int64_t m = t / P.H;
    const int64_t B = P.R / P.E;
    float s0 = 0.0f, s1 = 0.0f;
    const int var = MODE != 0 ? P.msg_var[m] : 0;
    const float *src = P.src + t;
#pragma unroll 8
    for (int64_t b = 0; b < B; ++b) {
        const float v = src[b * EH];
        if constexpr (MODE == 0) {
            s0 += v;
        } else if constexpr (MODE == 1) {
            s0 = fmaf(v, P.llr[b * P.N + var], s0);
            s1 += v;
        } else {
            const float d = P.dz[b * P.N + var];
            s0 = fmaf(d, v, s0);
            s1 += d;
        }
    }
    S0[t] = s0;
    if constexpr (MODE != 0) S1[t] = s1;
}

// Second pass: a workgroup of 4 waves per kChunkV messages (wave w takes every fourth, lanes =
// units).  Mode 0 sums per type in LDS (ds_add); modes 1 / 2 sum per lane, then over the waves in
// LDS.  Each workgroup then writes its partial vector to scratch and train_vecreduce_kernel sums
// the workgroups per entry, one global add each.  (Float atomics into the gradient from every
// workgroup serialise per cache line at L2: 0.17 ms per call whatever the workgroup count.)
constexpr int kChunkV = 64;
inline size_t vecfinal_lds(int T, int H) { return (size_t)std::max(T * H, 2 * 4 * H) * 4; }

template <int MODE>
__global__ __launch_bounds__(256) void train_vecfinal_kernel(VecT P, const float *__restrict__ S0,
                                                             const float *__restrict__ S1) {
    extern __shared__ float acc[];
    const int w = threadIdx.x >> 6;
    const int n = MODE == 0 ? P.T * P.H : 2 * 4 * P.H;
    for (int i = threadIdx.x; i < n; i += 256) acc[i] = 0.0f;
    __syncthreads();
    const int64_t m0 = (int64_t)blockIdx.x * kChunkV, m1 = min<int64_t>(m0 + kChunkV, P.E);
    for (int u = threadIdx.x & 63; u < P.H; u += 64) {  // lanes = units (and + 64, ... past 64)
        float a0 = 0.0f, a1 = 0.0f;
#pragma unroll 8
        for (int64_t m = m0 + w; m < m1; m += 4) {
            const float v = S0[m * P.H + u];
            if constexpr (MODE == 0) {
                atomicAdd(&acc[P.msg_type[m] * P.H + u], v);
            } else {
                a0 += v;
                a1 += S1[m * P.H + u];
            }
        }
        if constexpr (MODE != 0) {
            acc[w * P.H + u] = a0;
            acc[(4 + w) * P.H + u] = a1;
        }
    }
    __syncthreads();
    const bool part = P.part != nullptr;  // else (scratch too small) straight into the gradient
    if constexpr (MODE == 0) {
        for (int i = threadIdx.x; i < n; i += 256) {
            if (part) P.part[(int64_t)blockIdx.x * n + i] = acc[i];
            else if (acc[i] != 0.0f) atomicAdd(&P.g0[i], acc[i]);
        }
    } else if (w == 0) {
      for (int u = threadIdx.x; u < P.H; u += 64) {
        const float s0 = ((acc[u] + acc[P.H + u]) + acc[2 * P.H + u]) + acc[3 * P.H + u];
        const float s1 = ((acc[4 * P.H + u] + acc[5 * P.H + u]) + acc[6 * P.H + u]) + acc[7 * P.H + u];
        if (part) {
            P.part[(int64_t)blockIdx.x * 2 * P.H + u] = s0;
            P.part[(int64_t)blockIdx.x * 2 * P.H + P.H + u] = s1;
        } else {
            atomicAdd(&P.g0[u], s0);
            if (MODE == 1) atomicAdd(&P.g1[u], s1);
            else if (u == 0) atomicAdd(&P.g1[0], s1);  // dbo: S1 is the same for every unit
        }
      }
    }
}

// sum of the workgroups' partial vectors per entry (ascending workgroups), into the gradient
template <int MODE>
__global__ void train_vecreduce_kernel(VecT P, int nblk) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = MODE == 0 ? P.T * P.H : 2 * P.H;
    if (i >= n) return;
    float s = 0.0f;
    for (int b = 0; b < nblk; ++b) s += P.part[(int64_t)b * n + i];
    if (MODE == 0) atomicAdd(&P.g0[i], s);
    else if (i < P.H) atomicAdd(&P.g0[i], s);
    else if (MODE == 1) atomicAdd(&P.g1[i - P.H], s);
    else if (i == P.H) atomicAdd(&P.g1[0], s);  // dbo: S1 is the same for every unit
}

// the second pass alone, from frame sums S0 (and S1) formed elsewhere
int launch_vecfinal(const VecT &v0, const float *S0, const float *S1, hipStream_t s) {
    const int nblk = (int)((v0.E + kChunkV - 1) / kChunkV);
    const dim3 g2((unsigned)nblk);
    const size_t lds = vecfinal_lds(v0.T, v0.H);
    if (lds > 160 * 1024) return fail(LDPC_EUNSUPPORTED, "too many message types for the embedding gradient");
    if (lds > 64 * 1024) {
        LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(train_vecfinal_kernel<0>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(train_vecfinal_kernel<1>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(train_vecfinal_kernel<2>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    }
    const int n = v0.mode == 0 ? v0.T * v0.H : 2 * v0.H;
    VecT v = v0;
    if ((int64_t)nblk * n > v.part_cap) v.part = nullptr;
    if (v.mode == 0)
        hipLaunchKernelGGL(train_vecfinal_kernel<0>, g2, dim3(256), lds, s, v, S0, S1);
    else if (v.mode == 1)
        hipLaunchKernelGGL(train_vecfinal_kernel<1>, g2, dim3(256), lds, s, v, S0, S1);
    else
        hipLaunchKernelGGL(train_vecfinal_kernel<2>, g2, dim3(256), lds, s, v, S0, S1);
    LDPC_CHECK_LAUNCH("train_vecfinal_kernel");
    if (v.part) {
        const dim3 gr((unsigned)((n + 255) / 256));
        if (v.mode == 0) hipLaunchKernelGGL(train_vecreduce_kernel<0>, gr, dim3(256), 0, s, v, nblk);
        else if (v.mode == 1) hipLaunchKernelGGL(train_vecreduce_kernel<1>, gr, dim3(256), 0, s, v, nblk);
        else hipLaunchKernelGGL(train_vecreduce_kernel<2>, gr, dim3(256), 0, s, v, nblk);
        LDPC_CHECK_LAUNCH("train_vecreduce_kernel");
    }
    return LDPC_OK;
}

int launch_vec(const VecT &v, float *S0, float *S1, hipStream_t s) {
    const int64_t EH = v.E * v.H;
    const dim3 g1((unsigned)((EH + 255) / 256)), g2((unsigned)((v.E + kChunkV - 1) / kChunkV));
    (void)g2;
    if (v.mode == 0)
        hipLaunchKernelGGL(train_colsum_kernel<0>, g1, dim3(256), 0, s, v, S0, S1);
    else if (v.mode == 1)
        hipLaunchKernelGGL(train_colsum_kernel<1>, g1, dim3(256), 0, s, v, S0, S1);
    else
        hipLaunchKernelGGL(train_colsum_kernel<2>, g1, dim3(256), 0, s, v, S0, S1);
    LDPC_CHECK_LAUNCH("train_colsum_kernel");
    return launch_vecfinal(v, S0, S1, s);
}


struct TrainWs {
    float *Mv, *Mc, *dz, *dX, *dXp, *cbuf, *hv, *hc, *dhv, *dhc, *dco, *da, *db, *Mda, *Mdb;
    float *Mv1, *Mc1, *Gs1v, *Gs1c;  // second projection set (odd layers) for the side-stream recompute
    int64_t bytes;
};

TrainWs carve_train(const ldpc_gnn_plan *p, int H, int N, int64_t B, void *base) {
    auto al = [](int64_t x) { return (x + 63) / 64 * 64; };  // floats (256-B alignment)
    const int64_t reh = al(B * p->E * H), mv = al(B * p->Gv * H), mc = al(B * p->Gc * H), nz = al(B * N);
    float *c = static_cast<float *>(base);
    TrainWs w;
    int64_t o = 0;
    auto take = [&](int64_t n) { float *q = c + o; o += n; return q; };
    w.Mv = take(mv);
    w.Mc = take(mc);
    w.Mda = take(mv);
    w.Mdb = take(mc);
    w.dz = take(nz);
    w.dX = take(reh);
    w.dXp = take(reh);
    w.cbuf = take(reh);
    w.hv = take(reh);
    w.hc = take(reh);
    w.dhv = take(reh);
    w.dhc = take(reh);
    w.dco = take(reh);
    w.da = take(reh);
    w.db = take(reh);
    w.Mv1 = take(mv);
    w.Mc1 = take(mc);
    w.Gs1v = take(mv);
    w.Gs1c = take(mc);
    w.bytes = o * 4;
    return w;
}

int g_cus_t = 0;

// per-device, per-thread events of the backward's side-stream recompute (see bwd_overlap)
int train_events(hipEvent_t ready[2], hipEvent_t freed[2]) {
    constexpr int kMaxDev = 64;
    thread_local hipEvent_t ev[kMaxDev][4];
    int dev = 0;
    LDPC_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDev) return fail(LDPC_EUNSUPPORTED, "device index out of range");
    for (int i = 0; i < 4; ++i)
        if (!ev[dev][i]) LDPC_HIP(hipEventCreateWithFlags(&ev[dev][i], hipEventDisableTiming));
    ready[0] = ev[dev][0]; ready[1] = ev[dev][1]; freed[0] = ev[dev][2]; freed[1] = ev[dev][3];
    return LDPC_OK;
}

// LDPC_GNN_TRAIN_PROJ=0: the backward recomputes group means and runs GEMM1 / GEMM3' over
// [c; g] per message (A/B); default: projected group rows (train_mlp_bwd_mfma_kernel PJ)
int bwd_proj() {
    const char *e = std::getenv("LDPC_GNN_TRAIN_PROJ");  // read per call (tests toggle it)
    return e ? std::atoi(e) : 1;
}

// LDPC_GNN_TRAIN_S6=0: the projected-group backward MLP on fp32 MFMA (train_mlp_bwd_mfma_kernel)
// instead of bf16x6 splits (train_mlp_bwd_s6_kernel); read per call (A/B runs, tests)
int bwd_s6() {
    const char *e = std::getenv("LDPC_GNN_TRAIN_S6");
    return e ? std::atoi(e) : 1;
}
// LDPC_GNN_TRAIN_OVERLAP=1: the backward's forward recompute (group projections of layer l - 1)
// runs on a side stream into a second buffer set while layer l's gradients run on the caller's
// stream; 0: one set, in line.  42.3-42.5 vs 42.7-43.0 ms per B = 256 step (profiles/r03aj, three
// pairs on one box): the projection mostly competes with the gradient kernels for the CUs.
// Read per call.
int bwd_overlap() {
    const char *e = std::getenv("LDPC_GNN_TRAIN_OVERLAP");
    return e ? std::atoi(e) : 1;
}


}  // namespace
}  // namespace ldpc

using namespace ldpc;

extern "C" int64_t ldpc_gnn_train_workspace_size(const ldpc_gnn_plan *p, int hidden, int N, int64_t B, int layers) {
    if (!p || hidden <= 0 || hidden > kMaxTrainH || N <= 0 || B < 0 || layers <= 0)
        return fail(LDPC_EINVAL, "bad arguments (training needs hidden_dim <= 1024)");
    const int64_t fwd = gnn_fp32_train_workspace(p, hidden, N, B, layers);
    const int64_t bwd = carve_train(p, hidden, N, B, nullptr).bytes;
    return fwd > bwd ? fwd : bwd;
}

extern "C" int64_t ldpc_gnn_train_proj_floats(const ldpc_gnn_plan *p, int hidden, int64_t B, int layers) {
    if (!p || hidden <= 0 || B < 0 || layers <= 0) return fail(LDPC_EINVAL, "bad arguments");
    return gnn_proj_floats(p, hidden, B, layers);
}

extern "C" int ldpc_gnn_forward_train(const ldpc_gnn_plan *p, int hidden, int types, int layers,
                                      const float *d_weights, const int32_t *d_msg_type, const int32_t *d_msg_var,
                                      const float *d_llr, int N, int64_t B, float *d_probs, float *d_saved,
                                      void *d_work, int64_t work_bytes, void *stream) {
    return ldpc_gnn_forward_train_ex(p, hidden, types, layers, d_weights, d_msg_type, d_msg_var, d_llr, N, B, d_probs,
                                     d_saved, nullptr, d_work, work_bytes, stream);
}

extern "C" int ldpc_gnn_forward_train_ex(const ldpc_gnn_plan *p, int hidden, int types, int layers,
                                         const float *d_weights, const int32_t *d_msg_type, const int32_t *d_msg_var,
                                         const float *d_llr, int N, int64_t B, float *d_probs, float *d_saved,
                                         float *d_proj, void *d_work, int64_t work_bytes, void *stream) {
    if (!p) return fail(LDPC_EINVAL, "plan is NULL");
    if (hidden <= 0 || hidden > kMaxTrainH || types <= 0 || layers <= 0 || N <= 0 || B < 0)
        return fail(LDPC_EINVAL, "bad dimensions (training needs hidden_dim <= 1024)");
    if (B == 0) return LDPC_OK;
    if (!d_weights || !d_msg_type || !d_msg_var || !d_llr || !d_probs || !d_saved)
        return fail(LDPC_EINVAL, "NULL tensor");
    if (d_proj && gnn_proj_floats(p, hidden, B, layers) == 0) d_proj = nullptr;  // a path without the area
    return gnn_fp32_forward(p, hidden, types, layers, d_weights, d_msg_type, d_msg_var, d_llr, N, B, d_probs, d_saved,
                            d_work, work_bytes, static_cast<hipStream_t>(stream), d_proj);
}

extern "C" int ldpc_gnn_backward_ds(const ldpc_gnn_plan *p, int hidden, int types, int layers,
                                    const float *d_weights, const int32_t *d_msg_type, const int32_t *d_msg_var,
                                    const float *d_llr, int N, int64_t B, const float *d_probs,
                                    const float *d_grad_probs, const float *d_saved, const float *d_layer_probs,
                                    const float *d_grad_layer_probs, float *d_grad_weights, void *d_work,
                                    int64_t work_bytes, void *stream) {
    return ldpc_gnn_backward_ds_ex(p, hidden, types, layers, d_weights, d_msg_type, d_msg_var, d_llr, N, B, d_probs,
                                   d_grad_probs, d_saved, nullptr, d_layer_probs, d_grad_layer_probs, d_grad_weights,
                                   d_work, work_bytes, stream);
}

extern "C" int ldpc_gnn_backward_ds_ex(const ldpc_gnn_plan *p, int hidden, int types, int layers,
                                       const float *d_weights, const int32_t *d_msg_type, const int32_t *d_msg_var,
                                       const float *d_llr, int N, int64_t B, const float *d_probs,
                                       const float *d_grad_probs, const float *d_saved, const float *d_proj,
                                       const float *d_layer_probs, const float *d_grad_layer_probs,
                                       float *d_grad_weights, void *d_work, int64_t work_bytes, void *stream) {
    if (!p) return fail(LDPC_EINVAL, "plan is NULL");
    const int H = hidden, T = types, L = layers;
    if (H <= 0 || H > kMaxTrainH || T <= 0 || L <= 0 || N <= 0 || B < 0)
        return fail(LDPC_EINVAL, "bad dimensions (training needs hidden_dim <= 1024)");
    if (!d_weights || !d_msg_type || !d_msg_var || !d_llr || !d_probs || !d_grad_probs || !d_saved || !d_grad_weights)
        return fail(LDPC_EINVAL, "NULL tensor");
    if ((d_layer_probs == nullptr) != (d_grad_layer_probs == nullptr))
        return fail(LDPC_EINVAL, "d_layer_probs and d_grad_layer_probs go together");
    const bool ds = d_layer_probs != nullptr && L > 1;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t wfloats = 2LL * H + (int64_t)L * tl_floats(H, T);
    LDPC_HIP(hipMemsetAsync(d_grad_weights, 0, (size_t)wfloats * 4, s));
    if (B == 0) return LDPC_OK;
    TrainWs w = carve_train(p, H, N, B, d_work);
    if (!d_work || work_bytes < w.bytes)
        return fail(LDPC_EINVAL, "workspace too small: need " + std::to_string(w.bytes) + " bytes");
    if (!g_cus_t) {
        int dev = 0;
        LDPC_HIP(hipGetDevice(&dev));
        LDPC_HIP(hipDeviceGetAttribute(&g_cus_t, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int64_t E = p->E, R = B * E, n = R * H;
    const size_t lds_mlp = mlp_bwd_lds(H);
    // H > 64: train_mlp_bwd_wide_kernel with as many waves per workgroup (<= 4) as its LDS rows allow
    const int wide_waves = (int)std::max<size_t>(1, std::min<size_t>(4, (size_t)(160 * 1024) / mlp_bwd_wide_lds(H, 1)));
    if (H > kMaxH) {
        if (mlp_bwd_wide_lds(H, 1) > 160 * 1024) return fail(LDPC_EUNSUPPORTED, "hidden_dim too wide for the backward's LDS rows");
        LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(train_mlp_bwd_wide_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlp_bwd_wide_lds(H, wide_waves)));
    } else {
        LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(train_mlp_bwd_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_mlp));
    }
    LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(train_mlp_bwd_mfma_kernel<512>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlp_bwd_mfma_lds()));
    // projected groups (see train_mlp_bwd_mfma_kernel): H = 64 on MFMA with the plan's projection tiles
    const bool pj = H == 64 && bwd_proj() && p->n_ptiles > 0;
    // the forward's saved projections (ldpc_gnn_forward_train_ex): no recompute here
    const bool sp = pj && d_proj != nullptr;
    if (pj) {
        LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(train_mlp_bwd_mfma_kernel<512, true>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlp_bwd_mfma_lds()));
        LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(train_mlp_bwd_s6_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlp_bwd_s6_lds()));
    }
    auto blocks = [](int64_t work, int per) { return dim3((unsigned)((work + per - 1) / per)); };
    const unsigned red_grid = (unsigned)std::min<int64_t>((R + 63) / 64, (int64_t)g_cus_t * kOuterWgs);

    // head: dz, dX_L, dwo, dbo
    const float *WL[11];
    t_layer(d_weights, H, T, L - 1, WL);
    float *GL[11];
    t_layer(d_grad_weights, H, T, L - 1, GL);
    hipLaunchKernelGGL(train_head_kernel, blocks(B * N, 256), dim3(256), 0, s, d_probs, d_grad_probs, B * N, w.dz);
    LDPC_CHECK_LAUNCH("train_head_kernel");
    hipLaunchKernelGGL(train_dx_last_kernel, blocks(n, 256), dim3(256), 0, s, w.dz, d_msg_var, WL[9], H, E, N, n,
                       w.dX, 0);
    LDPC_CHECK_LAUNCH("train_dx_last_kernel");
    {
        VecT v{};
        v.part = w.dhv; v.part_cap = R * H;
        v.src = d_saved + (int64_t)(L - 1) * n;
        v.dz = w.dz;
        v.msg_type = d_msg_type;
        v.msg_var = d_msg_var;
        v.g0 = GL[9];
        v.g1 = GL[10];
        v.H = H; v.T = T; v.N = N; v.mode = 2; v.E = E; v.R = R;
        if (int rc = launch_vec(v, w.hv, w.hc, s)) return rc;
    }
    const bool ovl = pj && L > 1 && bwd_overlap() && !sp;
    hipStream_t s2 = nullptr;
    hipEvent_t ev_ready[2] = {}, ev_free[2] = {};
    int rc0 = 0;
    auto side_project = [&](int j) -> int {  // layer j's projections into set j & 1, on s2
        const float *xj = j > 0 ? d_saved + (int64_t)(j - 1) * n : nullptr;
        float *pv = (j & 1) ? w.Mv1 : w.Mv, *pc = (j & 1) ? w.Mc1 : w.Mc;
        float *gv = (j & 1) ? w.Gs1v : w.da, *gc = (j & 1) ? w.Gs1c : w.db;
        if (int rc = gnn_project_groups(p, T, d_weights, j, xj, d_msg_type, d_msg_var, d_llr, N, B, pv, pc, gv, gc, s2))
            return rc;
        LDPC_HIP(hipEventRecord(ev_ready[j & 1], s2));
        return LDPC_OK;
    };
    hipEvent_t fork = nullptr, join = nullptr;
    if (ovl) {
        if (int rc = gnn_side_stream(&s2, &fork, &join)) return rc;
        if (int rc = train_events(ev_ready, ev_free)) return rc;
        LDPC_HIP(hipEventRecord(fork, s));  // the workspace and inputs are the caller stream's
        LDPC_HIP(hipStreamWaitEvent(s2, fork, 0));
    }
    // the layers, then (side stream) a join on every exit, error returns included: nothing queued
    // on s2 may still write the caller's workspace once the caller's stream moves on
    auto layers_back = [&]() -> int {
    for (int l = L - 1; l >= 0; --l) {
        const float *W[11];
        t_layer(d_weights, H, T, l, W);
        float *Gw[11];
        t_layer(d_grad_weights, H, T, l, Gw);
        if (ds && l < L - 1) {  // deep supervision: layer l's output through the last layer's head
            const float *pl = d_layer_probs + (int64_t)l * B * N, *gl = d_grad_layer_probs + (int64_t)l * B * N;
            hipLaunchKernelGGL(train_head_kernel, blocks(B * N, 256), dim3(256), 0, s, pl, gl, B * N, w.dz);
            LDPC_CHECK_LAUNCH("train_head_kernel");
            hipLaunchKernelGGL(train_dx_last_kernel, blocks(n, 256), dim3(256), 0, s, w.dz, d_msg_var, WL[9], H, E, N,
                               n, w.dX, 1);
            LDPC_CHECK_LAUNCH("train_dx_last_kernel");
            VecT v{};
            v.part = w.dhv; v.part_cap = R * H;
            v.src = d_saved + (int64_t)l * n;
            v.dz = w.dz; v.msg_type = d_msg_type; v.msg_var = d_msg_var; v.g0 = GL[9]; v.g1 = GL[10];
            v.H = H; v.T = T; v.N = N; v.mode = 2; v.E = E; v.R = R;
            if (int rc = launch_vec(v, w.hv, w.hc, s)) return rc;
        }
        const float *x = l > 0 ? d_saved + (int64_t)(l - 1) * n : nullptr;
        // PJ: the group means of c go to da / db (free in this mode: no per-message group part);
        // with the side stream, odd layers use the second set
        const bool odd = ovl && (l & 1);
        float *Mv = odd ? w.Mv1 : w.Mv, *Mc = odd ? w.Mc1 : w.Mc;
        const float *Gsv = odd ? w.Gs1v : w.da, *Gsc = odd ? w.Gs1c : w.db;
        // projected rows the MLP backward reads (Pv / Pc) and the buffers that then receive the
        // group sums of dh (Mv / Mc): one set when recomputed here, apart with saved projections
        const float *Pv = Mv, *Pc = Mc;
        if (sp) {
            const int64_t G = p->Gv + p->Gc;
            const float *base = d_proj + (int64_t)l * B * G * 2 * H;
            Pv = base;
            Pc = base + B * p->Gv * H;
            Gsv = base + B * G * H;
            Gsc = base + B * G * H + B * p->Gv * H;
        } else if (ovl) {
            // side stream: layer l's set was filled one iteration earlier (or here, for the last
            // layer); layer l - 1's goes into the other set once layer l + 1 has released it
            if (l == L - 1 && (rc0 = side_project(l))) return rc0;
            if (l > 0) {
                if (l + 1 <= L - 1) LDPC_HIP(hipStreamWaitEvent(s2, ev_free[(l + 1) & 1], 0));
                if ((rc0 = side_project(l - 1))) return rc0;
            }
            LDPC_HIP(hipStreamWaitEvent(s, ev_ready[l & 1], 0));
        } else if (pj) {  // forward recompute: projected rows (Mv / Mc) and the group means (Gsv / Gsc)
            if (int rc = gnn_project_groups(p, T, d_weights, l, x, d_msg_type, d_msg_var, d_llr, N, B, Mv, Mc,
                                            w.da, w.db, s))  // = Gsv / Gsc here
                return rc;
        } else {  // group means of c (forward recompute)
            GmT g{};
            g.src = x; g.emb = W[0]; g.llr = d_llr; g.w_in = d_weights; g.b_in = d_weights + H;
            g.msg_type = d_msg_type; g.msg_var = d_msg_var;
            g.src_mode = x ? 1 : 2; g.H = H; g.N = N; g.E = E; g.B = B;
            g.ptr = p->vg_ptr; g.mem = p->vg_mem; g.inv = p->inv_v; g.G = p->Gv; g.dst = w.Mv; g.w = p->vg_w;
            if (int rc = launch_group_mean(g, s)) return rc;
            g.ptr = p->cg_ptr; g.mem = p->cg_mem; g.inv = p->inv_c; g.G = p->Gc; g.dst = w.Mc; g.w = p->cg_w;
            if (int rc = launch_group_mean(g, s)) return rc;
        }
        // MLP backward
        MlpT m{};
        m.x = x; m.llr = d_llr; m.w_in = d_weights; m.b_in = d_weights + H;
        m.Mv = Pv; m.Mc = Pc; m.dX = w.dX;
        m.msg_type = d_msg_type; m.msg_var = d_msg_var; m.vgroup = p->vgroup; m.cgroup = p->cgroup;
        m.emb = W[0]; m.w1v = W[1]; m.b1v = W[2]; m.w2v = W[3]; m.w1c = W[5]; m.b1c = W[6]; m.w2c = W[7];
        m.cbuf = pj ? nullptr : w.cbuf;  // PJ: train_dw1_kernel forms c itself
        m.hv = w.hv; m.hc = w.hc; m.dhv = w.dhv; m.dhc = w.dhc;
        m.dco = w.dco; m.da = w.da; m.db = w.db;
        m.H = H; m.N = N; m.Gv = p->Gv; m.Gc = p->Gc; m.E = E; m.R = R;
        if (H == 64) {  // fp32 MFMA / split MFMA kernels, 8 waves per workgroup
            const unsigned grid = (unsigned)std::min<int64_t>((R + 32 * 8 - 1) / (32 * 8), (int64_t)g_cus_t);
            if (pj && bwd_s6())
                hipLaunchKernelGGL(train_mlp_bwd_s6_kernel, dim3(grid), dim3(512), mlp_bwd_s6_lds(), s, m);
            else if (pj)
                hipLaunchKernelGGL((train_mlp_bwd_mfma_kernel<512, true>), dim3(grid), dim3(512), mlp_bwd_mfma_lds(), s, m);
            else
                hipLaunchKernelGGL(train_mlp_bwd_mfma_kernel<512>, dim3(grid), dim3(512), mlp_bwd_mfma_lds(), s, m);
            LDPC_CHECK_LAUNCH("train_mlp_bwd_mfma_kernel");
        } else if (H > kMaxH) {
            const int rows = wide_waves * kNM;
            const unsigned mgrid = (unsigned)std::min<int64_t>((R + rows - 1) / rows, (int64_t)g_cus_t * 8 / wide_waves);
            hipLaunchKernelGGL(train_mlp_bwd_wide_kernel, dim3(mgrid), dim3(64 * wide_waves), mlp_bwd_wide_lds(H, wide_waves),
                               s, m);
            LDPC_CHECK_LAUNCH("train_mlp_bwd_wide_kernel");
        } else {
            const unsigned mgrid = (unsigned)std::min<int64_t>((R + 4 * kNM - 1) / (4 * kNM), (int64_t)g_cus_t * 2);
            hipLaunchKernelGGL(train_mlp_bwd_kernel, dim3(mgrid), dim3(256), lds_mlp, s, m);
            LDPC_CHECK_LAUNCH("train_mlp_bwd_kernel");
        }
        if (pj) {
            // group sums of dh (into Mv / Mc: the projected rows are consumed), then the group part of
            // dz per group: Mda = W1v_right^T (sum dh) / |group|, Mdb likewise
            for (int side = 0; side < 2; ++side) {
                GmT gs{};
                gs.src = side ? w.dhc : w.dhv; gs.src_mode = 0; gs.sum_only = 1; gs.H = H; gs.N = N; gs.E = E; gs.B = B;
                gs.ptr = side ? p->cg_ptr : p->vg_ptr; gs.mem = side ? p->cg_mem : p->vg_mem;
                gs.inv = side ? p->inv_c : p->inv_v; gs.G = side ? p->Gc : p->Gv; gs.dst = side ? Mc : Mv;
                if (int rc = launch_group_mean(gs, s)) return rc;
            }
            const int64_t gtiles = (B * std::max(p->Gv, p->Gc) + 31) / 32;
            const unsigned ggrid = (unsigned)std::min<int64_t>((gtiles + 3) / 4, (int64_t)g_cus_t * 4);
            hipLaunchKernelGGL(train_group_back_kernel, dim3(ggrid), dim3(256), 0, s, Mv, Mc, W[1], W[5], p->inv_v,
                               p->inv_c, p->Gv, p->Gc, B, w.Mda, w.Mdb);
            LDPC_CHECK_LAUNCH("train_group_back_kernel");
        } else {
            // group means of the aggregated-input gradients (the mean operator is symmetric); a
            // general adjacency A (weighted plan): A^T of them, over the plan's transposed CSR
            GmT d{};
            d.src_mode = 0; d.H = H; d.N = N; d.E = E; d.B = B;
            d.src = w.da; d.ptr = p->vg_ptr; d.mem = p->vg_mem; d.inv = p->inv_v; d.G = p->Gv; d.dst = w.Mda;
            if (p->weighted) { d.ptr = p->vt_ptr; d.mem = p->vt_mem; d.w = p->vt_w; }
            if (int rc = launch_group_mean(d, s)) return rc;
            d.src = w.db; d.ptr = p->cg_ptr; d.mem = p->cg_mem; d.inv = p->inv_c; d.G = p->Gc; d.dst = w.Mdb;
            if (p->weighted) { d.ptr = p->ct_ptr; d.mem = p->ct_mem; d.w = p->ct_w; }
            if (int rc = launch_group_mean(d, s)) return rc;
        }
        if (pj) {
            // combined with the embedding gradient's frame sums after the weight gradients (below),
            // into hv / hc once dW2 has read them
        } else if (H % 4 == 0)
            hipLaunchKernelGGL(train_combine4_kernel, blocks(n / 4, 256), dim3(256), 0, s,
                               reinterpret_cast<float4 *>(w.dco), reinterpret_cast<const float4 *>(w.Mda),
                               reinterpret_cast<const float4 *>(w.Mdb), reinterpret_cast<const float4 *>(w.dX),
                               p->vgroup, p->cgroup, H / 4, p->Gv, p->Gc, E, n / 4, l > 0 ? 1 : 0,
                               reinterpret_cast<float4 *>(w.dXp));
        else
            hipLaunchKernelGGL(train_combine_kernel, blocks(n, 256), dim3(256), 0, s, w.dco, w.Mda, w.Mdb, w.dX,
                               p->vgroup, p->cgroup, H, p->Gv, p->Gc, E, n, l > 0 ? 1 : 0, w.dXp);
        LDPC_CHECK_LAUNCH("train_combine_kernel");
        // weight gradients
        OuterT o{};
        o.H = H; o.E = E; o.R = R;
        if (H == 64) {  // dW2v and dW2c in one pass over dX
            Dw2T d2{w.dX, w.hv, w.hc, Gw[3], Gw[7], Gw[4], Gw[8], R};
            hipLaunchKernelGGL(train_dw2_kernel, dim3(red_grid), dim3(256), 0, s, d2);
            LDPC_CHECK_LAUNCH("train_dw2_kernel");
        } else {  // general H: two passes
            o.A = w.dX; o.zsrc = w.hv; o.J = H; o.out = Gw[3]; o.bias = Gw[4];
            if (int rc = launch_outer(o, red_grid, s)) return rc;
            o.zsrc = w.hc; o.out = Gw[7]; o.bias = Gw[8];
            if (int rc = launch_outer(o, red_grid, s)) return rc;
        }
        // dW1_s = sum_m dh_s[m] (x) [c_m; g_s(group(m))]: the c half row by row; the group half as
        // sum_groups (sum_{m in group} dh_s[m]) (x) g_s(group) -- contiguous group rows instead of
        // a gathered group row per message (Mda / Mdb are free again after the combine step)
        if (pj) {  // the c half of both sides in one pass, c formed from x (no stored copy)
            Dw1T d{};
            d.dhv = w.dhv; d.dhc = w.dhc; d.x = x; d.emb = W[0]; d.llr = d_llr;
            d.w_in = d_weights; d.b_in = d_weights + H; d.msg_type = d_msg_type; d.msg_var = d_msg_var;
            d.gv = Gw[1]; d.gc = Gw[5]; d.bv = Gw[2]; d.bc = Gw[6];
            d.T = T; d.N = N; d.E = E; d.R = R;
            if (x)
                hipLaunchKernelGGL(train_dw1_kernel<1>, dim3(red_grid), dim3(256), dw1_lds(T), s, d);
            else
                hipLaunchKernelGGL(train_dw1_kernel<2>, dim3(red_grid), dim3(256), dw1_lds(T), s, d);
            LDPC_CHECK_LAUNCH("train_dw1_kernel");
        }
        for (int side = 0; side < 2; ++side) {
            // PJ: the group means are in Gsv / Gsc and the group sums of dh already in Mv / Mc
            const float *dh = side ? w.dhc : w.dhv, *Gs = pj ? (side ? Gsc : Gsv) : side ? w.Mc : w.Mv;
            float *dhsum = pj ? (side ? Mc : Mv) : side ? w.Mdb : w.Mda;
            float *gw = side ? Gw[5] : Gw[1], *gb = side ? Gw[6] : Gw[2];
            const int Gn = side ? p->Gc : p->Gv;
            if (!pj) {
                OuterT c{};
                c.H = H; c.E = E; c.R = R; c.A = dh; c.zsrc = w.cbuf; c.J = H; c.ld = 2 * H; c.col0 = 0;
                c.out = gw; c.bias = gb;
                if (int rc = launch_outer(c, red_grid, s)) return rc;
            }
            if (!pj && !p->weighted) {  // weighted: every message reads its own aggregated row
                GmT gs{};
                gs.src = dh; gs.src_mode = 0; gs.sum_only = 1; gs.H = H; gs.N = N; gs.E = E; gs.B = B;
                gs.ptr = side ? p->cg_ptr : p->vg_ptr; gs.mem = side ? p->cg_mem : p->vg_mem;
                gs.inv = side ? p->inv_c : p->inv_v; gs.G = Gn; gs.dst = dhsum;
                if (int rc = launch_group_mean(gs, s)) return rc;
            }
            OuterT g{};
            g.H = H; g.E = (int64_t)Gn; g.R = B * Gn; g.A = p->weighted ? dh : dhsum; g.zsrc = Gs; g.J = H; g.ld = 2 * H; g.col0 = H;
            g.out = gw; g.bias = nullptr;
            const unsigned ggrid = (unsigned)std::min<int64_t>((g.R + 63) / 64, (int64_t)g_cus_t * kOuterWgs);
            if (int rc = launch_outer(g, ggrid, s)) return rc;
        }
        if (ovl) LDPC_HIP(hipEventRecord(ev_free[l & 1], s));  // this layer's set is free again
        VecT v{};
        v.part = w.dhv; v.part_cap = R * H;
        v.src = w.dco; v.llr = d_llr; v.msg_type = d_msg_type; v.msg_var = d_msg_var;
        v.H = H; v.T = T; v.N = N; v.E = E; v.R = R;
        if (pj) {  // dx_l, and the frame sums of dc (hv) and of dc * llr (hc, layer 0)
            const int64_t EH = E * H;
            if (l == 0)
                hipLaunchKernelGGL(train_combine_sum_kernel<true>, blocks(EH, 256), dim3(256), 0, s, w.dco, w.Mda,
                                   w.Mdb, w.dX, p->vgroup, p->cgroup, d_msg_var, d_llr, H, p->Gv, p->Gc, N, E, B, 0,
                                   w.dXp, w.hv, w.hc);
            else
                hipLaunchKernelGGL(train_combine_sum_kernel<false>, blocks(EH, 256), dim3(256), 0, s, w.dco, w.Mda,
                                   w.Mdb, w.dX, p->vgroup, p->cgroup, d_msg_var, d_llr, H, p->Gv, p->Gc, N, E, B, 1,
                                   w.dXp, w.hv, w.hc);
            LDPC_CHECK_LAUNCH("train_combine_sum_kernel");
            v.mode = 0; v.g0 = Gw[0];
            if (int rc = launch_vecfinal(v, w.hv, w.hc, s)) return rc;
            if (l == 0) {  // dw_in from sum dc * llr, db_in from sum dc
                v.mode = 1; v.g0 = d_grad_weights; v.g1 = d_grad_weights + H;
                if (int rc = launch_vecfinal(v, w.hc, w.hv, s)) return rc;
            }
        } else {
            v.mode = 0; v.g0 = Gw[0];
            if (int rc = launch_vec(v, w.hv, w.hc, s)) return rc;
            if (l == 0) {
                v.mode = 1; v.g0 = d_grad_weights; v.g1 = d_grad_weights + H;
                if (int rc = launch_vec(v, w.hv, w.hc, s)) return rc;
            }
        }
        std::swap(w.dX, w.dXp);
    }
    return LDPC_OK;
    };
    const int rc = layers_back();
    if (ovl) {
        LDPC_HIP(hipEventRecord(join, s2));
        LDPC_HIP(hipStreamWaitEvent(s, join, 0));
    }
    return rc;
}

extern "C" int ldpc_gnn_backward(const ldpc_gnn_plan *p, int hidden, int types, int layers, const float *d_weights,
                                 const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N,
                                 int64_t B, const float *d_probs, const float *d_grad_probs, const float *d_saved,
                                 float *d_grad_weights, void *d_work, int64_t work_bytes, void *stream) {
    return ldpc_gnn_backward_ds(p, hidden, types, layers, d_weights, d_msg_type, d_msg_var, d_llr, N, B, d_probs,
                                d_grad_probs, d_saved, nullptr, nullptr, d_grad_weights, d_work, work_bytes, stream);
}

extern "C" int ldpc_gnn_layer_probs(const ldpc_gnn_plan *p, int hidden, int types, int layers, const float *d_weights,
                                    const int32_t *d_msg_var, const float *d_llr, int N, int64_t B,
                                    const float *d_saved, float *d_layer_probs, void *d_work, int64_t work_bytes,
                                    void *stream) {
    if (!p) return fail(LDPC_EINVAL, "plan is NULL");
    const int H = hidden, T = types, L = layers;
    if (H <= 0 || H > kMaxTrainH || T <= 0 || L <= 0 || N <= 0 || B < 0) return fail(LDPC_EINVAL, "bad dimensions");
    if (L < 2 || B == 0) return LDPC_OK;
    if (!d_weights || !d_msg_var || !d_llr || !d_saved || !d_layer_probs) return fail(LDPC_EINVAL, "NULL tensor");
    const int64_t E = p->E, R = B * E, mo = (R + 63) / 64 * 64;
    const int64_t need = (mo + gnn_csr_ints(E, N)) * 4;
    if (!d_work || work_bytes < need) return fail(LDPC_EINVAL, "workspace too small: need " + std::to_string(need) + " bytes");
    hipStream_t s = static_cast<hipStream_t>(stream);
    float *msg_out = static_cast<float *>(d_work);
    int32_t *csr = reinterpret_cast<int32_t *>(msg_out + mo);
    if (int rc = gnn_build_var_csr(d_msg_var, E, N, csr, s)) return rc;
    const float *WL[11];
    t_layer(d_weights, H, T, L - 1, WL);
    for (int l = 0; l < L - 1; ++l) {
        hipLaunchKernelGGL(train_msg_head_kernel, dim3((unsigned)((R * 16 + 255) / 256)), dim3(256), 0, s,
                           d_saved + (int64_t)l * R * H, H, R, WL[9], WL[10], msg_out);
        LDPC_CHECK_LAUNCH("train_msg_head_kernel");
        if (int rc = gnn_output(msg_out, csr, d_llr, E, N, B, nullptr, d_layer_probs + (int64_t)l * B * N, s)) return rc;
    }
    return LDPC_OK;
}
