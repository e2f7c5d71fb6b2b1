// gnn.hip -- message-centred GNN decoder forward for gfx950.
//
// Replaces MessageGNNDecoder.forward (message_gnn_decoder.py:190-317):
//   x0 = Linear(1,H)(llr[msg_var])                                      (:215-235)
//   per layer i:  c = x + emb_i[type]                                   (:81-90)
//                 a = A_v c,  b = A_c c   -- group means (the normalized clique adjacencies
//                                            of :410-469 are exactly segment means)
//                 y = MLP_v([c;a]) + MLP_c([c;b]),  x <- y (+ x if i > 0)  (:106-127, :261-262)
//   out_m = output_projection_{L-1}(x_m)                                (:270, :142)
//   probs = sigmoid(llr + sum_{m -> v} out_m)                           (:273-307)
//
// Kernels per layer (no E x E matrix anywhere):
//   gnn_group_mean_kernel   one wave per (frame, group): mean of c over the group's messages,
//                           H lanes, 256-B coalesced rows.  Layer 0 builds c from the LLRs.
//                           H = 64 runs gnn_group_mean_tile_kernel instead: one wave per 8 groups
//                           of one degree (the plan's group tiles), 8 lanes x 32 B per row.
//   gnn_group_proj_kernel   H = 64, group plans (default): the group mean AND its product with
//                           the group half of each side's first Linear (+ b1), one row per group,
//                           so the per-message GEMM1 runs over c only (see the kernel).
//   gnn_mlp2_kernel         H = 64, group plans (default): the MLP over c started from those rows.
//                           The two frame halves of a call run on two streams.
//   gnn_mlp_mfma_kernel     H = 64, general (CSR) adjacencies and LDPC_GNN_PROJ=0: the
//                           per-message [c; g] form.  Persistent, one 512-thread workgroup per CU holding the
//                           layer's four weight matrices (100 KB fp32, rows padded so one
//                           ds_read_b128 feeds four MFMA k-steps) in LDS; every wave owns a
//                           32-message tile and runs the four GEMMs on v_mfma_f32_32x32x2_f32 in
//                           the transposed orientation (hidden units on the MFMA rows, messages
//                           on the lanes), so GEMM1's accumulator IS GEMM2's B operand with no
//                           data movement; bias, ReLU, the v+c sum, the residual and (last
//                           layer) the output projection + per-variable scatter are fused.
//   gnn_mlp_generic_kernel  any H (VALU); used for H != 64 (e.g. the small-H test fixtures).
//   gnn_output_kernel       probs = sigmoid(sum of each variable's messages + llr), ascending order.
// precision 1 (bf16 features, bf16 MFMA) lives in gnn_bf16.hip.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "gnn.hpp"


namespace ldpc {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMfmaH = 64;
// other hidden widths run on gnn_mlp_generic_kernel: 4 waves x 4 H floats of LDS (64 KB at 1024)
constexpr int kMaxGenericH = 1024;
#ifndef LDPC_MLP2_WPS
#define LDPC_MLP2_WPS 3
#endif
#ifndef LDPC_MLP2_NT
#define LDPC_MLP2_NT 768
#endif
#ifndef LDPC_PROJ_WPS
#define LDPC_PROJ_WPS 2
#endif
#ifndef LDPC_PROJ_NT
#define LDPC_PROJ_NT 768
#endif
// LDPC_GNN_D1=0 keeps the Mv rows of degree-1 var groups (A/B runs)
bool d1_skip() {
    static bool t = [] {
        const char *e = std::getenv("LDPC_GNN_D1");
        return !(e && std::atoi(e) == 0);
    }();
    return t;
}
// LDPC_GNN_GM=0 selects the per-group fp32 group-mean kernel (A/B runs); default: group tiles
bool gm_tiles() {
    static bool t = [] {
        const char *e = std::getenv("LDPC_GNN_GM");
        return !(e && std::atoi(e) == 0);
    }();
    return t;
}

struct GnnLayer {
    // input features: x_in (B, E, H) or, for layer 0, the embedding of the LLRs
    const float *x_in;
    const float *llr;      // (B, N)
    const int32_t *msg_var;
    const float *w_in, *b_in;
    int N;
    // layer weights (blob section, see ldpc_amd.h)
    const float *emb, *w1v, *b1v, *w2v, *b2v, *w1c, *b1c, *w2c, *b2c, *wo, *bo;
    int T;
    const int32_t *msg_type;
    // plan
    const int32_t *vgroup, *cgroup, *vg_ptr, *vg_mem, *cg_ptr, *cg_mem;
    const float *inv_v, *inv_c;
    const float *vg_w, *cg_w;  // weighted plan: member weights (NULL for group plans)
    int Gv, Gc;
    int64_t E, B;
    // group means
    float *Mv, *Mc;  // (B, Gv, H), (B, Gc, H)
    // outputs
    float *x_out;    // (B, E, H); null on the last layer unless training saves its features
    float *msg_out;  // (B, E) projected message LLRs, last layer only
    int residual, last;
    int vside;       // 0: the check side alone (hybrid decoder, gnn_custom_var_forward)
    int d1;          // degree-1 var groups have no Mv row: the MLP uses the message's own c as g
    // hybrid decoder (gnn_custom_var_forward): x_in holds the previous layer's F and the features
    // are x = (v2c w_in + b_in) + F, formed where a row is read (custom_combine_kernel's exact
    // float sequence) instead of being written back between the layers
    const float *hv2c = nullptr;  // (B, E)
    const float *wt = nullptr;    // H != 64, gnn_mlp_tiled_kernel: this layer's W1v^T, W2v^T, W1c^T, W2c^T
    // training backward (gnn_project_groups): the projection kernel also writes the group means
    // it projects, (B, Gv, H) / (B, Gc, H)
    float *gsave_v = nullptr, *gsave_c = nullptr;
    // gnn_mlp2s_kernel message tiles in the plan's order (gnn.hpp mt_perm: degree-1 var groups'
    // messages first): tperm[32 k + j] = message of slot j of a frame's tile k (-1 = padding), its
    // first ntile_v1 tiles hold degree-1 messages only.  Null: tiles of 32 consecutive messages.
    const int32_t *tperm = nullptr;
    int ntile_pf = 0, ntile_v1 = 0;
    // fp32 row walk (gnn_mlp2s_kernel RW, plan rw_*): rw_n check tile groups per frame; the MLP writes
    // each check's sum of its output rows to S_out (B, Gc, 64) for the next layer, whose projection
    // forms the check-side means as S_in * inv_c + memb (this layer's mean type embedding per check)
    const int4 *rw_meta = nullptr;
    int rw_n = 0;
    float *S_out = nullptr;
    const float *S_in = nullptr, *memb = nullptr;
    const float *memb_v = nullptr;  // this layer's mean type embedding per var group (Gv, 64): the var-side
                                    // gather then sums x alone (gnn_group_proj_kernel)
};


__device__ __forceinline__ float4 hyb_x(float4 f, float v, float4 w, float4 c) {
    return make_float4((v * w.x + c.x) + f.x, (v * w.y + c.y) + f.y, (v * w.z + c.z) + f.z, (v * w.w + c.w) + f.w);
}

// feature u of message m of frame b *before* the type embedding
__device__ __forceinline__ float x_feat(const GnnLayer &P, int64_t b, int64_t m, int u, int H) {
    if (P.hv2c)  // hybrid decoder: x = (v2c w_in + b_in) + F (custom_combine_kernel's float sequence)
        return (P.hv2c[b * P.E + m] * P.w_in[u] + P.b_in[u]) + P.x_in[(b * P.E + m) * H + u];
    if (P.x_in) return P.x_in[(b * P.E + m) * H + u];
    const float l = P.llr[b * P.N + P.msg_var[m]];
    return l * P.w_in[u] + P.b_in[u];  // Linear(1, H)
}

// ------------------------------------------------------------------------ group means
__global__ __launch_bounds__(256) void gnn_group_mean_kernel(GnnLayer P, int H) {
    const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t G = P.Gv + P.Gc;
    if (wid >= P.B * G) return;
    const int64_t b = wid / G;
    const int g = (int)(wid - b * G);
    const bool isv = g < P.Gv;
    if (isv && !P.vside) return;  // the hybrid decoder's check side alone
    const int gg = isv ? g : g - P.Gv;
    const int32_t *ptr = isv ? P.vg_ptr : P.cg_ptr;
    const int32_t *mem = isv ? P.vg_mem : P.cg_mem;
    const float inv = isv ? P.inv_v[gg] : P.inv_c[gg];
    const float *wts = isv ? P.vg_w : P.cg_w;
    float *dst = (isv ? P.Mv + (b * P.Gv + gg) * H : P.Mc + (b * P.Gc + gg) * H);
    const int p0 = ptr[gg], p1 = ptr[gg + 1];
    for (int u = lane; u < H; u += 64) {
        float s = 0.0f;
        for (int p = p0; p < p1; ++p) {
            const int m = mem[p];
            const float c = x_feat(P, b, m, u, H) + P.emb[P.msg_type[m] * H + u];
            if (wts)  // general adjacency (message_gnn_decoder.py:108/118: bmm(A, c)), nonzeros ascending
                s += wts[p] * c;
            else
                s += c;
        }
        dst[u] = s * inv;
    }
}

// H = 64 fp32: 16 lanes per group (float4 each), 4 groups per wave, members unrolled by 4 so
// every lane keeps 4 x 16 B in flight (the plain kernel above is latency-bound at ~1.7 TB/s).
__global__ __launch_bounds__(256) void gnn_group_mean_h64_kernel(GnnLayer P) {
    const int lane = threadIdx.x & 63, q = lane & 15;
    const int64_t gid = (xcd_block(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6)) * 4 + (lane >> 4);
    const int64_t G = P.Gv + P.Gc;
    if (gid >= P.B * G) return;
    const int64_t b = gid / G;
    const int g = (int)(gid - b * G);
    const bool isv = g < P.Gv;
    const int gg = isv ? g : g - P.Gv;
    const int32_t *ptr = isv ? P.vg_ptr : P.cg_ptr;
    const int32_t *mem = isv ? P.vg_mem : P.cg_mem;
    const float inv = isv ? P.inv_v[gg] : P.inv_c[gg];
    float4 *dst = reinterpret_cast<float4 *>(isv ? P.Mv + (b * P.Gv + gg) * 64 : P.Mc + (b * P.Gc + gg) * 64) + q;
    const int p0 = ptr[gg], p1 = ptr[gg + 1];
    auto feat = [&](int m) -> float4 {
        const float4 e = reinterpret_cast<const float4 *>(P.emb + P.msg_type[m] * 64)[q];
        float4 x;
        if (P.x_in) {
            x = reinterpret_cast<const float4 *>(P.x_in + (b * P.E + m) * 64)[q];
        } else {
            const float l = P.llr[b * P.N + P.msg_var[m]];
            const float4 w = reinterpret_cast<const float4 *>(P.w_in)[q], bb = reinterpret_cast<const float4 *>(P.b_in)[q];
            x = make_float4(l * w.x + bb.x, l * w.y + bb.y, l * w.z + bb.z, l * w.w + bb.w);
        }
        return make_float4(x.x + e.x, x.y + e.y, x.z + e.z, x.w + e.w);
    };
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    int p = p0;
    for (; p + 4 <= p1; p += 4) {
        const float4 a = feat(mem[p]), bq = feat(mem[p + 1]), c = feat(mem[p + 2]), d = feat(mem[p + 3]);
        acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
        acc.x += bq.x; acc.y += bq.y; acc.z += bq.z; acc.w += bq.w;
        acc.x += c.x; acc.y += c.y; acc.z += c.z; acc.w += c.w;
        acc.x += d.x; acc.y += d.y; acc.z += d.z; acc.w += d.w;
    }
    for (; p < p1; ++p) {
        const float4 a = feat(mem[p]);
        acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    }
    *dst = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
}

// H = 64 fp32 on the plan's group tiles (gnn.hpp): one wave sums 8 groups of ONE degree, so no
// lane idles behind a longer group of its wave; 8 lanes x 32 B per 256-B row, members unrolled
// by 4 (8 x 16 B of features in flight per lane).  Same per-message sum order as above
// (ascending members, x + emb first), so the rows are bit-identical.
struct GtTiles {
    const int2 *meta;
    const int32_t *grp, *mem;
    int n_tiles;
    int first;  // P.d1: the leading degree-1 var tiles are skipped (their mean is c itself)
};

__global__ __launch_bounds__(256) void gnn_group_mean_tile_kernel(GnnLayer P, GtTiles G) {
    const uint32_t w = (uint32_t)(xcd_block(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6));
    const uint32_t nt = (uint32_t)(G.n_tiles - G.first);
    if (w >= (uint32_t)P.B * nt) return;
    const uint32_t b = w / nt, t = w - b * nt + (uint32_t)G.first;
    const int lane = threadIdx.x & 63, q = lane >> 3, p0 = 8 * (lane & 7);
    const int2 md = G.meta[t];
    const int g = G.grp[8 * t + q];
    const int32_t *mem = G.mem + md.y + q;
    float4 a0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), a1 = a0;
    auto add = [](float4 &acc, float4 x, float4 e) {
        acc.x += x.x + e.x; acc.y += x.y + e.y; acc.z += x.z + e.z; acc.w += x.w + e.w;
    };
    const float4 *emb = reinterpret_cast<const float4 *>(P.emb + p0);
    if (P.x_in) {
        const float4 *xb = reinterpret_cast<const float4 *>(P.x_in + (int64_t)b * P.E * 64 + p0);
        int i = 0;
        for (; i + 4 <= md.x; i += 4) {
            const int m0 = mem[8 * i], m1 = mem[8 * i + 8], m2 = mem[8 * i + 16], m3 = mem[8 * i + 24];
            const float4 x00 = xb[m0 * 16], x01 = xb[m0 * 16 + 1], x10 = xb[m1 * 16], x11 = xb[m1 * 16 + 1];
            const float4 x20 = xb[m2 * 16], x21 = xb[m2 * 16 + 1], x30 = xb[m3 * 16], x31 = xb[m3 * 16 + 1];
            const int t0 = P.msg_type[m0] * 16, t1 = P.msg_type[m1] * 16;
            const int t2 = P.msg_type[m2] * 16, t3 = P.msg_type[m3] * 16;
            add(a0, x00, emb[t0]); add(a1, x01, emb[t0 + 1]);
            add(a0, x10, emb[t1]); add(a1, x11, emb[t1 + 1]);
            add(a0, x20, emb[t2]); add(a1, x21, emb[t2 + 1]);
            add(a0, x30, emb[t3]); add(a1, x31, emb[t3 + 1]);
        }
        for (; i < md.x; ++i) {
            const int m = mem[8 * i], tt = P.msg_type[m] * 16;
            add(a0, xb[m * 16], emb[tt]); add(a1, xb[m * 16 + 1], emb[tt + 1]);
        }
    } else {
        const float4 w0 = reinterpret_cast<const float4 *>(P.w_in + p0)[0], w1 = reinterpret_cast<const float4 *>(P.w_in + p0)[1];
        const float4 c0 = reinterpret_cast<const float4 *>(P.b_in + p0)[0], c1 = reinterpret_cast<const float4 *>(P.b_in + p0)[1];
        for (int i = 0; i < md.x; ++i) {
            const int m = mem[8 * i], tt = P.msg_type[m] * 16;
            const float l = P.llr[(int64_t)b * P.N + P.msg_var[m]];
            add(a0, make_float4(l * w0.x + c0.x, l * w0.y + c0.y, l * w0.z + c0.z, l * w0.w + c0.w), emb[tt]);
            add(a1, make_float4(l * w1.x + c1.x, l * w1.y + c1.y, l * w1.z + c1.z, l * w1.w + c1.w), emb[tt + 1]);
        }
    }
    if (g < 0) return;
    const bool isv = g < P.Gv;
    const int gg = isv ? g : g - P.Gv;
    const float inv = isv ? P.inv_v[gg] : P.inv_c[gg];
    float4 *dst = reinterpret_cast<float4 *>((isv ? P.Mv + ((int64_t)b * P.Gv + gg) * 64 : P.Mc + ((int64_t)b * P.Gc + gg) * 64) + p0);
    dst[0] = make_float4(a0.x * inv, a0.y * inv, a0.z * inv, a0.w * inv);
    dst[1] = make_float4(a1.x * inv, a1.y * inv, a1.z * inv, a1.w * inv);
}

// ------------------------------------------------------------------------ fused MLP, H = 64
// LDS image (floats): W1vT[128][64] W2vT[64][64] W1cT[128][64] W2cT[64][64]
//                     b1v b2v b1c b2c wo [64 each]  emb[T][64]
// Weights are stored row-major per output unit, rows padded (132 / 68 floats: a 16-lane phase of
// ds_read_b128 then hits 64 distinct banks), so one ds_read_b128 feeds four MFMA k-steps.
constexpr int kS1 = 132, kS2 = 68;
constexpr int kW1 = 64 * kS1, kW2 = 64 * kS2;
constexpr int kOffW1v = 0, kOffW2v = kW1, kOffW1c = kW1 + kW2, kOffW2c = 2 * kW1 + kW2;
constexpr int kOffBias = 2 * kW1 + 2 * kW2;  // b1v, b2v, b1c, b2c, wo
constexpr int kOffEmb = kOffBias + 5 * 64;
// type-embedding rows padded to 68 floats: lanes of one tile read the rows of different types at
// the same column, and a 256-B row stride would put all of them on one LDS bank
constexpr int kEmbStride = 68;

__device__ __forceinline__ int crow(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

template <int kMlpThreads>
// both variants cap registers at 2 waves per SIMD: the 256-thread one then leaves half of every
// SIMD's register file to the group-mean waves of the other stream
__global__ __launch_bounds__(kMlpThreads, 2) void gnn_mlp_mfma_kernel(GnnLayer P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int H = kMfmaH;
    const int tid = threadIdx.x;
    // stage the layer's weights, transposed so lanes read consecutive output units
    for (int i = tid; i < 128 * 64; i += kMlpThreads) {
        const int o = i / 128, k = i - o * 128;
        lds[kOffW1v + o * kS1 + k] = P.w1v[i];
        lds[kOffW1c + o * kS1 + k] = P.w1c[i];
    }
    for (int i = tid; i < 64 * 64; i += kMlpThreads) {
        const int o = i / 64, k = i - o * 64;
        lds[kOffW2v + o * kS2 + k] = P.w2v[i];
        lds[kOffW2c + o * kS2 + k] = P.w2c[i];
    }
    if (tid < 64) {
        lds[kOffBias + tid] = P.b1v[tid];
        lds[kOffBias + 64 + tid] = P.b2v[tid];
        lds[kOffBias + 128 + tid] = P.b1c[tid];
        lds[kOffBias + 192 + tid] = P.b2c[tid];
        lds[kOffBias + 256 + tid] = P.last ? P.wo[tid] : 0.0f;
    }
    for (int i = tid; i < P.T * 64; i += kMlpThreads) lds[kOffEmb + (i >> 6) * kEmbStride + (i & 63)] = P.emb[i];
    __syncthreads();

    const int lane = tid & 63, j = lane & 31, half = lane >> 5;
    const int wave = tid >> 6;
    const int64_t R = P.B * P.E;
    const int64_t ntiles = (R + 31) / 32;
    const float bo = P.last ? P.bo[0] : 0.0f;
    const TileWalk tw = xcd_tiles(ntiles, kMlpThreads / 64, wave);
    for (int64_t t = tw.first; t < tw.end; t += tw.stride) {
        const int64_t row = t * 32 + j;
        const bool ok = row < R;
        const int64_t rr = ok ? row : R - 1;
        const int64_t b = rr / P.E, m = rr - b * P.E;
        // B operands: half 0 lanes carry c (k = 0..63), half 1 lanes carry a, then b (k = 64..127)
        float in[H];
        const float4 *grp = nullptr;  // half 1: the group-mean row of the current side
        // a degree-1 var group's mean is the message's own c (x + emb, times 1/1): half 1 builds
        // it exactly as half 0 does, so the group-mean launch writes no row for it
        const int vg = P.vgroup[m];
        const bool self_g = P.d1 && half == 1 && P.vg_ptr[vg + 1] - P.vg_ptr[vg] == 1;
        if (half == 0 || self_g) {
            const int ty = P.msg_type[m];
            const float *e = lds + kOffEmb + ty * kEmbStride;
            if (P.x_in) {
                const float4 *xr = reinterpret_cast<const float4 *>(P.x_in + rr * H);
#pragma unroll
                for (int q = 0; q < H / 4; ++q) {
                    const float4 v = xr[q];
                    in[4 * q + 0] = v.x + e[4 * q + 0];
                    in[4 * q + 1] = v.y + e[4 * q + 1];
                    in[4 * q + 2] = v.z + e[4 * q + 2];
                    in[4 * q + 3] = v.w + e[4 * q + 3];
                }
            } else {
                const float l = P.llr[b * P.N + P.msg_var[m]];
#pragma unroll
                for (int u = 0; u < H; ++u) in[u] = (l * P.w_in[u] + P.b_in[u]) + e[u];
            }
        } else {
            grp = reinterpret_cast<const float4 *>(P.Mv + (b * P.Gv + vg) * H);
#pragma unroll
            for (int q = 0; q < H / 4; ++q) {
                const float4 v = grp[q];
                in[4 * q + 0] = v.x; in[4 * q + 1] = v.y; in[4 * q + 2] = v.z; in[4 * q + 3] = v.w;
            }
        }
        if (half == 1) grp = reinterpret_cast<const float4 *>(P.Mc + (b * P.Gc + P.cgroup[m]) * H);
        f32x16 y0 = {}, y1 = {};
        // per-lane weight offsets, made opaque so the loop-invariant LDS reads are not hoisted
        int w1lane = j * kS1 + half * 64, w2lane = j * kS2 + 4 * half;
        asm volatile("" : "+v"(w1lane), "+v"(w2lane));
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            if (side == 1 && half == 1) {
#pragma unroll
                for (int q = 0; q < H / 4; ++q) {
                    const float4 v = grp[q];
                    in[4 * q + 0] = v.x; in[4 * q + 1] = v.y; in[4 * q + 2] = v.z; in[4 * q + 3] = v.w;
                }
            }
            const float *W1 = lds + (side == 0 ? kOffW1v : kOffW1c);
            const float *W2 = lds + (side == 0 ? kOffW2v : kOffW2c);
            const float *b1 = lds + kOffBias + (side == 0 ? 0 : 128);
            // GEMM1^T: h[u][msg] = sum_k W1[u][k] * in[k][msg], k = half*64 + kk
            f32x16 h0 = {}, h1 = {};
#pragma unroll
            for (int kk = 0; kk < 64; kk += 4) {
                const float4 wa = *reinterpret_cast<const float4 *>(W1 + w1lane + kk);
                const float4 wb = *reinterpret_cast<const float4 *>(W1 + w1lane + 32 * kS1 + kk);
                const float a4[4] = {wa.x, wa.y, wa.z, wa.w}, b4[4] = {wb.x, wb.y, wb.z, wb.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    h0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[i], in[kk + i], h0, 0, 0, 0);
                    h1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b4[i], in[kk + i], h1, 0, 0, 0);
                }
            }
            // bias + ReLU; register r of row tile rt holds unit 32*rt + crow(r, half)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                h0[r] = relu_nan(h0[r] + b1[crow(r, half)]);
                h1[r] = relu_nan(h1[r] + b1[32 + crow(r, half)]);
            }
            // GEMM2^T: y[o][msg] += sum_u W2[o][u] * h[u][msg]; step (rt, r) pairs unit
            // crow(r,0) (half 0) with crow(r,1) (half 1) -- exactly the registers each lane holds
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                // registers 4 rq .. 4 rq + 3 hold units crow(4 rq + i, half) = 8 rq + 4 half + i
                const float *w = W2 + w2lane + 8 * rq;
                const float4 a0 = *reinterpret_cast<const float4 *>(w);                 // o = j,      u
                const float4 a1 = *reinterpret_cast<const float4 *>(w + 32 * kS2);      // o = 32 + j, u
                const float4 c0 = *reinterpret_cast<const float4 *>(w + 32);            // o = j,      32 + u
                const float4 c1 = *reinterpret_cast<const float4 *>(w + 32 * kS2 + 32); // o = 32 + j, 32 + u
                const float A0[4] = {a0.x, a0.y, a0.z, a0.w}, A1[4] = {a1.x, a1.y, a1.z, a1.w};
                const float C0[4] = {c0.x, c0.y, c0.z, c0.w}, C1[4] = {c1.x, c1.y, c1.z, c1.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = 4 * rq + i;
                    y0 = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[i], h0[r], y0, 0, 0, 0);
                    y1 = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[i], h0[r], y1, 0, 0, 0);
                    y0 = __builtin_amdgcn_mfma_f32_32x32x2f32(C0[i], h1[r], y0, 0, 0, 0);
                    y1 = __builtin_amdgcn_mfma_f32_32x32x2f32(C1[i], h1[r], y1, 0, 0, 0);
                }
            }
        }
        // epilogue: + b2v + b2c (+ residual); lane holds units 32*ot + crow(r, half) of message j
        const float *b2v = lds + kOffBias + 64, *b2c = lds + kOffBias + 192, *wo = lds + kOffBias + 256;
        float part = 0.0f;
#pragma unroll
        for (int ot = 0; ot < 2; ++ot) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int o0 = 32 * ot + 8 * q + 4 * half;
                float4 v;
                float *vv = reinterpret_cast<float *>(&v);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float acc = ot == 0 ? y0[4 * q + i] : y1[4 * q + i];
                    vv[i] = (acc + b2v[o0 + i]) + b2c[o0 + i];
                }
                if (P.residual) {
                    const float4 xr = *reinterpret_cast<const float4 *>(P.x_in + rr * H + o0);
                    v.x += xr.x; v.y += xr.y; v.z += xr.z; v.w += xr.w;
                }
                if (P.last) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) part += vv[i] * wo[o0 + i];
                }
                if (ok && P.x_out) *reinterpret_cast<float4 *>(P.x_out + row * H + o0) = v;
            }
        }
        if (P.last) {
            part += __shfl_xor(part, 32, 64);
            if (ok && half == 0) P.msg_out[b * P.E + m] = part + bo;
        }
    }
}

// ------------------------------------------------------------------------ projected groups, H = 64
// The first Linear of each side takes [c; g] with g the mean of c over the message's group
// (message_gnn_decoder.py:106-118), so  W1 [c; g] + b1 = W1_left c + (W1_right g + b1).  The
// bracket is one row per GROUP: gnn_group_proj_kernel computes it once per group (1664 + 1344 rows
// per BG2 Z = 32 frame instead of 2 x 6304 per-message products) and the MLP starts its GEMM1
// accumulator from it, so GEMM1 runs over the 64 units of c only: 2/3 of the per-message MFMA work.
// A degree-1 var group's row is W1_right c of its own message, so no message needs a special case.
//
// gnn_group_proj_kernel: one wave per (frame, 32-group tile of one side): lane (j, half) sums units
// half*32 .. +31 of c over group j's members (ascending, as the group-mean kernels), scales by
// 1/|group| -- exactly the B operand of v_mfma_f32_32x32x2_f32 for K = 64 -- then 2 x 32 MFMAs
// against W1_right (LDS) and + b1.  Rows go to Mv / Mc (same shape as the group means).
// LDS (floats): W1vR [64][68], W1cR [64][68], b1v, b1c, w_in, b_in [64 each], emb [T][68].
constexpr int kPS = 68;
// F16 (default): W1_right g as scaled two-term f16 splits on v_mfma_f32_32x32x16_f16 (as the MLP's
// products, gnn_mlp2s_kernel): 24 MFMAs of 32 cycles per tile instead of 64 fp32 MFMAs of 64 cycles
// (+2.6 % on gnn-z32, profiles/r05/ab_r05pf16).  The images are W1vR (hi, lo), W1cR (hi, lo), rows of
// kPRow halves (16-B aligned, padded).  !F16 (weights whose rows span more than the split's range,
// LDPC_GNN_FP32_PRODUCTS): the fp32 images W1vR [64][68], W1cR [64][68] in the same region.
constexpr int kPRow = 72, kPImg = 64 * kPRow;
constexpr int kPOffB = 4 * kPImg / 2, kPOffEmb = kPOffB + 4 * 64;
constexpr int kPOffW1c = 64 * kPS;
static_assert(2 * 64 * kPS <= kPOffB, "the fp32 images fit the f16 images' region");
inline size_t proj_lds_bytes(int T, int waves) { return (size_t)(kPOffEmb + T * kPS + waves * 32 * kPS) * 4; }  // + 32 group means per wave

struct ProjTiles {
    const int4 *meta;
    const int32_t *grp, *deg, *mem;
    int n_tiles;
    int first;  // tiles before `first` are skipped (the var-side tiles, for the check side alone)
};

// GEN = false (the row walk's launches): the generic gather of typed member rows is compiled out.
// Under the row walk every tile takes another branch (check side: S_in; var side: memb_v; layer 0:
// the LLRs), and that branch's registers (two members x 8 groups x float4 rows and their types in
// flight) were what spilled the whole 12-wave kernel (20 VGPRs at the 168-VGPR budget).
template <int NT, bool HYB = false, bool F16 = true, bool GEN = true>
__global__ __launch_bounds__(NT, (NT == 256 ? LDPC_PROJ_WPS : 2)) void gnn_group_proj_kernel(GnnLayer P, ProjTiles T) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x;
    __shared__ int wmax_bits;
    int wexp = 0;
    _Float16 *pimg = reinterpret_cast<_Float16 *>(lds);
    if constexpr (F16) {
        // one power-of-two scale for both images: the largest |w| to at most 2^15
        if (tid == 0) wmax_bits = 0;
        __syncthreads();
        {
            float m = 0.0f;
            for (int i = tid; i < 64 * 64; i += NT)
                m = fmaxf(m, fmaxf(fabsf(P.w1v[(i >> 6) * 128 + 64 + (i & 63)]), fabsf(P.w1c[(i >> 6) * 128 + 64 + (i & 63)])));
            atomicMax(&wmax_bits, __float_as_int(m));
        }
        __syncthreads();
        wexp = min(col_exp(__int_as_float(wmax_bits)), 126);
        const float wsc = pow2f(wexp);
        for (int i = tid; i < 64 * 64; i += NT) {
            const int o = i >> 6, k = i & 63;
            split2h_store(P.w1v[o * 128 + 64 + k] * wsc, pimg + o * kPRow + k, kPImg);
            split2h_store(P.w1c[o * 128 + 64 + k] * wsc, pimg + 2 * kPImg + o * kPRow + k, kPImg);
        }
    } else {
        for (int i = tid; i < 64 * 64; i += NT) {
            const int o = i >> 6, k = i & 63;
            lds[o * kPS + k] = P.w1v[o * 128 + 64 + k];
            lds[kPOffW1c + o * kPS + k] = P.w1c[o * 128 + 64 + k];
        }
    }
    if (tid < 64) {
        lds[kPOffB + tid] = P.b1v[tid];
        lds[kPOffB + 64 + tid] = P.b1c[tid];
        lds[kPOffB + 128 + tid] = P.w_in[tid];
        lds[kPOffB + 192 + tid] = P.b_in[tid];
    }
    for (int i = tid; i < P.T * 64; i += NT) lds[kPOffEmb + (i >> 6) * kPS + (i & 63)] = P.emb[i];
    __syncthreads();
    const int lane = tid & 63, j = lane & 31, half = lane >> 5, wave = tid >> 6;
    // this wave's 32 group means, [32][68] after the shared image
    float *gm = lds + kPOffEmb + P.T * kPS + wave * 32 * kPS;
    const int c4 = 4 * (lane & 15), r4 = lane >> 4;
    const int nt = T.n_tiles - T.first;
    const int64_t ntiles = P.B * nt;
    const TileWalk tw = xcd_tiles(ntiles, NT / 64, wave);
    for (int64_t tt = tw.first; tt < tw.end; tt += tw.stride) {
        const int64_t b = tt / nt;
        const int t = T.first + (int)(tt - b * nt);
        const int4 md = T.meta[t];
        // group means, 16 lanes x 16 B per 256-B row: lane (r, c) owns units 4c .. 4c+3 of the tile's
        // groups 4p + r, p < 8, all eight summed side by side so that every lane keeps eight rows in
        // flight.  Per unit the members are summed in ascending order (x + emb first), x 1/|group|.
        int dg[8];
        float4 acc[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            dg[p] = T.deg[32 * t + 4 * p + r4];
            acc[p] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
        const int32_t *mem = T.mem + md.z + r4;
        if (md.x && P.S_in) {
            // check side after a row-walk MLP: the group's sum of feature rows is one row of S_in, so
            // the mean of c = x + emb over the group is S * inv + memb (the group's mean type
            // embedding) -- one 256-B row per group instead of a gather of its members
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const int slot = 4 * p + r4, g = T.grp[32 * t + slot];
                float4 mean = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (g >= 0) {
                    const float4 sv = *reinterpret_cast<const float4 *>(P.S_in + ((int64_t)b * P.Gc + g) * 64 + c4);
                    const float4 e = *reinterpret_cast<const float4 *>(P.memb + (int64_t)g * 64 + c4);
                    const float inv = P.inv_c[g];
                    mean = make_float4(sv.x * inv + e.x, sv.y * inv + e.y, sv.z * inv + e.z, sv.w * inv + e.w);
                    if (P.gsave_c) *reinterpret_cast<float4 *>(P.gsave_c + ((int64_t)b * P.Gc + g) * 64 + c4) = mean;
                }
                *reinterpret_cast<float4 *>(gm + slot * kPS + c4) = mean;
            }
        } else {
        if (P.x_in && P.memb_v && !md.x) {
            // var side: the members' x rows summed alone (no type gathers), then mean = sum * inv +
            // the group's mean type embedding; the member indices two rows ahead are loaded before
            // this pair's rows, so the rows' wait does not also wait for them
            const float *xb = P.x_in + (int64_t)b * P.E * 64 + c4;
            int mi[8], mj[8];
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                mi[p] = mem[4 * p];
                mj[p] = mem[32 + 4 * p];
            }
            for (int i = 0; i < md.y; i += 2) {
                int ni[8], nj[8];
                const int i2 = i + 2 < md.y ? i + 2 : i;  // the table holds maxdeg + 1 rows
#pragma unroll
                for (int p = 0; p < 8; ++p) {
                    ni[p] = mem[32 * i2 + 4 * p];
                    nj[p] = mem[32 * (i2 + 1) + 4 * p];
                }
                float4 x[8], y[8];
#pragma unroll
                for (int p = 0; p < 8; ++p) {
                    x[p] = *reinterpret_cast<const float4 *>(xb + (int64_t)mi[p] * 64);
                    y[p] = *reinterpret_cast<const float4 *>(xb + (int64_t)mj[p] * 64);
                }
#pragma unroll
                for (int p = 0; p < 8; ++p) {
                    if (i < dg[p]) { acc[p].x += x[p].x; acc[p].y += x[p].y; acc[p].z += x[p].z; acc[p].w += x[p].w; }
                    if (i + 1 < dg[p]) { acc[p].x += y[p].x; acc[p].y += y[p].y; acc[p].z += y[p].z; acc[p].w += y[p].w; }
                    mi[p] = ni[p];
                    mj[p] = nj[p];
                }
            }
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const int slot = 4 * p + r4, g = T.grp[32 * t + slot];
                float4 mean = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (g >= 0) {
                    const float inv = P.inv_v[g];
                    const float4 e = *reinterpret_cast<const float4 *>(P.memb_v + (int64_t)g * 64 + c4);
                    mean = make_float4(acc[p].x * inv + e.x, acc[p].y * inv + e.y, acc[p].z * inv + e.z, acc[p].w * inv + e.w);
                    if (P.gsave_v) *reinterpret_cast<float4 *>(P.gsave_v + ((int64_t)b * P.Gv + g) * 64 + c4) = mean;
                }
                *reinterpret_cast<float4 *>(gm + slot * kPS + c4) = mean;
            }
        } else {
        if (GEN && P.x_in) {
            const float *xb = P.x_in + (int64_t)b * P.E * 64 + c4;
            const float *eb = lds + kPOffEmb + c4;
            int mi[8], mj[8];
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                mi[p] = mem[4 * p];
                mj[p] = mem[32 + 4 * p];  // the table holds maxdeg + 1 rows (last one padding)
            }
            auto accum = [&](const float4 (&x)[8], const int (&ty)[8], int i) {
#pragma unroll
                for (int p = 0; p < 8; ++p) {
                    if (i < dg[p]) {
                        const float4 e = *reinterpret_cast<const float4 *>(eb + ty[p] * kPS);
                        acc[p].x += x[p].x + e.x; acc[p].y += x[p].y + e.y;
                        acc[p].z += x[p].z + e.z; acc[p].w += x[p].w + e.w;
                    }
                }
            };
            for (int i = 0; i < md.y; i += 2) {  // two members of all eight groups in flight
                float4 x[8], y[8];
                int tx[8], tyy[8];
#pragma unroll
                for (int p = 0; p < 8; ++p) {
                    x[p] = *reinterpret_cast<const float4 *>(xb + (int64_t)mi[p] * 64);
                    y[p] = *reinterpret_cast<const float4 *>(xb + (int64_t)mj[p] * 64);
                    tx[p] = P.msg_type[mi[p]];
                    tyy[p] = P.msg_type[mj[p]];
                }
                if (HYB && P.hv2c) {  // hybrid: x = (v2c w_in + b_in) + F
                    const float *vb = P.hv2c + (int64_t)b * P.E;
                    const float4 w = *reinterpret_cast<const float4 *>(lds + kPOffB + 128 + c4);
                    const float4 c = *reinterpret_cast<const float4 *>(lds + kPOffB + 192 + c4);
#pragma unroll
                    for (int p = 0; p < 8; ++p) {
                        x[p] = hyb_x(x[p], vb[mi[p]], w, c);
                        y[p] = hyb_x(y[p], vb[mj[p]], w, c);
                    }
                }
                if (i + 2 < md.y) {
#pragma unroll
                    for (int p = 0; p < 8; ++p) {
                        mi[p] = mem[32 * (i + 2) + 4 * p];
                        mj[p] = mem[32 * (i + 3) + 4 * p];
                    }
                }
                accum(x, tx, i);
                accum(y, tyy, i + 1);
            }
        } else {
            const float4 w = *reinterpret_cast<const float4 *>(lds + kPOffB + 128 + c4);
            const float4 bi = *reinterpret_cast<const float4 *>(lds + kPOffB + 192 + c4);
            for (int i = 0; i < md.y; ++i) {
#pragma unroll
                for (int p = 0; p < 8; ++p) {
                    if (i < dg[p]) {
                        const int m = mem[32 * i + 4 * p];
                        const float l = P.llr[(int64_t)b * P.N + P.msg_var[m]];
                        const float4 e = *reinterpret_cast<const float4 *>(lds + kPOffEmb + P.msg_type[m] * kPS + c4);
                        acc[p].x += (l * w.x + bi.x) + e.x; acc[p].y += (l * w.y + bi.y) + e.y;  // Linear(1, H) + emb
                        acc[p].z += (l * w.z + bi.z) + e.z; acc[p].w += (l * w.w + bi.w) + e.w;
                    }
                }
            }
        }
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int slot = 4 * p + r4, g = T.grp[32 * t + slot];
            const float inv = g >= 0 ? (md.x ? P.inv_c : P.inv_v)[g] : 0.0f;
            const float4 mean = make_float4(acc[p].x * inv, acc[p].y * inv, acc[p].z * inv, acc[p].w * inv);
            *reinterpret_cast<float4 *>(gm + slot * kPS + c4) = mean;
            if (P.gsave_v && g >= 0)
                *reinterpret_cast<float4 *>((md.x ? P.gsave_c + ((int64_t)b * P.Gc + g) * 64
                                                  : P.gsave_v + ((int64_t)b * P.Gv + g) * 64) + c4) = mean;
        }
        }
        }
        __builtin_amdgcn_wave_barrier();
        f32x16 h0 = {}, h1 = {};
        if constexpr (F16) {
        // B operand of k-step s: lane (j, half) <- group j's units 16 s + 8 half .. + 7, scaled by a
        // power of two (the group's largest |g| to at most 2^15); the accumulators are scaled back
        float4 gv[8];
        float gmx = 0.0f;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            gv[q] = *reinterpret_cast<const float4 *>(gm + j * kPS + 16 * (q >> 1) + 8 * half + 4 * (q & 1));
            gmx = fmaxf(gmx, fmaxf(fmaxf(fabsf(gv[q].x), fabsf(gv[q].y)), fmaxf(fabsf(gv[q].z), fabsf(gv[q].w))));
        }
        __builtin_amdgcn_wave_barrier();
        gmx = fmaxf(gmx, __shfl_xor(gmx, 32, 64));
        const int gexp = col_exp_w(gmx, wexp);
        const float gsc = pow2f(gexp), igsc = pow2f(-gexp - wexp);
        const _Float16 *Wi = pimg + (md.x ? 2 * kPImg : 0) + j * kPRow + 8 * half;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float4 a = gv[2 * s], c = gv[2 * s + 1];
            const float v[8] = {a.x * gsc, a.y * gsc, a.z * gsc, a.w * gsc, c.x * gsc, c.y * gsc, c.z * gsc, c.w * gsc};
            f16x8_t b0, b1;
            split2h(v, b0, b1);
            h0 = mfma3h(Wi + 16 * s, b0, b1, h0, kPImg);
            h1 = mfma3h(Wi + 32 * kPRow + 16 * s, b0, b1, h1, kPImg);
        }
        h0 *= igsc;
        h1 *= igsc;
        } else {
        // B operand: lane (j, half) <- group j's units 8 q + 4 half + i (q < 8)
        float g32[32];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float4 v = *reinterpret_cast<const float4 *>(gm + j * kPS + 8 * q + 4 * half);
            g32[4 * q] = v.x; g32[4 * q + 1] = v.y; g32[4 * q + 2] = v.z; g32[4 * q + 3] = v.w;
        }
        __builtin_amdgcn_wave_barrier();
        const float *W = lds + (md.x ? kPOffW1c : 0);
        int wl = j * kPS + 4 * half;  // step kk + i pairs unit 8 (kk/4) + i (half 0) with + 4 (half 1)
        asm volatile("" : "+v"(wl));
#pragma unroll
        for (int kk = 0; kk < 32; kk += 4) {
            const float4 wa = *reinterpret_cast<const float4 *>(W + wl + 2 * kk);
            const float4 wb = *reinterpret_cast<const float4 *>(W + wl + 32 * kPS + 2 * kk);
            const float a4[4] = {wa.x, wa.y, wa.z, wa.w}, b4[4] = {wb.x, wb.y, wb.z, wb.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                h0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[i], g32[kk + i], h0, 0, 0, 0);
                h1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b4[i], g32[kk + i], h1, 0, 0, 0);
            }
        }
        }
        const int g = T.grp[32 * t + j];
        if (g < 0) continue;
        const float *b1 = lds + kPOffB + 64 * md.x;
        float *dst = md.x ? P.Mc + ((int64_t)b * P.Gc + g) * 64 : P.Mv + ((int64_t)b * P.Gv + g) * 64;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int u = 8 * q + 4 * half;  // registers 4q .. 4q+3 hold units crow(4q + i, half) = u + i
            *reinterpret_cast<float4 *>(dst + u) =
                make_float4(h0[4 * q] + b1[u], h0[4 * q + 1] + b1[u + 1], h0[4 * q + 2] + b1[u + 2], h0[4 * q + 3] + b1[u + 3]);
            *reinterpret_cast<float4 *>(dst + 32 + u) =
                make_float4(h1[4 * q] + b1[32 + u], h1[4 * q + 1] + b1[33 + u], h1[4 * q + 2] + b1[34 + u],
                            h1[4 * q + 3] + b1[35 + u]);
        }
    }
}

// ------------------------------------------------------------------------ MLP over projected groups
// As gnn_mlp_mfma_kernel, but GEMM1 is W1_left c (K = 64: lane half h carries units 32 h .. +31 of
// c, one k of each half per MFMA step) started from the message's projected group rows (above),
// and nothing else changes: ReLU, GEMM2 of both sides into one accumulator, b2v + b2c, residual,
// output projection.  Per 32-message tile 2 x (64 + 64) MFMAs instead of 2 x (128 + 64).
// LDS (floats): W1vL [64][68], W1cL, W2v [64][68], W2c, then b2v, b2c, wo [64 each], emb [T][68].
constexpr int kM2OffW1c = 64 * kPS, kM2OffW2v = 2 * 64 * kPS, kM2OffW2c = 3 * 64 * kPS;
constexpr int kM2OffB = 4 * 64 * kPS, kM2OffEmb = kM2OffB + 3 * 64;
inline size_t mlp2_lds_bytes(int T) { return (size_t)(kM2OffEmb + T * kPS) * 4; }

template <int NT, int WPS, bool HYB = false>
__global__ __launch_bounds__(NT, WPS) void gnn_mlp2_kernel(GnnLayer P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x;
    for (int i = tid; i < 64 * 64; i += NT) {
        const int o = i >> 6, k = i & 63;
        lds[o * kPS + k] = P.w1v[o * 128 + k];
        lds[kM2OffW1c + o * kPS + k] = P.w1c[o * 128 + k];
        lds[kM2OffW2v + o * kPS + k] = P.w2v[i];
        lds[kM2OffW2c + o * kPS + k] = P.w2c[i];
    }
    if (tid < 64) {
        lds[kM2OffB + tid] = P.vside ? P.b2v[tid] : 0.0f;
        lds[kM2OffB + 64 + tid] = P.b2c[tid];
        lds[kM2OffB + 128 + tid] = P.last ? P.wo[tid] : 0.0f;
    }
    for (int i = tid; i < P.T * 64; i += NT) lds[kM2OffEmb + (i >> 6) * kPS + (i & 63)] = P.emb[i];
    __syncthreads();

    const int lane = tid & 63, j = lane & 31, half = lane >> 5, wave = tid >> 6;
    const int64_t R = P.B * P.E;
    const int64_t ntiles = (R + 31) / 32;
    const float bo = P.last ? P.bo[0] : 0.0f;
    const TileWalk tw = xcd_tiles(ntiles, NT / 64, wave);
    for (int64_t t = tw.first; t < tw.end; t += tw.stride) {
        const int64_t row = t * 32 + j;
        const bool ok = row < R;
        const int64_t rr = ok ? row : R - 1;
        const int64_t b = rr / P.E, m = rr - b * P.E;
        float in[32];
        {
            // lane half h carries units 8 q + 4 h + i (float4 chunk 2 q + h of the row)
            const float *e = lds + kM2OffEmb + P.msg_type[m] * kPS + 4 * half;
            if (P.x_in) {
                const float *xr = P.x_in + rr * 64 + 4 * half;
                const float hv = HYB && P.hv2c ? P.hv2c[rr] : 0.0f;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    float4 v = *reinterpret_cast<const float4 *>(xr + 8 * q);
                    if (HYB && P.hv2c)  // hybrid: x = (v2c w_in + b_in) + F
                        v = hyb_x(v, hv, *reinterpret_cast<const float4 *>(P.w_in + 8 * q + 4 * half),
                                  *reinterpret_cast<const float4 *>(P.b_in + 8 * q + 4 * half));
                    in[4 * q + 0] = v.x + e[8 * q + 0];
                    in[4 * q + 1] = v.y + e[8 * q + 1];
                    in[4 * q + 2] = v.z + e[8 * q + 2];
                    in[4 * q + 3] = v.w + e[8 * q + 3];
                }
            } else {
                const float l = P.llr[b * P.N + P.msg_var[m]];
#pragma unroll
                for (int k = 0; k < 32; ++k) {
                    const int u = 8 * (k >> 2) + 4 * half + (k & 3);
                    in[k] = (l * P.w_in[u] + P.b_in[u]) + e[8 * (k >> 2) + (k & 3)];
                }
            }
        }
        const float *pv = P.Mv + (b * P.Gv + P.vgroup[m]) * 64 + 4 * half;
        const float *pc = P.Mc + (b * P.Gc + P.cgroup[m]) * 64 + 4 * half;
        f32x16 y0 = {}, y1 = {};
        int w1lane = j * kPS + 4 * half, w2lane = j * kPS + 4 * half;
        asm volatile("" : "+v"(w1lane), "+v"(w2lane));
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            if (side == 0 && !P.vside) continue;
            const float *pr = side == 0 ? pv : pc;
            f32x16 h0, h1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // registers 4q .. 4q+3 <-> units 8q + 4 half + i (+ 32 for h1)
                const float4 a = *reinterpret_cast<const float4 *>(pr + 8 * q);
                const float4 c = *reinterpret_cast<const float4 *>(pr + 32 + 8 * q);
                h0[4 * q] = a.x; h0[4 * q + 1] = a.y; h0[4 * q + 2] = a.z; h0[4 * q + 3] = a.w;
                h1[4 * q] = c.x; h1[4 * q + 1] = c.y; h1[4 * q + 2] = c.z; h1[4 * q + 3] = c.w;
            }
            const float *W1 = lds + (side == 0 ? 0 : kM2OffW1c);
            const float *W2 = lds + (side == 0 ? kM2OffW2v : kM2OffW2c);
#pragma unroll
            for (int kk = 0; kk < 32; kk += 4) {
                const float4 wa = *reinterpret_cast<const float4 *>(W1 + w1lane + 2 * kk);
                const float4 wb = *reinterpret_cast<const float4 *>(W1 + w1lane + 32 * kPS + 2 * kk);
                const float a4[4] = {wa.x, wa.y, wa.z, wa.w}, b4[4] = {wb.x, wb.y, wb.z, wb.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    h0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[i], in[kk + i], h0, 0, 0, 0);
                    h1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b4[i], in[kk + i], h1, 0, 0, 0);
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                h0[r] = relu_nan(h0[r]);
                h1[r] = relu_nan(h1[r]);
            }
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                const float *w = W2 + w2lane + 8 * rq;
                const float4 a0 = *reinterpret_cast<const float4 *>(w);
                const float4 a1 = *reinterpret_cast<const float4 *>(w + 32 * kPS);
                const float4 c0 = *reinterpret_cast<const float4 *>(w + 32);
                const float4 c1 = *reinterpret_cast<const float4 *>(w + 32 * kPS + 32);
                const float A0[4] = {a0.x, a0.y, a0.z, a0.w}, A1[4] = {a1.x, a1.y, a1.z, a1.w};
                const float C0[4] = {c0.x, c0.y, c0.z, c0.w}, C1[4] = {c1.x, c1.y, c1.z, c1.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = 4 * rq + i;
                    y0 = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[i], h0[r], y0, 0, 0, 0);
                    y1 = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[i], h0[r], y1, 0, 0, 0);
                    y0 = __builtin_amdgcn_mfma_f32_32x32x2f32(C0[i], h1[r], y0, 0, 0, 0);
                    y1 = __builtin_amdgcn_mfma_f32_32x32x2f32(C1[i], h1[r], y1, 0, 0, 0);
                }
            }
        }
        const float *b2v = lds + kM2OffB, *b2c = lds + kM2OffB + 64, *wo = lds + kM2OffB + 128;
        float part = 0.0f;
#pragma unroll
        for (int ot = 0; ot < 2; ++ot) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int o0 = 32 * ot + 8 * q + 4 * half;
                float4 v;
                float *vv = reinterpret_cast<float *>(&v);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float acc = ot == 0 ? y0[4 * q + i] : y1[4 * q + i];
                    vv[i] = (acc + b2v[o0 + i]) + b2c[o0 + i];
                }
                if (P.residual) {
                    const float4 xr = *reinterpret_cast<const float4 *>(P.x_in + rr * 64 + o0);
                    v.x += xr.x; v.y += xr.y; v.z += xr.z; v.w += xr.w;
                }
                if (P.last) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) part += vv[i] * wo[o0 + i];
                }
                if (ok && P.x_out) *reinterpret_cast<float4 *>(P.x_out + row * 64 + o0) = v;
            }
        }
        if (P.last) {
            part += __shfl_xor(part, 32, 64);
            if (ok && half == 0) P.msg_out[b * P.E + m] = part + bo;
        }
    }
}


// ------------------------------------------------------------------------ MLP over projected groups, fp32 by split MFMAs
// Default (LDPC_S6_F16, round 5): scaled two-term f16 splits.  The weights are scaled by one power of
// two (largest |w| to at most 2^15), each message's activation column by another (its largest
// |value|, bounded by max |x| + max |emb[type]| for GEMM1 and by max relu(h) over both sides for
// GEMM2), so v = v0 + v1 with v0 = f16(v), v1 = f16(v - v0) holds 22 significant bits in the f16
// normal range, and a product is a1 b0 + a0 b1 + a0 b0 on v_mfma_f32_32x32x16_f16 (the dropped a1 b1
// is below 2^-22 of the column's largest product); the accumulators start from the scaled additive
// term and are scaled back exactly after the GEMM.  3 MFMAs per K = 16 instead of 6: 61.4-61.6 k vs
// 57.0-57.2 k cw/s on cfg4 (profiles/r05/ab_r05f16e); test_split_mlp_is_fp32_accurate holds its bar
// (error against the float64 oracle within 2x of an fp32 GEMM's).  The bf16x6 form below remains the
// LDPC_S6_F16=0 build:
// gnn_mlp2_kernel's math with every fp32 product on v_mfma_f32_32x32x16_bf16: each fp32 operand is
// split into three bf16 terms, v = v0 + v1 + v2 (v0 = bf16(v), v1 = bf16(v - v0), v2 = bf16(v - v0 -
// v1): 24 significant bits, every subtraction exact), and a product a b is the six terms
// a2 b0 + a1 b1 + a0 b2 + a1 b0 + a0 b1 + a0 b0 (the dropped ones are below 2^-24 |a b|), each exact
// in the fp32 accumulator.  The result is an fp32 GEMM up to summation order -- the same class of
// difference as between any two fp32 GEMMs -- at 6 x 32 instead of 8 x 64 MFMA cycles per K = 16
// (2.67x less matrix time).  Weights: three split images per matrix in LDS (bf16, 72-element rows,
// conflict-free ds_read_b128); activations (c for GEMM1, relu(h) for GEMM2) are split in registers.
// K order: GEMM1's k-step s, lane half h, element i is unit pi16(16 s + 8 h + i) =
// 32 (s>>1) + 16 (s&1) + 8 (i>>2) + 4 h + (i&3), which is the unit that lane owns in register
// 8 (s&1) + i of accumulator tile s>>1: so GEMM2's B operand is GEMM1's accumulator as it stands,
// and the x values loaded for GEMM1 are the residual the lane adds to its output registers.
// LDPC_S6_F16 (default): the MLP's fp32 products as scaled two-term f16 splits (3 MFMAs per product)
// instead of three-term bf16 splits (6); LDPC_S6_PCEARLY: the check side's projected row seeds the
// accumulators (the f16 kernel's registers have no room for the late add)
#ifndef LDPC_S6_F16
#define LDPC_S6_F16 1
#endif
#ifndef LDPC_S6_PCEARLY
#define LDPC_S6_PCEARLY LDPC_S6_F16
#endif
#if LDPC_S6_F16
typedef _Float16 s6_t;
typedef f16x8_t s6x8_t;
constexpr int kS6Split = 2;
#else
typedef __bf16 s6_t;
typedef bf16x8_t s6x8_t;
constexpr int kS6Split = 3;
#endif
// LDPC_S6_PCLDS (default): the row walk copies its unit's 32 projected check rows into LDS at the
// unit's first tile (lane-private slots), so the unit's other tiles do not re-read them from L2,
// where the walk's streaming rows have long evicted them (+7.1 % on gnn-z32, profiles/r05/ab_r05pcl);
// it needs the swizzled unpadded weight images (LDPC_S6_SW) to fit 160 KB
#ifndef LDPC_S6_PCLDS
#define LDPC_S6_PCLDS 1
#endif
#ifndef LDPC_S6_SW
#define LDPC_S6_SW LDPC_S6_PCLDS
#endif
#if LDPC_S6_SW
constexpr int kS6Row = 64;                                         // elements per image row
#else
constexpr int kS6Row = 72;                                         // elements per image row
#endif
constexpr int kS6Img = 64 * kS6Row;                                // elements per split image
// element (row o, column p) of a split image: padded rows, or 128-B rows whose 16-B chunks are
// XOR-swizzled by row pair (a fragment read's 16 lanes then cover all 64 banks)
__host__ __device__ constexpr int s6_at(int o, int p) {
#if LDPC_S6_SW
    return o * 64 + ((((p >> 3) ^ ((o >> 1) & 7))) << 3) + (p & 7);
#else
    return o * kS6Row + p;
#endif
}
constexpr int kS6OffW2 = 2 * kS6Split * kS6Img;                    // W1L (side, split), then W2
constexpr int kS6Bytes = 4 * kS6Split * kS6Img * 2;                // 4 matrices x kS6Split images
constexpr int kS6OffB = kS6Bytes / 4;                              // floats: b2v, b2c, wo
constexpr int kS6OffEmb = kS6OffB + 3 * 64;                        // floats: emb [T][kPS]
// then, with degree-1 tiles (GnnLayer tperm), the three split images of W1v_left + W1v_right
// (f16 splits: then max |emb[t]| per type, T floats)
__host__ __device__ inline int s6_off_d1(int T) { return ((kS6OffEmb + T * kPS + T) * 4 + 15) / 16 * 16; }
inline size_t mlp2s_lds_bytes(int T, bool d1) { return (size_t)s6_off_d1(T) + (d1 ? kS6Split * kS6Img * 2 : 0); }
// row walk with LDPC_S6_PCLDS: after the degree-1 image's slot, 8 KB per wave of staged check rows
__host__ __device__ inline int s6_off_pc(int T) { return s6_off_d1(T) + kS6Split * kS6Img * 2; }
inline size_t mlp2s_rw_lds_bytes(int T, bool d1, int waves) {
    return LDPC_S6_PCLDS ? (size_t)s6_off_pc(T) + (size_t)waves * 32 * 64 * 4 : mlp2s_lds_bytes(T, d1);
}

// Degree-1 tiles (tperm set, var side): a degree-1 var group's mean is the message's own c, so
// W1v [c; g] = (W1v_left + W1v_right) c -- one fp32 sum per weight, rounded once and split like the
// other weights -- and GEMM1 starts from b1v instead of a projected row, which the projection
// kernel then does not write for those groups (ProjTiles first = n_ptiles_v1).
// PCL (row walk only): the units' check rows staged in LDS (LDPC_S6_PCLDS, when the LDS has room)
template <int NT, int WPS, bool HYB = false, bool RW = false, bool PCL = false>
__global__ __launch_bounds__(NT, WPS) void gnn_mlp2s_kernel(GnnLayer P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    s6_t *img = reinterpret_cast<s6_t *>(lds);
    const int tid = threadIdx.x;
    const bool d1img = (P.tperm || RW) && P.ntile_v1 && P.vside;  // the combined image, when degree-1 tiles exist
#if LDPC_S6_F16
    // one power-of-two scale for every weight image: the largest |w| to at most 2^15
    __shared__ int wmax_bits;
    if (tid == 0) wmax_bits = 0;
    __syncthreads();
    {
        float m = 0.0f;
        for (int i = tid; i < 64 * 64; i += NT) {
            const int o = i >> 6, u = i & 63;
            m = fmaxf(m, fmaxf(fmaxf(fabsf(P.w1v[o * 128 + u]), fabsf(P.w1c[o * 128 + u])),
                               fmaxf(fabsf(P.w2v[o * 64 + u]), fabsf(P.w2c[o * 64 + u]))));
            if (d1img) m = fmaxf(m, fabsf(P.w1v[o * 128 + u] + P.w1v[o * 128 + 64 + u]));
        }
        atomicMax(&wmax_bits, __float_as_int(m));
    }
    __syncthreads();
    const int wexp = min(col_exp(__int_as_float(wmax_bits)), 126);
    const float wsc = pow2f(wexp);
#endif
    for (int i = tid; i < 64 * 64; i += NT) {
        const int o = i >> 6, p = i & 63, u = pi16(p);
        const float w[4] = {P.w1v[o * 128 + u], P.w1c[o * 128 + u], P.w2v[o * 64 + u], P.w2c[o * 64 + u]};
#pragma unroll
        for (int q = 0; q < 4; ++q)  // q: W1v, W1c, W2v, W2c -> images kS6Split q ..
#if LDPC_S6_F16
            split2h_store(w[q] * wsc, img + 2 * q * kS6Img + s6_at(o, p), kS6Img);
#else
            split_store(w[q], img + 3 * q * kS6Img + s6_at(o, p), kS6Img);
#endif
    }
    s6_t *img_d1 = reinterpret_cast<s6_t *>(reinterpret_cast<char *>(lds) + s6_off_d1(P.T));
    if (d1img)
        for (int i = tid; i < 64 * 64; i += NT) {
            const int o = i >> 6, p = i & 63, u = pi16(p);
#if LDPC_S6_F16
            split2h_store((P.w1v[o * 128 + u] + P.w1v[o * 128 + 64 + u]) * wsc, img_d1 + s6_at(o, p), kS6Img);
#else
            split_store(P.w1v[o * 128 + u] + P.w1v[o * 128 + 64 + u], img_d1 + s6_at(o, p), kS6Img);
#endif
        }
    if (tid < 64) {
        lds[kS6OffB + tid] = (P.vside ? P.b2v[tid] : 0.0f) + P.b2c[tid];  // both output biases
        lds[kS6OffB + 64 + tid] = P.b2c[tid];
        lds[kS6OffB + 128 + tid] = P.last ? P.wo[tid] : 0.0f;
    }
    // emb rows kPS = 68 floats apart: lanes of different types read different rows (64 apart, every
    // row would sit on the same banks)
    for (int i = tid; i < P.T * 64; i += NT) lds[kS6OffEmb + (i >> 6) * kPS + (i & 63)] = P.emb[i];
#if LDPC_S6_F16
    for (int t = tid; t < P.T; t += NT) {  // max |emb[t]|: |c| <= max |x| + this bounds a column's scale
        float m = 0.0f;
        for (int u = 0; u < 64; ++u) m = fmaxf(m, fabsf(P.emb[t * 64 + u]));
        lds[kS6OffEmb + P.T * kPS + t] = m;
    }
#endif
    __syncthreads();

    const int lane = tid & 63, j = lane & 31, half = lane >> 5, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: the walk's indices in SGPRs
    const float bo = P.last ? P.bo[0] : 0.0f;
    // A fragment of row j (+ 32 kS6Row: rows 32 .., whose swizzle equals row j's), k-step s
    auto aof = [&](int s) { return s6_at(j, 16 * s + 8 * half); };
    const bool vs = HYB ? P.vside != 0 : true;  // the var side (only the hybrid kernel runs without it)
    float S[32];  // row walk: this lane's check's running sum of output rows (its half's 32 units)

    // A tile's features before the type embedding: x[s][i] = feature pi16(16 s + 8 h + i) of row rr
    // (float4 pairs), or layer 0's input embedding of the message's LLR.
    auto load_x = [&](float (&x)[4][8], int64_t b, int64_t m, int64_t rr) {
        if (P.x_in) {
            const float *xr = P.x_in + rr * 64 + 4 * half;
            const float hv = HYB && P.hv2c ? P.hv2c[rr] : 0.0f;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int u0 = 32 * (s >> 1) + 16 * (s & 1) + 8 * q;  // + 4 half (in xr)
                    float4 v = *reinterpret_cast<const float4 *>(xr + u0);
                    if (HYB && P.hv2c)
                        v = hyb_x(v, hv, *reinterpret_cast<const float4 *>(P.w_in + u0 + 4 * half),
                                  *reinterpret_cast<const float4 *>(P.b_in + u0 + 4 * half));
                    x[s][4 * q] = v.x; x[s][4 * q + 1] = v.y; x[s][4 * q + 2] = v.z; x[s][4 * q + 3] = v.w;
                }
            }
        } else {
            const float l = P.llr[b * P.N + P.msg_var[m]];
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int u = pi16(16 * s + 8 * half + i);
                    x[s][i] = l * P.w_in[u] + P.b_in[u];
                }
        }
    };
    // a projected group row, as the lane's accumulator registers: r[t][4 q + i] = unit 32 t + 8 q + 4 h + i
    auto load_acc = [](f32x16 (&r)[2], const float *p) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 a = *reinterpret_cast<const float4 *>(p + 8 * q);
            const float4 c = *reinterpret_cast<const float4 *>(p + 32 + 8 * q);
            r[0][4 * q] = a.x; r[0][4 * q + 1] = a.y; r[0][4 * q + 2] = a.z; r[0][4 * q + 3] = a.w;
            r[1][4 * q] = c.x; r[1][4 * q + 1] = c.y; r[1][4 * q + 2] = c.z; r[1][4 * q + 3] = c.w;
        }
    };

    // One 32-message tile: slot j is message m of frame b (row rr of x); ok = a real message (a padding
    // slot computes on a valid row and writes nothing); d1t = a degree-1 var tile; pc = the slot's
    // projected check row (+ 4 half); x = the tile's features (load_x), typ = its message type, pv = its
    // var side's starting accumulators (the projected group row W1v_right g + b1v, or b1v on a degree-1
    // tile).  Row walk (RW): the tile also loads the NEXT tile's x (row xn, once GEMM1 has read
    // this tile's) and var-side row (frame bn, var group vgn, degree-1 d1n; once GEMM2 has consumed
    // this tile's var side) into x and pv, so their latency hides under this tile's MFMAs.
    auto tile = [&](int64_t b, int64_t m, int64_t rr, bool ok, const float *pc, float (&x)[4][8], int typ,
                    f32x16 (&pv)[2], bool d1t, const float *xn, int64_t bn, int vgn, bool d1n, int pcm) {
        const float *e = lds + kS6OffEmb + typ * kPS;
        // the per-walk constants are re-read from LDS at every tile (an opaque offset: hoisted out of the
        // walk they would hold 64 VGPRs)
        int boff = kS6OffB;
        asm volatile("" : "+s"(boff));
        const float *b2 = lds + boff, *wo = lds + boff + 128;
        // GEMM1 of both sides per k-step over one split of c (c = x + emb[type] is the same for
        // both); the var side's accumulators start from its projected group row W1_right g + b1
        f32x16 hs[2][2];
        hs[0][0] = pv[0];
        hs[0][1] = pv[1];
#if LDPC_S6_PCEARLY
#if LDPC_S6_PCLDS
        // pcm (uniform): 0 = the check row from global, else from the lane's LDS slots, which the row
        // walk fills at the unit's first tile (float4 q of lane l at pcs[64 q + l]: conflict-free)
        if (PCL && pcm) {
            const float4 *pcs = reinterpret_cast<const float4 *>(reinterpret_cast<const char *>(lds) + s6_off_pc(P.T)) + wave * 512 + lane;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 a = pcs[64 * q], c = pcs[64 * (4 + q)];
                hs[1][0][4 * q] = a.x; hs[1][0][4 * q + 1] = a.y; hs[1][0][4 * q + 2] = a.z; hs[1][0][4 * q + 3] = a.w;
                hs[1][1][4 * q] = c.x; hs[1][1][4 * q + 1] = c.y; hs[1][1][4 * q + 2] = c.z; hs[1][1][4 * q + 3] = c.w;
            }
        } else {
            load_acc(hs[1], pc);
        }
#else
        load_acc(hs[1], pc);
#endif
#else
        // the check side's projected row is added after GEMM1 (its load lands under the MFMAs)
        f32x16 pcr[2];
        load_acc(pcr, pc);
        hs[1][0] = f32x16{};
        hs[1][1] = f32x16{};
#endif
        const s6_t *W1v = d1t ? img_d1 : img, *W1c = img + kS6Split * kS6Img;
#if LDPC_S6_F16
        // the message's c scaled by a power of two (its largest |c| to at most 2^15), the
        // accumulators by that times the weights' scale: products of scaled two-term f16 splits
        float cm = 0.0f;
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < 8; ++i) cm = fmaxf(cm, fabsf(x[s][i]));
        cm = fmaxf(cm, __shfl_xor(cm, 32, 64)) + lds[kS6OffEmb + P.T * kPS + typ];  // >= max |c|
        const int cexp = col_exp_w(cm, wexp);
        const float csc = pow2f(cexp), asc = pow2f(cexp + wexp), iasc = pow2f(-cexp - wexp);
        hs[0][0] *= asc;
        hs[0][1] *= asc;
#if LDPC_S6_PCEARLY
        hs[1][0] *= asc;
        hs[1][1] *= asc;
#endif
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            float c[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) c[i] = (x[s][i] + e[pi16(16 * s + 8 * half + i)]) * csc;
            s6x8_t c0, c1;
            split2h(c, c0, c1);
            if (vs) {
                hs[0][0] = mfma3h(W1v + aof(s), c0, c1, hs[0][0], kS6Img);
                hs[0][1] = mfma3h(W1v + 32 * kS6Row + aof(s), c0, c1, hs[0][1], kS6Img);
            }
            hs[1][0] = mfma3h(W1c + aof(s), c0, c1, hs[1][0], kS6Img);
            hs[1][1] = mfma3h(W1c + 32 * kS6Row + aof(s), c0, c1, hs[1][1], kS6Img);
            __builtin_amdgcn_sched_barrier(0);
        }
        hs[0][0] *= iasc;
        hs[0][1] *= iasc;
        hs[1][0] *= iasc;
        hs[1][1] *= iasc;
#else
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            float c[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) c[i] = x[s][i] + e[pi16(16 * s + 8 * half + i)];
            bf16x8_t c0, c1, c2;
            split3(c, c0, c1, c2);
            if (vs) {
                hs[0][0] = mfma6(W1v + aof(s), c0, c1, c2, hs[0][0], kS6Img);
                hs[0][1] = mfma6(W1v + 32 * kS6Row + aof(s), c0, c1, c2, hs[0][1], kS6Img);
            }
            hs[1][0] = mfma6(W1c + aof(s), c0, c1, c2, hs[1][0], kS6Img);
            hs[1][1] = mfma6(W1c + 32 * kS6Row + aof(s), c0, c1, c2, hs[1][1], kS6Img);
            __builtin_amdgcn_sched_barrier(0);  // one k-step's A fragments live at a time (VGPRs)
        }
#endif
#if !LDPC_S6_PCEARLY
        hs[1][0] += pcr[0];
        hs[1][1] += pcr[1];
#endif
        // GEMM2's accumulators start from the residual and the output biases: register 4 q + i of
        // tile ot is unit 32 ot + 8 q + 4 half + i = x[2 ot + (q >> 1)][4 (q & 1) + i]
        f32x16 y0, y1;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int o = 8 * q + 4 * half + i;
                y0[4 * q + i] = (P.residual ? x[q >> 1][4 * (q & 1) + i] : 0.0f) + b2[o];
                y1[4 * q + i] = (P.residual ? x[2 + (q >> 1)][4 * (q & 1) + i] : 0.0f) + b2[32 + o];
            }
        if constexpr (RW) {  // x is consumed: the next tile's (layer 0 computes its x at the tile)
            if (P.x_in)
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        const float4 v = *reinterpret_cast<const float4 *>(xn + 32 * (s >> 1) + 16 * (s & 1) + 8 * q);
                        x[s][4 * q] = v.x; x[s][4 * q + 1] = v.y; x[s][4 * q + 2] = v.z; x[s][4 * q + 3] = v.w;
                    }
        }
#if LDPC_S6_F16
        // both sides' relu(h) under one column scale (they accumulate into the same y)
        float hm = 0.0f;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            if (side == 0 && !vs) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) hm = fmaxf(hm, fmaxf(hs[side][0][r], hs[side][1][r]));
        }
        hm = fmaxf(hm, __shfl_xor(hm, 32, 64));  // >= 0: the largest relu(h)
        const int hexp = col_exp_w(hm, wexp);
        const float hsc = pow2f(hexp), ysc = pow2f(hexp + wexp), iysc = pow2f(-hexp - wexp);
        y0 *= ysc;
        y1 *= ysc;
#endif
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            if (side == 0 && !vs) continue;
            const f32x16 &h0 = hs[side][0], &h1 = hs[side][1];
            const s6_t *W2 = img + kS6OffW2 + kS6Split * side * kS6Img;
#pragma unroll
            for (int s = 0; s < 4; ++s) {  // GEMM2: y += W2 relu(h); k-step s = registers 8 (s&1) .. of h_{s>>1}
                float hr[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) hr[i] = relu_nan(s < 2 ? h0[8 * (s & 1) + i] : h1[8 * (s & 1) + i]);
#if LDPC_S6_F16
#pragma unroll
                for (int i = 0; i < 8; ++i) hr[i] *= hsc;
                s6x8_t r0, r1;
                split2h(hr, r0, r1);
                y0 = mfma3h(W2 + aof(s), r0, r1, y0, kS6Img);
                y1 = mfma3h(W2 + 32 * kS6Row + aof(s), r0, r1, y1, kS6Img);
#else
                bf16x8_t r0, r1, r2;
                split3(hr, r0, r1, r2);
                y0 = mfma6(W2 + aof(s), r0, r1, r2, y0, kS6Img);
                y1 = mfma6(W2 + 32 * kS6Row + aof(s), r0, r1, r2, y1, kS6Img);
#endif
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (RW) {  // the var side is consumed: the next tile's var-side row
                if (side == 0) load_acc(pv, (d1n ? P.b1v : P.Mv + (bn * P.Gv + vgn) * 64) + 4 * half);
            }
        }
#if LDPC_S6_F16
        y0 *= iysc;
        y1 *= iysc;
#endif
        float part = 0.0f;
#pragma unroll
        for (int ot = 0; ot < 2; ++ot) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int o0 = 32 * ot + 8 * q + 4 * half;
                const f32x16 &y = ot == 0 ? y0 : y1;
                const float4 v = make_float4(y[4 * q], y[4 * q + 1], y[4 * q + 2], y[4 * q + 3]);
                if (P.last) {
                    part += v.x * wo[o0]; part += v.y * wo[o0 + 1];
                    part += v.z * wo[o0 + 2]; part += v.w * wo[o0 + 3];
                }
                if (ok && P.x_out) *reinterpret_cast<float4 *>(P.x_out + rr * 64 + o0) = v;
                if constexpr (RW) {  // the check's sum of next-layer features (row walk)
                    S[16 * ot + 4 * q] += v.x; S[16 * ot + 4 * q + 1] += v.y;
                    S[16 * ot + 4 * q + 2] += v.z; S[16 * ot + 4 * q + 3] += v.w;
                }
            }
        }
        if (P.last) {
            part += __shfl_xor(part, 32, 64);
            if (ok && half == 0) P.msg_out[b * P.E + m] = part + bo;
        }
    };
    // a tile's var-side starting row: b1v on a degree-1 tile, else its projected group row
    auto pv_row = [&](int64_t b, int64_t m, bool d1t) -> const float * {
        return (d1t || !vs ? P.b1v : P.Mv + (b * P.Gv + P.vgroup[m]) * 64) + 4 * half;
    };
    if constexpr (RW) {
        // Row walk (plan rw_*): a unit is one frame's check tile group -- up to 32 consecutive checks of
        // one degree d whose messages are contiguous runs (the reference's check-major order,
        // message_gnn_decoder.py:397-406) -- run as d tiles, tile i holding message i of every check
        // (lane j = check j).  Every tile of the unit reads the same 32 projected check rows, and the
        // lane sums its check's output rows in registers: the next layer's check-group sums leave the
        // kernel as one row per check (S_out) instead of being gathered from the feature rows again.
        // Units per launch < 2^31 (B * rw_n <= B * E, bounded by the caller's chunking).
        const int64_t nunits = P.B * P.rw_n;
        const TileWalk tw = xcd_tiles(nunits, NT / 64, wave);
        if (tw.first >= tw.end) return;
        const uint32_t rwn = (uint32_t)P.rw_n;
        // unit meta through the scalar cache (uniform addresses; a vector load here would make the
        // walk wait on the vector counter, i.e. on the prefetches issued before it)
        typedef const __attribute__((address_space(4))) int *MetaP;
        const MetaP mp = (MetaP)P.rw_meta;
        auto meta = [&](int k) { return make_int4(mp[4 * k], mp[4 * k + 1], mp[4 * k + 2], mp[4 * k + 3]); };
        // the walk's position: unit u = frame b, meta md = {first message, checks, degree, degree-1
        // tile mask}, first check group cg0 (lane j: check group cg0 + j), tile i; the lane's message m
        // (okc: the lane holds a real check; a padding lane repeats lane 0's message, writes nothing)
        int64_t u = tw.first;
        int64_t b = (uint32_t)u / rwn;
        int cu = (int)(u - b * rwn), i = 0;
        int4 md = meta(2 * cu);
        int cg0 = mp[8 * cu + 4];
        bool okc = j < md.y;
        int m = md.x + (okc ? j : 0) * md.z;
        bool d1 = P.ntile_v1 && (md.w & 1);
        float x[4][8];
        f32x16 pv[2];
        int typ = P.msg_type[m];
        if (P.x_in) load_x(x, b, m, b * P.E + m);
        if (vs) load_acc(pv, pv_row(b, m, d1));
#pragma unroll
        for (int k = 0; k < 32; ++k) S[k] = 0.0f;
        for (;;) {
            // the next tile: (u, i + 1), else the first tile of the wave's next unit; past the wave's
            // last tile the current one again (loads of valid rows, discarded)
            const bool inunit = i + 1 < md.z;
            bool more = true;
            int64_t uq = u, bq = b;
            int iq = i + 1, mq = m + 1, cg0q = cg0;
            int4 mdq = md;
            bool okq = okc;
            if (!inunit) {  // uniform
                const int64_t un = u + tw.stride;
                more = un < tw.end;
                uq = more ? un : u;
                bq = (uint32_t)uq / rwn;
                const int cq = (int)(uq - bq * rwn);
                mdq = meta(2 * cq);
                cg0q = mp[8 * cq + 4];
                okq = j < mdq.y;
                iq = more ? 0 : i;
                mq = mdq.x + (okq ? j : 0) * mdq.z + iq;
            }
            const bool d1q = P.ntile_v1 && ((mdq.w >> iq) & 1);
            const int typq = P.msg_type[mq], vgq = P.vgroup[mq];
            const int cg = cg0 + (okc ? j : 0);
            if (!P.x_in) load_x(x, b, m, b * P.E + m);  // layer 0: x from the LLR at the tile
#if LDPC_S6_PCLDS
            if (PCL && i == 0) {  // the unit's first tile: its 32 projected check rows into the lanes' LDS slots
                const float *pc = P.Mc + (b * P.Gc + cg) * 64 + 4 * half;
                float4 *pcs = reinterpret_cast<float4 *>(reinterpret_cast<char *>(lds) + s6_off_pc(P.T)) + wave * 512 + lane;
                float4 v[8];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    v[q] = *reinterpret_cast<const float4 *>(pc + 8 * q);
                    v[4 + q] = *reinterpret_cast<const float4 *>(pc + 32 + 8 * q);
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) pcs[64 * q] = v[q];
            }
#endif
            tile(b, m, b * P.E + m, okc, P.Mc + (b * P.Gc + cg) * 64 + 4 * half, x, typ, pv, d1,
                 P.x_in + (bq * P.E + mq) * 64 + 4 * half, bq, vgq, d1q, 1);
            if (!inunit) {  // the unit's last tile: its checks' sums
                if (okc && P.S_out) {
                    float *dst = P.S_out + (b * P.Gc + cg) * 64;
#pragma unroll
                    for (int ot = 0; ot < 2; ++ot)
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const float4 v = make_float4(S[16 * ot + 4 * q], S[16 * ot + 4 * q + 1],
                                                         S[16 * ot + 4 * q + 2], S[16 * ot + 4 * q + 3]);
                            *reinterpret_cast<float4 *>(dst + 32 * ot + 8 * q + 4 * half) = v;
                        }
                }
#pragma unroll
                for (int k = 0; k < 32; ++k) S[k] = 0.0f;
            }
            if (!more) break;
            u = uq; i = iq; b = bq; md = mdq; cg0 = cg0q; okc = okq; m = mq; d1 = d1q; typ = typq;
        }
        return;
    }
    const int64_t R = P.B * P.E;
    const int64_t tpf = P.tperm ? P.ntile_pf : 1;
    const int64_t ntiles = P.tperm ? P.B * tpf : (R + 31) / 32;
    const TileWalk tw = xcd_tiles(ntiles, NT / 64, wave);
    // (frame, in-frame tile) of the tperm walk, advanced without divisions: tw.stride = sb frames + sk tiles
    const int64_t sb = tw.stride / tpf, sk = tw.stride - sb * tpf;
    int64_t tb = tw.first / tpf, tk = tw.first - tb * tpf;
    // (frame, message) of row t * 32 + j of the plain walk, likewise (row stride 32 tw.stride)
    const int64_t rs = 32 * tw.stride, rsb = rs / P.E, rsm = rs - rsb * P.E;
    int64_t pb = (tw.first * 32 + j) / P.E, pm = tw.first * 32 + j - pb * P.E;
    for (int64_t t = tw.first; t < tw.end; t += tw.stride) {
        int64_t rr, b, m;
        bool ok, d1t = false;
        if (P.tperm) {  // slot j of the frame's tile k (padding: the tile's first message, not written)
            b = tb;
            const int64_t k = tk;
            const int32_t mm = P.tperm[k * 32 + j];
            ok = mm >= 0;
            m = ok ? mm : P.tperm[k * 32];
            rr = b * P.E + m;
            d1t = k < P.ntile_v1;
            tb += sb;
            tk += sk;
            if (tk >= tpf) { tk -= tpf; ++tb; }
        } else {
            const int64_t row = t * 32 + j;
            ok = row < R;
            rr = ok ? row : R - 1;
            b = ok ? pb : P.B - 1;
            m = ok ? pm : P.E - 1;
            pb += rsb;
            pm += rsm;
            if (pm >= P.E) { pm -= P.E; ++pb; }
        }
        float x[4][8];
        f32x16 pv[2];
        load_x(x, b, m, rr);
        if (vs) load_acc(pv, pv_row(b, m, d1t));
        tile(b, m, rr, ok, P.Mc + (b * P.Gc + P.cgroup[m]) * 64 + 4 * half, x, P.msg_type[m], pv, d1t, nullptr, 0, 0, false, 0);
    }
}

// ------------------------------------------------------------------------ fused MLP, any H
// one wave per message, lanes = output units (lane, lane + 64, ...); VALU fp32.
__global__ __launch_bounds__(256) void gnn_mlp_generic_kernel(GnnLayer P, int H) {
    extern __shared__ __attribute__((aligned(16))) float sh[];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float *in = sh + w * (4 * H);  // [c (H) | a or b (H) | h (H) | y (H)]
    float *y = in + 3 * H;         // both sides' second Linear, summed per unit
    const int64_t R = P.B * P.E;
    for (int64_t row = (int64_t)blockIdx.x * 4 + w; row < R; row += (int64_t)gridDim.x * 4) {
        const int64_t b = row / P.E, m = row - b * P.E;
        const int ty = P.msg_type[m];
        for (int o = lane; o < H; o += 64) y[o] = 0.0f;
        for (int side = 0; side < 2; ++side) {
            const float *W1 = side ? P.w1c : P.w1v, *b1 = side ? P.b1c : P.b1v;
            const float *W2 = side ? P.w2c : P.w2v, *b2 = side ? P.b2c : P.b2v;
            const float *M = side ? P.Mc + (b * P.Gc + P.cgroup[m]) * H : P.Mv + (b * P.Gv + P.vgroup[m]) * H;
            for (int u = lane; u < H; u += 64) {
                in[u] = x_feat(P, b, m, u, H) + P.emb[ty * H + u];
                in[H + u] = M[u];
            }
            __builtin_amdgcn_wave_barrier();
            for (int o = lane; o < H; o += 64) {
                float s = b1[o];
                for (int k = 0; k < 2 * H; ++k) s += W1[o * 2 * H + k] * in[k];
                in[2 * H + o] = relu_nan(s);
            }
            __builtin_amdgcn_wave_barrier();
            for (int o = lane; o < H; o += 64) {
                float s = b2[o];
                for (int u = 0; u < H; ++u) s += W2[o * H + u] * in[2 * H + u];
                y[o] += s;
            }
            __builtin_amdgcn_wave_barrier();
        }
        float part = 0.0f;
        for (int o = lane; o < H; o += 64) {
            float v = y[o];
            if (P.residual) v += P.x_in[row * H + o];
            if (P.last) part += v * P.wo[o];
            if (P.x_out) P.x_out[row * H + o] = v;
        }
        if (P.last) {
            for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
            if (lane == 0) P.msg_out[b * P.E + m] = part + P.bo[0];
        }
    }
}

// H != 64 up to kTiledMaxH: the MLP tiled -- each wave takes kTiledNM = 8 messages at once, lanes =
// output units, so every weight word is loaded once per 8 messages instead of once per message,
// from a per-layer transposed copy (gnn_wt_kernel: W1s^T [2H][H], W2s^T [H][H]) whose rows the lanes
// read coalesced; the 8 messages' inputs sit k-major in LDS ([k][8]: two ds_read_b128 per k) and
// each product is one fma.  (fp32 with fma chains in k order: within the fp32 bar of the reference,
// not bit-identical to gnn_mlp_generic_kernel's mul-then-add.)  VALU, not MFMA: H = 64 is the
// tuned width.
// Up to kTiledMaxH = 1024: one wave's rows are 128 H bytes of LDS (128 KB at H = 1024).  The training
// backward (gnn_train.hip train_mlp_bwd_wide_kernel) recomputes these products in the same fma order,
// so this is the training forward at every H != 64.
constexpr int kTiledNM = 8, kTiledMaxH = 1024;
inline int tiled_waves(int H) { return std::max(1, std::min(4, (64 * 1024) / (kTiledNM * 4 * H * 4))); }

__global__ void gnn_wt_kernel(const float *__restrict__ w1v, const float *__restrict__ w2v,
                              const float *__restrict__ w1c, const float *__restrict__ w2c, int H,
                              float *__restrict__ wt) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, per = 3LL * H * H;
    if (t >= 2 * per) return;
    const int side = (int)(t / per);
    const int64_t r = t - side * per;
    const float *w1 = side ? w1c : w1v, *w2 = side ? w2c : w2v;
    if (r < 2LL * H * H) {
        const int k = (int)(r / H), o = (int)(r - (int64_t)k * H);
        wt[t] = w1[(int64_t)o * 2 * H + k];
    } else {
        const int64_t q = r - 2LL * H * H;
        const int u = (int)(q / H), o = (int)(q - (int64_t)u * H);
        wt[t] = w2[(int64_t)o * H + u];
    }
}

__global__ __launch_bounds__(256) void gnn_mlp_tiled_kernel(GnnLayer P, int H) {
    extern __shared__ __attribute__((aligned(16))) float sh[];
    constexpr int NM = kTiledNM;
    const int nw = blockDim.x >> 6, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float *in = sh + w * NM * 4 * H;  // [2H][NM] c | group mean, then h [H][NM], y [H][NM]
    float *hh = in + NM * 2 * H, *yy = hh + NM * H;
    const float4 *in4 = reinterpret_cast<const float4 *>(in), *hh4 = reinterpret_cast<const float4 *>(hh);
    const int64_t R = P.B * P.E;
    for (int64_t r0 = ((int64_t)blockIdx.x * nw + w) * NM; r0 < R; r0 += (int64_t)gridDim.x * nw * NM) {
        for (int o = lane; o < H; o += 64)
#pragma unroll
            for (int i = 0; i < NM; ++i) yy[o * NM + i] = 0.0f;
        for (int side = P.vside ? 0 : 1; side < 2; ++side) {  // vside 0: the check side alone (hybrid)
            const float *W1T = P.wt + (int64_t)side * 3 * H * H, *W2T = W1T + 2LL * H * H;
            const float *b1 = side ? P.b1c : P.b1v, *b2 = side ? P.b2c : P.b2v;
            for (int i = 0; i < NM; ++i) {
                const int64_t row = r0 + i;
                if (row < R) {
                    const int64_t b = row / P.E, m = row - b * P.E;
                    const int ty = P.msg_type[m];
                    const float *M = side ? P.Mc + (b * P.Gc + P.cgroup[m]) * H : P.Mv + (b * P.Gv + P.vgroup[m]) * H;
                    for (int u = lane; u < H; u += 64) {
                        in[u * NM + i] = x_feat(P, b, m, u, H) + P.emb[ty * H + u];
                        in[(H + u) * NM + i] = M[u];
                    }
                } else {
                    for (int u = lane; u < 2 * H; u += 64) in[u * NM + i] = 0.0f;
                }
            }
            __builtin_amdgcn_wave_barrier();
            for (int o = lane; o < H; o += 64) {
                float s[NM];
#pragma unroll
                for (int i = 0; i < NM; ++i) s[i] = b1[o];
                for (int k = 0; k < 2 * H; ++k) {
                    const float wk = W1T[(int64_t)k * H + o];
                    const float4 x0 = in4[2 * k], x1 = in4[2 * k + 1];
                    s[0] = fmaf(wk, x0.x, s[0]); s[1] = fmaf(wk, x0.y, s[1]);
                    s[2] = fmaf(wk, x0.z, s[2]); s[3] = fmaf(wk, x0.w, s[3]);
                    s[4] = fmaf(wk, x1.x, s[4]); s[5] = fmaf(wk, x1.y, s[5]);
                    s[6] = fmaf(wk, x1.z, s[6]); s[7] = fmaf(wk, x1.w, s[7]);
                }
                float4 *h4 = reinterpret_cast<float4 *>(hh + o * NM);
                h4[0] = make_float4(relu_nan(s[0]), relu_nan(s[1]), relu_nan(s[2]), relu_nan(s[3]));
                h4[1] = make_float4(relu_nan(s[4]), relu_nan(s[5]), relu_nan(s[6]), relu_nan(s[7]));
            }
            __builtin_amdgcn_wave_barrier();
            for (int o = lane; o < H; o += 64) {
                float s[NM];
#pragma unroll
                for (int i = 0; i < NM; ++i) s[i] = b2[o];
                for (int u = 0; u < H; ++u) {
                    const float wu = W2T[(int64_t)u * H + o];
                    const float4 x0 = hh4[2 * u], x1 = hh4[2 * u + 1];
                    s[0] = fmaf(wu, x0.x, s[0]); s[1] = fmaf(wu, x0.y, s[1]);
                    s[2] = fmaf(wu, x0.z, s[2]); s[3] = fmaf(wu, x0.w, s[3]);
                    s[4] = fmaf(wu, x1.x, s[4]); s[5] = fmaf(wu, x1.y, s[5]);
                    s[6] = fmaf(wu, x1.z, s[6]); s[7] = fmaf(wu, x1.w, s[7]);
                }
#pragma unroll
                for (int i = 0; i < NM; ++i) yy[o * NM + i] += s[i];
            }
            __builtin_amdgcn_wave_barrier();
        }
        for (int i = 0; i < NM; ++i) {
            const int64_t row = r0 + i;
            if (row >= R) break;  // wave-uniform
            const int64_t b = row / P.E, m = row - b * P.E;
            float part = 0.0f;
            for (int o = lane; o < H; o += 64) {
                float v = yy[o * NM + i];
                if (P.residual) v += P.x_in[row * H + o];
                if (P.last) part += v * P.wo[o];
                if (P.x_out) P.x_out[row * H + o] = v;
            }
            if (P.last) {
                for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
                if (lane == 0) P.msg_out[b * P.E + m] = part + P.bo[0];
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// per-call CSR of msg_var: ints = ptr[N + 1] | cursor[N + 1] | mem[E]
__global__ void csr_count_kernel(const int32_t *__restrict__ msg_var, int64_t E, int32_t *__restrict__ cnt) {
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m < E) atomicAdd(&cnt[msg_var[m] + 1], 1);
}
__global__ __launch_bounds__(1024) void csr_scan_kernel(int32_t *__restrict__ ptr, int32_t *__restrict__ cur, int N) {
    __shared__ int32_t part[1024];
    const int t = threadIdx.x, per = (N + 1 + 1023) / 1024, lo = t * per, hi = min(lo + per, N + 1);
    int32_t s = 0;
    for (int i = lo; i < hi; ++i) s += ptr[i];
    part[t] = s;
    __syncthreads();
    if (t == 0)
        for (int i = 1; i < 1024; ++i) part[i] += part[i - 1];
    __syncthreads();
    s = t ? part[t - 1] : 0;
    for (int i = lo; i < hi; ++i) {
        s += ptr[i];
        ptr[i] = s;  // inclusive over the shifted counts = exclusive start of variable i
        cur[i] = s;
    }
}
__global__ void csr_fill_kernel(const int32_t *__restrict__ msg_var, int64_t E, int32_t *__restrict__ cur,
                                int32_t *__restrict__ mem) {
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m < E) mem[atomicAdd(&cur[msg_var[m]], 1)] = (int32_t)m;
}
__global__ void csr_sort_kernel(const int32_t *__restrict__ ptr, int N, int32_t *__restrict__ mem) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;  // ascending message order per variable
    if (v >= N) return;
    for (int i = ptr[v] + 1; i < ptr[v + 1]; ++i) {
        const int32_t x = mem[i];
        int j = i - 1;
        for (; j >= ptr[v] && mem[j] > x; --j) mem[j + 1] = mem[j];
        mem[j + 1] = x;
    }
}
// A frame whose LLRs or projected messages hold an inf or NaN decodes to NaN everywhere: the
// reference aggregates with a dense bmm (message_gnn_decoder.py:108, :118), where 0 * inf = 0 * NaN
// = NaN reaches every message of the frame in the first layer that carries one (an inf LLR already
// in layer 0; in this build's segment means only the group's neighbours would see it).  A
// non-finite feature stays non-finite through the residual to the last layer's messages, so the
// frame's LLR row and its msg_out row decide.  One workgroup per frame, frames grid-strided.
__device__ __forceinline__ bool nonfinite(float v) { return (__float_as_uint(v) & 0x7f800000u) == 0x7f800000u; }

__global__ __launch_bounds__(256) void gnn_output_csr_kernel(const float *__restrict__ msg_out, const int32_t *__restrict__ ints,
                                                             const float *__restrict__ llr, int64_t E, int N, int64_t B,
                                                             const uint8_t *__restrict__ active, float *__restrict__ probs) {
    const int32_t *ptr = ints, *mem = ints + 2 * N + 2;
    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        if (active && !active[b]) continue;  // uniform over the workgroup
        const float *mo = msg_out + b * E, *lr = llr + b * N;
        bool bad = false;
        for (int64_t e = threadIdx.x; e < E; e += 256) bad |= nonfinite(mo[e]);
        for (int v = threadIdx.x; v < N; v += 256) bad |= nonfinite(lr[v]);
        bad = __syncthreads_or(bad);
        for (int v = threadIdx.x; v < N; v += 256) {
            float s = 0.0f;  // var_llrs[var] += decoded_llrs[b, msg] in ascending msg (:277-296)
            for (int q = ptr[v]; q < ptr[v + 1]; ++q) s += mo[mem[q]];
            probs[b * N + v] = bad ? __int_as_float(0x7fc00000) : 1.0f / (1.0f + expf(-(s + lr[v])));  // (:298-307)
        }
    }
}
// The same sums with the frame's msg_out row staged in LDS (coalesced 16-B loads) when it fits: the
// per-variable 4-B gathers above touch a cache line per message and re-fetch evicted lines (their
// counter bytes were ~50x the row's).  Same order.
constexpr int64_t kOutLdsMaxE = 16384;
__global__ __launch_bounds__(256) void gnn_output_lds_kernel(const float *__restrict__ msg_out, const int32_t *__restrict__ ints,
                                                             const float *__restrict__ llr, int64_t E, int N, int64_t B,
                                                             const uint8_t *__restrict__ active, float *__restrict__ probs) {
    extern __shared__ __attribute__((aligned(16))) float mo[];
    const int32_t *ptr = ints, *mem = ints + 2 * N + 2;
    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        if (active && !active[b]) continue;  // uniform over the workgroup
        __syncthreads();                     // the previous frame's reads are done
        const float *src = msg_out + b * E;
        bool bad = false;
        if ((E & 3) == 0)
            for (int64_t e = threadIdx.x; e < E / 4; e += 256) {
                const float4 v = reinterpret_cast<const float4 *>(src)[e];
                bad = bad || nonfinite(v.x) || nonfinite(v.y) || nonfinite(v.z) || nonfinite(v.w);
                reinterpret_cast<float4 *>(mo)[e] = v;
            }
        else
            for (int64_t e = threadIdx.x; e < E; e += 256) {
                mo[e] = src[e];
                bad |= nonfinite(mo[e]);
            }
        for (int v = threadIdx.x; v < N; v += 256) bad |= nonfinite(llr[b * N + v]);
        bad = __syncthreads_or(bad);
        for (int v = threadIdx.x; v < N; v += 256) {
            float s = 0.0f;
            for (int q = ptr[v]; q < ptr[v + 1]; ++q) s += mo[mem[q]];
            const int64_t i = b * N + v;
            probs[i] = bad ? __int_as_float(0x7fc00000) : 1.0f / (1.0f + expf(-(s + llr[i])));
        }
    }
}


__global__ void gnn_fill_kernel(int32_t *p, int64_t n, int32_t v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// Row walk: memb[l][g][u] = (1 / |g|) sum over check group g's messages (ascending) of emb_l[type][u],
// the mean type embedding each layer's check-side group mean adds to S * inv (gnn_group_proj_kernel);
// the same per var group (memb_v), added to the var side's sum of x rows * inv
__global__ void gnn_memb_kernel(const float *__restrict__ emb0, int64_t layer_stride, const int32_t *__restrict__ msg_type,
                                const int32_t *__restrict__ cg_ptr, const int32_t *__restrict__ cg_mem,
                                const float *__restrict__ inv_c, int Gc, int layers, float *__restrict__ memb) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)layers * Gc * 64) return;
    const int64_t l = i / ((int64_t)Gc * 64);
    const int g = (int)(i / 64 - l * Gc), u = (int)(i & 63);
    const float *emb = emb0 + l * layer_stride;
    float s = 0.0f;
    for (int k = cg_ptr[g]; k < cg_ptr[g + 1]; ++k) s += emb[msg_type[cg_mem[k]] * 64 + u];
    memb[i] = s * inv_c[g];
}

int64_t layer_floats(int H, int T) { return (int64_t)T * H + 2 * (2LL * H * H + H + (int64_t)H * H + H) + H + 1; }

// H = 32 k other than 64 (gnn_wide.hip) on the MFMA row GEMMs (group plans; inference)
bool wide_on(const ldpc_gnn_plan *p, int H) { return gnn_wide_supported(H) && !p->weighted && p->n_gtiles > 0; }

struct Ws {
    float *xa, *xb, *Mv, *Mc, *msg_out, *wt;
    float *Pv, *Pc, *hbuf;  // wide path: projected group rows (B, G, H), MLP hidden rows (B, E, 2 H)
    char *wimg;             // wide path, H = 96 / 128: every layer's fused-MLP slice images
    int *wexp;              // ... and their weight exponents (2 per layer)
    float *wmemb;           // wide path: every layer's mean type embedding per group (L, Gv + Gc, H)
    uint32_t *xmax[2], *hmax, *gmax_v, *gmax_c;  // wide path: each row's largest |value| (f16 splits)
    float *S, *memb;  // row walk (H = 64, plan rw_*): per-check feature sums (B, Gc, H), mean type embeddings (L, Gc, H)
    float *memb_v;    // ... and per var group (L, Gv, H)
    int32_t *csr;
    int64_t bytes;
};

// train: the training forward (d_saved), which never takes the wide path -- the backward
// (gnn_train.hip) recomputes h and the ReLU masks with gnn_mlp_tiled_kernel's fma chains
Ws carve(const ldpc_gnn_plan *p, int H, int N, int64_t B, int layers, int precision, void *base, bool train = false) {
    Ws w{};
    auto al = [](int64_t x) { return (x + 255) / 256 * 256; };
    const int64_t es = 4;  // bytes per stored feature (fp32 path)
    (void)precision;
    const bool wide = wide_on(p, H) && !train;  // the last layer's rows are stored too (its head reads them)
    const int64_t xb = layers > 1 || wide ? al(B * p->E * H * es) : 0;
    const int64_t xb2 = layers > 2 || (wide && layers > 1) ? xb : 0;
    const int64_t mv = al(B * (int64_t)p->Gv * H * es), mc = al(B * (int64_t)p->Gc * H * es);
    const int64_t vs = al(B * p->E * 4), cs = al(gnn_csr_ints(p->E, N) * 4);
    char *c = static_cast<char *>(base);
    w.xa = reinterpret_cast<float *>(c);
    w.xb = reinterpret_cast<float *>(c + xb);
    w.Mv = reinterpret_cast<float *>(c + xb + xb2);
    w.Mc = reinterpret_cast<float *>(c + xb + xb2 + mv);
    w.msg_out = reinterpret_cast<float *>(c + xb + xb2 + mv + mc);
    w.csr = reinterpret_cast<int32_t *>(c + xb + xb2 + mv + mc + vs);
    // H != 64 (gnn_mlp_tiled_kernel): every layer's transposed MLP weights, 6 H^2 floats each
    // (formed once per call, before the frame halves fork onto two streams)
    const int64_t wtb = H != 64 && H <= kTiledMaxH && !wide ? al(6LL * H * H * 4 * layers) : 0;
    w.wt = wtb ? reinterpret_cast<float *>(c + xb + xb2 + mv + mc + vs + cs) : nullptr;
    const int64_t rwb = H == 64 && p->n_rw > 0 && layers > 1 ? mc : 0;
    const int64_t mbb = rwb ? al((int64_t)layers * (p->Gc + p->Gv) * H * es) : 0;
    char *r = c + xb + xb2 + mv + mc + vs + cs + wtb;
    w.S = rwb ? reinterpret_cast<float *>(r) : nullptr;
    w.memb = rwb ? reinterpret_cast<float *>(r + rwb) : nullptr;
    w.memb_v = rwb ? w.memb + (int64_t)layers * p->Gc * H : nullptr;
    const int64_t hb = wide ? al(B * p->E * 2 * H * es) : 0;
    char *q = r + rwb + mbb;
    w.Pv = wide ? reinterpret_cast<float *>(q) : nullptr;
    w.Pc = wide ? reinterpret_cast<float *>(q + mv) : nullptr;
    w.hbuf = wide ? reinterpret_cast<float *>(q + mv + mc) : nullptr;
    // row maxima: x (two, with the feature ping-pong), h, group rows: 4 B per row
    const int64_t rm = al(B * p->E * 4), gmv = al(B * (int64_t)p->Gv * 4), gmc = al(B * (int64_t)p->Gc * 4);
    char *z = q + (wide ? mv + mc + hb : 0);
    w.xmax[0] = wide ? reinterpret_cast<uint32_t *>(z) : nullptr;
    w.xmax[1] = wide ? reinterpret_cast<uint32_t *>(z + rm) : nullptr;
    w.hmax = wide ? reinterpret_cast<uint32_t *>(z + 2 * rm) : nullptr;
    w.gmax_v = wide ? reinterpret_cast<uint32_t *>(z + 3 * rm) : nullptr;
    w.gmax_c = wide ? reinterpret_cast<uint32_t *>(z + 3 * rm + gmv) : nullptr;
    const int64_t fib = wide ? al(gnn_wide_fused_bytes(H, layers)) : 0, feb = fib ? al(2LL * layers * 4) : 0;
    char *f = z + (wide ? 3 * rm + gmv + gmc : 0);
    w.wimg = fib ? f : nullptr;
    w.wexp = fib ? reinterpret_cast<int *>(f + fib) : nullptr;
    const int64_t wmb = wide ? al((int64_t)layers * (p->Gv + p->Gc) * H * 4) : 0;
    w.wmemb = wmb ? reinterpret_cast<float *>(f + fib + feb) : nullptr;
    w.bytes = xb + xb2 + mv + mc + vs + cs + wtb + rwb + mbb + (wide ? mv + mc + hb + 3 * rm + gmv + gmc : 0) + fib + feb + wmb;
    return w;
}

// ------------------------------------------------------------------------ hybrid GNN (CustomVariable*)
// CustomVariableMessageGNNDecoder (message_gnn_decoder.py:758-879) cannot run in the reference
// (SURVEY.md section 0).  This build defines a layer by the steps MGD:672-755 spell out, per frame:
//   c = x + emb[type];  b = A_c c (check groups);  F = MLP_c([c; b])                      (:704-726)
//   l_m = output_projection(F_m)                     the layer's own head               (:729)
//   v2c_m = (llr_v + sum_{m' -> v} l_m') - l_m,  then 0.5 v2c_m + 0.5 l_m  (every layer: the
//           decoder passes iteration i + 1 >= 1, MGD:851, so the damping of :659-663 always applies)
//   x <- input_embedding(v2c_m) + F_m   (the decoder's Linear(1, H): the layer has none, :745)  (:745-753)
// and the decoder's output (:855-877): out_m = output_projection_L(x_m),
//   probs_v = sigmoid(sum_{m -> v} out_m / deg_v + llr_v)   (row-normalised mapping, :858-870).
// Kernels: the projection / MLP kernels above on the check side alone (vside = 0), then these.

// v2c (B, E) from the layer's projected check messages l = msg_out (B, E); one thread per (frame,
// variable), its messages in ascending order (the per-call CSR of msg_var)
__global__ __launch_bounds__(256) void custom_var_llr_kernel(const float *__restrict__ l, const int32_t *__restrict__ csr,
                                                             const float *__restrict__ llr, int64_t E, int N, int64_t B,
                                                             float *__restrict__ v2c) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * N) return;
    const int64_t b = i / N;
    const int v = (int)(i - b * N);
    const int32_t *ptr = csr_ptr(csr), *mem = csr_mem(csr, N);
    const int p0 = ptr[v], p1 = ptr[v + 1];
    if (p1 == p0) return;
    const float *lb = l + b * E;
    float sum = lb[mem[p0]];
    for (int q = p0 + 1; q < p1; ++q) sum = sum + lb[mem[q]];
    const float total = llr[i] + sum;
    for (int q = p0; q < p1; ++q) {
        const float c = lb[mem[q]];
        const float x = total - c;
        v2c[b * E + mem[q]] = 0.5f * x + 0.5f * c;
    }
}

// x_m = (v2c_m w_in + b_in) + F_m in place (64 floats per message, 16 lanes x float4); on the last
// layer instead out_m = wo . x_m + bo into msg_out
__global__ __launch_bounds__(256) void custom_combine_kernel(float *__restrict__ x, const float *__restrict__ v2c,
                                                             const float *__restrict__ w_in, const float *__restrict__ b_in,
                                                             int64_t R, const float *__restrict__ wo,
                                                             const float *__restrict__ bo, float *__restrict__ msg_out) {
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const int q = threadIdx.x & 15;
    if (r >= R) return;
    const float v = v2c[r];
    float4 *xr = reinterpret_cast<float4 *>(x + r * 64) + q;
    const float4 f = *xr, w = reinterpret_cast<const float4 *>(w_in)[q], c = reinterpret_cast<const float4 *>(b_in)[q];
    const float4 o = make_float4((v * w.x + c.x) + f.x, (v * w.y + c.y) + f.y, (v * w.z + c.z) + f.z, (v * w.w + c.w) + f.w);
    if (!wo) {
        *xr = o;
        return;
    }
    const float4 k = reinterpret_cast<const float4 *>(wo)[q];
    float part = o.x * k.x + o.y * k.y + o.z * k.z + o.w * k.w;
    for (int off = 8; off > 0; off >>= 1) part += __shfl_xor(part, off, 16);
    if (q == 0) msg_out[r] = part + bo[0];
}

// The same head for any H: out_m = wo . ((v2c w_in + b_in) + F_m) + bo, 16 lanes per row over the units
__global__ __launch_bounds__(256) void custom_combine_any_kernel(const float *__restrict__ x, const float *__restrict__ v2c,
                                                                 const float *__restrict__ w_in, const float *__restrict__ b_in,
                                                                 int H, int64_t R, const float *__restrict__ wo,
                                                                 const float *__restrict__ bo, float *__restrict__ msg_out) {
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const int q = threadIdx.x & 15;
    if (r >= R) return;
    const float v = v2c[r];
    const float *f = x + r * H;
    float part = 0.0f;
    for (int u = q; u < H; u += 16) part += ((v * w_in[u] + b_in[u]) + f[u]) * wo[u];
    for (int off = 8; off > 0; off >>= 1) part += __shfl_xor(part, off, 16);
    if (q == 0) msg_out[r] = part + bo[0];
}

// probs[b][v] = sigmoid(sum_{m -> v} out_m * (1 / deg_v) + llr[b][v]), ascending message order
__global__ void custom_output_kernel(const float *__restrict__ msg_out, const int32_t *__restrict__ csr,
                                     const float *__restrict__ llr, int64_t E, int N, int64_t n,
                                     float *__restrict__ probs) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t b = i / N;
    const int v = (int)(i - b * N);
    const int32_t *ptr = csr_ptr(csr), *mem = csr_mem(csr, N);
    const int p0 = ptr[v], p1 = ptr[v + 1];
    const float w = 1.0f / ((float)(p1 - p0) + 1e-10f);  // mapping / (row sum + 1e-10), :859
    const float *mo = msg_out + b * E;
    float s = 0.0f;
    for (int q = p0; q < p1; ++q) s += mo[mem[q]] * w;
    probs[i] = 1.0f / (1.0f + expf(-(s + llr[i])));
}

int g_num_cus = 0;

constexpr int kMlp2Wps = LDPC_MLP2_WPS, kMlp2Nt = LDPC_MLP2_NT;
// 2 waves per SIMD: both sides' GEMM1 share one split of c (226 VGPRs, no spills); 51.6 k vs 49.9 k
// cw/s for the per-side form at 3 waves per SIMD (168 VGPRs, spilling), profiles/r04
#ifndef LDPC_MLP2S_WPS
#define LDPC_MLP2S_WPS 2
#endif
#ifndef LDPC_MLP2S_NT
#define LDPC_MLP2S_NT 512
#endif
constexpr int kMlp2sWps = LDPC_MLP2S_WPS, kMlp2sNt = LDPC_MLP2S_NT;
// LDPC_GNN_SPLIT=0: the projected-group MLP on v_mfma_f32_32x32x2_f32 (gnn_mlp2_kernel); default:
// the same fp32 products as three-term bf16 splits on the bf16 MFMA (gnn_mlp2s_kernel).  Read per
// call (tests compare the two).
bool split_path() {
    const char *e = std::getenv("LDPC_GNN_SPLIT");
    return !(e && std::atoi(e) == 0);
}

// LDPC_GNN_ROWWALK=0 keeps the tile walk of gnn_mlp2s_kernel and the gathered check-side means
// (A/B runs); default: the row walk when the plan has check tile groups.  Read per call.
bool rowwalk_path() {
    const char *e = std::getenv("LDPC_GNN_ROWWALK");
    return !(e && std::atoi(e) == 0);
}

// LDPC_GNN_PCLDS=0 runs the row walk without its LDS-staged check rows (the kernel that codes with
// too many message types for the staging get); default: staged when they fit.  Read per call.
bool pclds_path() {
    const char *e = std::getenv("LDPC_GNN_PCLDS");
    return !(e && std::atoi(e) == 0);
}

// LDPC_GNN_PROJ=0 keeps the per-message [c; g] GEMM1 (gnn_mlp_mfma_kernel) for A/B runs
bool proj_path() {
    static bool t = [] {
        const char *e = std::getenv("LDPC_GNN_PROJ");
        return !(e && std::atoi(e) == 0);
    }();
    return t;
}


// LDPC_GNN_STREAMS=1 runs the fp32 forward as one frame range on the caller's stream (A/B runs);
// default 2: two frame halves on two streams, so one half's HBM-bound group-mean launch runs in
// the register/wave slots the other half's MFMA-bound MLP leaves free on every CU.
int gnn_streams() {
    static int t = [] {
        const char *e = std::getenv("LDPC_GNN_STREAMS");
        return (e && std::atoi(e) == 1) ? 1 : 2;
    }();
    return t;
}

}  // namespace
}  // namespace ldpc

// One non-blocking side stream per device, created once (under a lock) and kept for the process, and a
// fork/join event pair per device AND calling thread: two host threads decoding on one device record
// their own events, so a join never orders against another thread's launches.  (Launches of two
// threads on the shared side stream serialise, which is correct.)
int ldpc::gnn_side_stream(hipStream_t *side, hipEvent_t *fork, hipEvent_t *join) {
    constexpr int kMaxDev = 64;
    static hipStream_t streams[kMaxDev];
    static std::mutex mu;
    thread_local hipEvent_t forks[kMaxDev], joins[kMaxDev];
    int dev = 0;
    LDPC_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDev) return fail(LDPC_EUNSUPPORTED, "device index out of range");
    {
        std::lock_guard<std::mutex> g(mu);
        if (!streams[dev]) LDPC_HIP(hipStreamCreateWithFlags(&streams[dev], hipStreamNonBlocking));
        *side = streams[dev];
    }
    if (!forks[dev]) {
        LDPC_HIP(hipEventCreateWithFlags(&forks[dev], hipEventDisableTiming));
        LDPC_HIP(hipEventCreateWithFlags(&joins[dev], hipEventDisableTiming));
    }
    *fork = forks[dev];
    *join = joins[dev];
    return LDPC_OK;
}

using namespace ldpc;

int ldpc::gnn_build_var_csr(const int32_t *d_msg_var, int64_t E, int N, int32_t *d_ints, hipStream_t s) {
    int32_t *ptr = d_ints, *cur = d_ints + N + 1, *mem = d_ints + 2 * N + 2;
    LDPC_HIP(hipMemsetAsync(ptr, 0, (size_t)(N + 1) * 4, s));
    const unsigned ge = (unsigned)((E + 255) / 256);
    hipLaunchKernelGGL(csr_count_kernel, dim3(ge), dim3(256), 0, s, d_msg_var, E, ptr);
    hipLaunchKernelGGL(csr_scan_kernel, dim3(1), dim3(1024), 0, s, ptr, cur, N);
    hipLaunchKernelGGL(csr_fill_kernel, dim3(ge), dim3(256), 0, s, d_msg_var, E, cur, mem);
    hipLaunchKernelGGL(csr_sort_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, ptr, N, mem);
    LDPC_CHECK_LAUNCH("gnn csr kernels");
    return LDPC_OK;
}

int ldpc::gnn_output(const float *d_msg_out, const int32_t *d_ints, const float *d_llr, int64_t E, int N, int64_t B,
                     const uint8_t *d_active, float *d_probs, hipStream_t s) {
    const int64_t n = B * N;
    if (E <= kOutLdsMaxE && B > 0) {
        if (g_num_cus == 0) {
            int dev = 0;
            LDPC_HIP(hipGetDevice(&dev));
            LDPC_HIP(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev));
        }
        const unsigned grid = (unsigned)std::min<int64_t>(B, (int64_t)std::max(g_num_cus, 1) * 8);
        hipLaunchKernelGGL(gnn_output_lds_kernel, dim3(grid), dim3(256), (size_t)E * 4, s, d_msg_out, d_ints, d_llr, E, N, B,
                           d_active, d_probs);
        LDPC_CHECK_LAUNCH("gnn_output_lds_kernel");
        return LDPC_OK;
    }
    if (g_num_cus == 0) {
        int dev = 0;
        LDPC_HIP(hipGetDevice(&dev));
        LDPC_HIP(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    (void)n;
    hipLaunchKernelGGL(gnn_output_csr_kernel, dim3((unsigned)std::min<int64_t>(B, (int64_t)std::max(g_num_cus, 1) * 8)), dim3(256),
                       0, s, d_msg_out, d_ints, d_llr, E, N, B, d_active, d_probs);
    LDPC_CHECK_LAUNCH("gnn_output_csr_kernel");
    return LDPC_OK;
}

extern "C" int ldpc_gnn_plan_create(int64_t E, int n_vgroups, const int32_t *h_vgroup, int n_cgroups,
                                    const int32_t *h_cgroup, ldpc_gnn_plan **out) {
    if (!out) return fail(LDPC_EINVAL, "out is NULL");
    *out = nullptr;
    if (E <= 0 || n_vgroups <= 0 || n_cgroups <= 0 || !h_vgroup || !h_cgroup)
        return fail(LDPC_EINVAL, "bad GNN plan arguments");
    std::vector<int32_t> vptr(n_vgroups + 1, 0), cptr(n_cgroups + 1, 0), vmem(E), cmem(E);
    for (int64_t m = 0; m < E; ++m) {
        if (h_vgroup[m] < 0 || h_vgroup[m] >= n_vgroups || h_cgroup[m] < 0 || h_cgroup[m] >= n_cgroups)
            return fail(LDPC_EINVAL, "group label out of range");
        vptr[h_vgroup[m] + 1]++;
        cptr[h_cgroup[m] + 1]++;
    }
    for (int g = 0; g < n_vgroups; ++g) vptr[g + 1] += vptr[g];
    for (int g = 0; g < n_cgroups; ++g) cptr[g + 1] += cptr[g];
    {
        std::vector<int32_t> fv(vptr.begin(), vptr.end() - 1), fc(cptr.begin(), cptr.end() - 1);
        for (int64_t m = 0; m < E; ++m) {  // members in ascending message order
            vmem[fv[h_vgroup[m]]++] = (int32_t)m;
            cmem[fc[h_cgroup[m]]++] = (int32_t)m;
        }
    }
    std::vector<float> inv(n_vgroups + n_cgroups);
    for (int g = 0; g < n_vgroups; ++g) {
        const int d = vptr[g + 1] - vptr[g];
        inv[g] = d ? 1.0f / (float)d : 0.0f;
    }
    for (int g = 0; g < n_cgroups; ++g) {
        const int d = cptr[g + 1] - cptr[g];
        inv[n_vgroups + g] = d ? 1.0f / (float)d : 0.0f;
    }
    // bf16 path: group tiles of 8 groups of one degree (gnn.hpp), var side then check side
    std::vector<int32_t> gt_meta, gt_grp, gt_mem;
    auto add_tiles = [&](const std::vector<int32_t> &ptr, const std::vector<int32_t> &mem, int ngroups, int gbase) {
        std::vector<int32_t> order;
        for (int g = 0; g < ngroups; ++g)
            if (ptr[g + 1] > ptr[g]) order.push_back(g);  // a group with no messages is never read
        std::stable_sort(order.begin(), order.end(),
                         [&](int a, int b) { return ptr[a + 1] - ptr[a] < ptr[b + 1] - ptr[b]; });
        for (size_t i = 0; i < order.size();) {
            const int d = ptr[order[i] + 1] - ptr[order[i]];
            size_t n = 0;
            while (n < 8 && i + n < order.size() && ptr[order[i + n] + 1] - ptr[order[i + n]] == d) ++n;
            gt_meta.push_back(d);
            gt_meta.push_back((int32_t)gt_mem.size());
            for (int k = 0; k < d; ++k)
                for (size_t q = 0; q < 8; ++q)
                    gt_mem.push_back(q < n ? mem[ptr[order[i + q]] + k] : mem[ptr[order[i]] + k]);
            for (size_t q = 0; q < 8; ++q) gt_grp.push_back(q < n ? gbase + order[i + q] : -1);
            i += n;
        }
    };
    add_tiles(vptr, vmem, n_vgroups, 0);
    int n_v1 = 0;  // var tiles come first, sorted by degree: the degree-1 ones lead
    while (2 * n_v1 < (int)gt_meta.size() && gt_meta[2 * n_v1] == 1) ++n_v1;
    const int n_gt_v = (int)(gt_meta.size() / 2);
    add_tiles(cptr, cmem, n_cgroups, n_vgroups);
    // bf16 MLP tiles (gnn.hpp ct_m0): whole check groups when each is a contiguous message run of
    // at most 32 (greedy, in message order), else plain 32-message tiles
    bool aligned = true;
    for (int g = 0; g < n_cgroups && aligned; ++g) {
        const int d = cptr[g + 1] - cptr[g];
        aligned = d <= 32 && (d == 0 || cmem[cptr[g + 1] - 1] - cmem[cptr[g]] == d - 1);
    }
    std::vector<int32_t> ct_m0{0};
    if (aligned) {
        int64_t m = 0;
        while (m < E) {
            const int g = h_cgroup[m];
            const int d = cptr[g + 1] - cptr[g];  // the group's run starts at m (contiguous, ascending)
            if (m + d - ct_m0.back() > 32) ct_m0.push_back((int32_t)m);
            m += d;
        }
    } else {
        for (int64_t m = 32; m < E; m += 32) ct_m0.push_back((int32_t)m);
    }
    ct_m0.push_back((int32_t)E);
    // fp32 row walk: check tile groups (gnn.hpp rw_*), used when they fill >= 90 % of their tiles
    std::vector<int32_t> rw_meta, rw_cg;
    bool rw_d1 = true, rw_contig = true;  // rw_contig: lane k of a unit holds check group first + k
    if (aligned) {
        auto vdeg1 = [&](int64_t m) { return vptr[h_vgroup[m] + 1] - vptr[h_vgroup[m]] == 1; };
        int64_t m = 0, slots = 0, d1_msgs = 0, d1_in_tiles = 0;
        for (int64_t q = 0; q < E; ++q) d1_msgs += vdeg1(q);
        while (m < E) {
            const int d = cptr[h_cgroup[m] + 1] - cptr[h_cgroup[m]];
            const int64_t m0 = m;
            int n = 0;
            while (n < 32 && m < E && cptr[h_cgroup[m] + 1] - cptr[h_cgroup[m]] == d) {
                rw_cg.push_back(h_cgroup[m]);
                ++n;
                m += d;
            }
            for (int k = n; k < 32; ++k) rw_cg.push_back(-1);
            int32_t mask = 0;
            for (int i = 0; i < d; ++i) {
                bool all = true;
                for (int k = 0; k < n && all; ++k) all = vdeg1(m0 + (int64_t)k * d + i);
                if (all) {
                    mask |= (int32_t)(1u << i);
                    d1_in_tiles += n;
                }
            }
            for (int k = 1; k < n; ++k) rw_contig = rw_contig && rw_cg[rw_cg.size() - 32 + k] == rw_cg[rw_cg.size() - 32] + k;
            rw_meta.insert(rw_meta.end(), {(int32_t)m0, n, d, mask, rw_cg[rw_cg.size() - 32], 0, 0, 0});
            slots += 32LL * d;
        }
        rw_d1 = d1_in_tiles == d1_msgs;
        if (!rw_d1)
            for (size_t c = 0; c < rw_meta.size(); c += 8) rw_meta[c + 3] = 0;
        if ((double)E < 0.9 * (double)slots || !rw_contig) rw_meta.clear();
        rw_cg.clear();
    }
    // fp32 path: projection tiles of 32 groups of one side (gnn.hpp), each side sorted by degree
    std::vector<int32_t> pt;  // meta [4 n] | grp [32 n] | deg [32 n] | mem
    std::vector<int32_t> pt_meta, pt_grp, pt_deg, pt_mem;
    auto add_ptiles = [&](const std::vector<int32_t> &ptr, const std::vector<int32_t> &mem, int ngroups, int side) {
        std::vector<int32_t> order;
        for (int g = 0; g < ngroups; ++g)
            if (ptr[g + 1] > ptr[g]) order.push_back(g);
        std::stable_sort(order.begin(), order.end(),
                         [&](int a, int b) { return ptr[a + 1] - ptr[a] < ptr[b + 1] - ptr[b]; });
        for (size_t i = 0; i < order.size(); i += 32) {
            const size_t n = std::min<size_t>(32, order.size() - i);
            int dmax = 0;
            for (size_t q = 0; q < n; ++q) dmax = std::max(dmax, ptr[order[i + q] + 1] - ptr[order[i + q]]);
            pt_meta.insert(pt_meta.end(), {side, dmax, (int32_t)pt_mem.size(), 0});
            for (int k = 0; k <= dmax; ++k)  // one padding row: the kernel reads members in pairs
                for (size_t q = 0; q < 32; ++q) {
                    const int g = q < n ? order[i + q] : -1;
                    pt_mem.push_back(g >= 0 && k < ptr[g + 1] - ptr[g] ? mem[ptr[g] + k] : 0);
                }
            for (size_t q = 0; q < 32; ++q) {
                pt_grp.push_back(q < n ? order[i + q] : -1);
                pt_deg.push_back(q < n ? ptr[order[i + q] + 1] - ptr[order[i + q]] : 0);
            }
        }
    };
    add_ptiles(vptr, vmem, n_vgroups, 0);
    const int n_ptiles_v = (int)(pt_meta.size() / 4);
    int n_ptiles_v1 = 0;  // leading var tiles of degree-1 groups only (padding has degree 0)
    while (n_ptiles_v1 < n_ptiles_v &&
           std::all_of(pt_deg.begin() + 32 * n_ptiles_v1, pt_deg.begin() + 32 * (n_ptiles_v1 + 1),
                       [](int32_t d) { return d <= 1; }))
        ++n_ptiles_v1;
    add_ptiles(cptr, cmem, n_cgroups, 1);
    // bf16 projected MLP: degree-1 var groups' messages first, each part padded to whole tiles
    std::vector<int32_t> mperm;
    auto vdeg = [&](int64_t m) { return vptr[h_vgroup[m] + 1] - vptr[h_vgroup[m]]; };
    for (int64_t m = 0; m < E; ++m)
        if (vdeg(m) == 1) mperm.push_back((int32_t)m);
    while (mperm.size() % 32) mperm.push_back(-1);
    const int n_mtiles_v1 = (int)(mperm.size() / 32);
    for (int64_t m = 0; m < E; ++m)
        if (vdeg(m) != 1) mperm.push_back((int32_t)m);
    while (mperm.size() % 32) mperm.push_back(-1);
    pt.insert(pt.end(), pt_meta.begin(), pt_meta.end());
    pt.insert(pt.end(), pt_grp.begin(), pt_grp.end());
    pt.insert(pt.end(), pt_deg.begin(), pt_deg.end());
    pt.insert(pt.end(), pt_mem.begin(), pt_mem.end());
    pt.insert(pt.end(), mperm.begin(), mperm.end());
    std::vector<int32_t> blob;
    blob.insert(blob.end(), h_vgroup, h_vgroup + E);
    blob.insert(blob.end(), h_cgroup, h_cgroup + E);
    blob.insert(blob.end(), vptr.begin(), vptr.end());
    blob.insert(blob.end(), vmem.begin(), vmem.end());
    blob.insert(blob.end(), cptr.begin(), cptr.end());
    blob.insert(blob.end(), cmem.begin(), cmem.end());
    const size_t gt_words = gt_meta.size() + gt_grp.size() + gt_mem.size();
    auto *p = new ldpc_gnn_plan();
    p->n_gtiles = (int)(gt_meta.size() / 2);
    p->n_gtiles_v1 = n_v1;
    p->E = E;
    p->Gv = n_vgroups;
    p->Gc = n_cgroups;
    hipError_t e1 = hipGetDevice(&p->device);
    hipError_t e2 = hipMalloc(&p->d_tab, blob.size() * 4);
    hipError_t e3 = hipMalloc(&p->d_inv, inv.size() * 4);
    hipError_t e4 = hipMalloc(&p->d_gt, gt_words * 4);
    hipError_t e5 = hipMalloc(&p->d_pt, pt.size() * 4);
    hipError_t e6 = hipMalloc(&p->d_ct, ct_m0.size() * 4);
    hipError_t e7 = rw_meta.empty() ? hipSuccess : hipMalloc(&p->d_rw, rw_meta.size() * 4);
    if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess || e4 != hipSuccess || e5 != hipSuccess ||
        e6 != hipSuccess || e7 != hipSuccess) {
        ldpc_gnn_plan_destroy(p);
        return fail(LDPC_EHIP, "GNN plan allocation failed");
    }
    if (hipMemcpy(p->d_tab, blob.data(), blob.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_inv, inv.data(), inv.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_gt, gt_meta.data(), gt_meta.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_gt + gt_meta.size(), gt_grp.data(), gt_grp.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_gt + gt_meta.size() + gt_grp.size(), gt_mem.data(), gt_mem.size() * 4,
                  hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_pt, pt.data(), pt.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_ct, ct_m0.data(), ct_m0.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (p->d_rw && hipMemcpy(p->d_rw, rw_meta.data(), rw_meta.size() * 4, hipMemcpyHostToDevice) != hipSuccess)) {
        ldpc_gnn_plan_destroy(p);
        return fail(LDPC_EHIP, "GNN plan upload failed");
    }
    p->n_rw = (int)(rw_meta.size() / 8);
    p->rw_d1 = p->n_rw > 0 && rw_d1;
    p->rw_meta = reinterpret_cast<const int4 *>(p->d_rw);
    p->n_ptiles = (int)(pt_meta.size() / 4);
    p->n_ptiles_v = n_ptiles_v;
    p->n_ptiles_v1 = n_ptiles_v1;
    p->pt_meta = reinterpret_cast<const int4 *>(p->d_pt);
    p->pt_grp = p->d_pt + pt_meta.size();
    p->pt_deg = p->pt_grp + pt_grp.size();
    p->pt_mem = p->pt_deg + pt_deg.size();
    p->mt_perm = p->pt_mem + pt_mem.size();
    p->n_mtiles = (int)(mperm.size() / 32);
    p->n_mtiles_v1 = n_mtiles_v1;
    p->n_gtiles_v = n_gt_v;
    p->n_ctiles = (int)ct_m0.size() - 1;
    p->ct_aligned = aligned;
    p->ct_m0 = p->d_ct;
    p->vgroup = p->d_tab;
    p->cgroup = p->vgroup + E;
    p->vg_ptr = p->cgroup + E;
    p->vg_mem = p->vg_ptr + n_vgroups + 1;
    p->cg_ptr = p->vg_mem + E;
    p->cg_mem = p->cg_ptr + n_cgroups + 1;
    p->inv_v = p->d_inv;
    p->inv_c = p->d_inv + n_vgroups;
    p->gt_meta = reinterpret_cast<const int2 *>(p->d_gt);
    p->gt_grp = p->d_gt + gt_meta.size();
    p->gt_mem = p->gt_grp + gt_grp.size();
    *out = p;
    return LDPC_OK;
}

// General adjacencies (message_gnn_decoder.py:93-118: any (E x E) matrix after the reference's
// zero-pad / crop) as two CSR matrices: row m lists the messages j with A[m, j] != 0, ascending, and
// their values.  Every message reads aggregation row m of each side, so the MLP kernels run
// unchanged on rows that are bmm(A, c) instead of group means.
extern "C" int ldpc_gnn_plan_create_csr(int64_t E, const int32_t *h_v_ptr, const int32_t *h_v_col, const float *h_v_val,
                                        const int32_t *h_c_ptr, const int32_t *h_c_col, const float *h_c_val,
                                        ldpc_gnn_plan **out) {
    if (!out) return fail(LDPC_EINVAL, "out is NULL");
    *out = nullptr;
    if (E <= 0 || E > (1 << 30) || !h_v_ptr || !h_c_ptr) return fail(LDPC_EINVAL, "bad GNN CSR plan arguments");
    const int64_t nv = h_v_ptr[E], nc = h_c_ptr[E];
    if (h_v_ptr[0] != 0 || h_c_ptr[0] != 0 || nv < 0 || nc < 0 || (nv && (!h_v_col || !h_v_val)) ||
        (nc && (!h_c_col || !h_c_val)))
        return fail(LDPC_EINVAL, "bad CSR arrays");
    for (int64_t m = 0; m < E; ++m)
        if (h_v_ptr[m + 1] < h_v_ptr[m] || h_c_ptr[m + 1] < h_c_ptr[m]) return fail(LDPC_EINVAL, "CSR row pointers must ascend");
    for (int64_t i = 0; i < nv; ++i)
        if (h_v_col[i] < 0 || h_v_col[i] >= E) return fail(LDPC_EINVAL, "CSR column out of range");
    for (int64_t i = 0; i < nc; ++i)
        if (h_c_col[i] < 0 || h_c_col[i] >= E) return fail(LDPC_EINVAL, "CSR column out of range");
    std::vector<int32_t> blob;
    blob.reserve(2 * E + 2 * (E + 1) + nv + nc);
    for (int64_t m = 0; m < E; ++m) blob.push_back((int32_t)m);  // vgroup: own row
    for (int64_t m = 0; m < E; ++m) blob.push_back((int32_t)m);  // cgroup: own row
    blob.insert(blob.end(), h_v_ptr, h_v_ptr + E + 1);
    blob.insert(blob.end(), h_v_col, h_v_col + nv);
    blob.insert(blob.end(), h_c_ptr, h_c_ptr + E + 1);
    blob.insert(blob.end(), h_c_col, h_c_col + nc);
    std::vector<float> inv(2 * E, 1.0f), wts;
    wts.insert(wts.end(), h_v_val, h_v_val + nv);
    wts.insert(wts.end(), h_c_val, h_c_val + nc);
    wts.push_back(0.0f);
    // the transposes: a counting sort of the nonzeros by column, rows ascending within a column
    std::vector<int32_t> tt;
    std::vector<float> tw;
    tt.reserve(2 * (E + 1) + nv + nc);
    tw.reserve(nv + nc + 1);
    auto transpose = [&](const int32_t *ptr, const int32_t *col, const float *val, int64_t nnz) {
        const size_t p0 = tt.size();
        tt.resize(p0 + E + 1, 0);
        int32_t *tp = tt.data() + p0;
        for (int64_t i = 0; i < nnz; ++i) tp[col[i] + 1]++;
        for (int64_t j = 0; j < E; ++j) tp[j + 1] += tp[j];
        std::vector<int32_t> cur(tp, tp + E), mem(nnz);
        std::vector<float> w(nnz);
        for (int64_t m = 0; m < E; ++m)
            for (int32_t i = ptr[m]; i < ptr[m + 1]; ++i) {
                const int32_t k = cur[col[i]]++;
                mem[k] = (int32_t)m;
                w[k] = val[i];
            }
        tt.insert(tt.end(), mem.begin(), mem.end());
        tw.insert(tw.end(), w.begin(), w.end());
    };
    transpose(h_v_ptr, h_v_col, h_v_val, nv);
    transpose(h_c_ptr, h_c_col, h_c_val, nc);
    tw.push_back(0.0f);
    auto *p = new ldpc_gnn_plan();
    p->E = E;
    p->Gv = (int)E;
    p->Gc = (int)E;
    p->weighted = true;
    if (hipGetDevice(&p->device) != hipSuccess || hipMalloc(&p->d_tab, blob.size() * 4) != hipSuccess ||
        hipMalloc(&p->d_inv, inv.size() * 4) != hipSuccess || hipMalloc(&p->d_w, wts.size() * 4) != hipSuccess ||
        hipMalloc(&p->d_tt, tt.size() * 4) != hipSuccess || hipMalloc(&p->d_tw, tw.size() * 4) != hipSuccess) {
        ldpc_gnn_plan_destroy(p);
        return fail(LDPC_EHIP, "GNN plan allocation failed");
    }
    if (hipMemcpy(p->d_tab, blob.data(), blob.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_inv, inv.data(), inv.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_w, wts.data(), wts.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_tt, tt.data(), tt.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_tw, tw.data(), tw.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        ldpc_gnn_plan_destroy(p);
        return fail(LDPC_EHIP, "GNN plan upload failed");
    }
    p->vgroup = p->d_tab;
    p->cgroup = p->vgroup + E;
    p->vg_ptr = p->cgroup + E;
    p->vg_mem = p->vg_ptr + E + 1;
    p->cg_ptr = p->vg_mem + nv;
    p->cg_mem = p->cg_ptr + E + 1;
    p->inv_v = p->d_inv;
    p->inv_c = p->d_inv + E;
    p->vg_w = p->d_w;
    p->cg_w = p->d_w + nv;
    p->vt_ptr = p->d_tt;
    p->vt_mem = p->vt_ptr + E + 1;
    p->ct_ptr = p->vt_mem + nv;
    p->ct_mem = p->ct_ptr + E + 1;
    p->vt_w = p->d_tw;
    p->ct_w = p->d_tw + nv;
    *out = p;
    return LDPC_OK;
}

extern "C" int ldpc_gnn_plan_destroy(ldpc_gnn_plan *p) {
    if (!p) return LDPC_OK;
    if (p->d_tab) (void)hipFree(p->d_tab);
    if (p->d_inv) (void)hipFree(p->d_inv);
    if (p->d_w) (void)hipFree(p->d_w);
    if (p->d_tt) (void)hipFree(p->d_tt);
    if (p->d_tw) (void)hipFree(p->d_tw);
    if (p->d_gt) (void)hipFree(p->d_gt);
    if (p->d_pt) (void)hipFree(p->d_pt);
    if (p->d_ct) (void)hipFree(p->d_ct);
    if (p->d_rw) (void)hipFree(p->d_rw);
    delete p;
    return LDPC_OK;
}

extern "C" int64_t ldpc_gnn_weights_size(int hidden, int types, int layers) {
    if (hidden <= 0 || types <= 0 || layers <= 0) return fail(LDPC_EINVAL, "bad GNN dimensions");
    return 2LL * hidden + (int64_t)layers * layer_floats(hidden, types);
}

extern "C" int64_t ldpc_gnn_workspace_size(const ldpc_gnn_plan *p, int hidden, int N, int64_t B, int layers,
                                           int precision) {
    if (!p || hidden <= 0 || N <= 0 || B < 0 || layers <= 0) return fail(LDPC_EINVAL, "bad arguments");
    if (precision == 1) return gnn_bf16_workspace(p, N, B, layers);
    return carve(p, hidden, N, B, layers, precision, nullptr).bytes;
}

int64_t ldpc::gnn_fp32_train_workspace(const ldpc_gnn_plan *p, int hidden, int N, int64_t B, int layers) {
    return carve(p, hidden, N, B, layers, 0, nullptr, true).bytes;
}

// the forward writes the area only on its projected-group path (the same predicate as its `proj`)
int64_t ldpc::gnn_proj_floats(const ldpc_gnn_plan *p, int hidden, int64_t B, int layers) {
    if (hidden != kMfmaH || p->weighted || p->n_ptiles <= 0 || !proj_path()) return 0;
    return (int64_t)layers * B * (p->Gv + p->Gc) * 2 * hidden;
}

int ldpc::gnn_fp32_forward(const ldpc_gnn_plan *p, int hidden, int types, int layers, const float *d_weights,
                           const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N, int64_t B,
                           float *d_probs, float *d_saved, void *d_work, int64_t work_bytes, hipStream_t s,
                           float *d_proj, bool fp32_products) {
    const int H = hidden;
    const bool train = d_saved != nullptr;
    Ws w = carve(p, H, N, B, layers, 0, d_work, train);
    if (!d_work || work_bytes < w.bytes)
        return fail(LDPC_EINVAL, "workspace too small: need " + std::to_string(w.bytes) + " bytes");
    if (!g_num_cus) {
        int dev = 0;
        LDPC_HIP(hipGetDevice(&dev));
        LDPC_HIP(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    if (int rc = gnn_build_var_csr(d_msg_var, p->E, N, w.csr, s)) return rc;
    GnnLayer L{};
    L.llr = d_llr;
    L.msg_var = d_msg_var;
    L.w_in = d_weights;
    L.b_in = d_weights + H;
    L.N = N;
    L.T = types;
    L.msg_type = d_msg_type;
    L.vgroup = p->vgroup; L.cgroup = p->cgroup;
    L.vg_ptr = p->vg_ptr; L.vg_mem = p->vg_mem; L.cg_ptr = p->cg_ptr; L.cg_mem = p->cg_mem;
    L.inv_v = p->inv_v; L.inv_c = p->inv_c;
    L.vg_w = p->vg_w; L.cg_w = p->cg_w;
    L.Gv = p->Gv; L.Gc = p->Gc;
    L.E = p->E; L.B = B;
    L.Mv = w.Mv; L.Mc = w.Mc;
    L.vside = 1;
    const bool mfma = H == kMfmaH;
    const bool wide = wide_on(p, H) && !train;
    if (!mfma && H > kMaxGenericH) return fail(LDPC_EUNSUPPORTED, "hidden_dim must be <= " + std::to_string(kMaxGenericH));
    const size_t mfma_lds = (size_t)(kOffEmb + types * kEmbStride) * 4;
    if (mfma && mfma_lds > 160 * 1024) return fail(LDPC_EUNSUPPORTED, "too many message types for the LDS image");
    const int mt = 512;  // MLP workgroups of 8 waves (the default of every measured round)
    const void *mfma_fn = reinterpret_cast<const void *>(gnn_mlp_mfma_kernel<512>);
    if (mfma) LDPC_HIP(hipFuncSetAttribute(mfma_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mfma_lds));
    // projected-group path (H = 64, group plans; LDPC_GNN_PROJ=0 selects the per-message [c; g]
    // kernels for A/B runs)
    const bool proj = mfma && !p->weighted && p->n_ptiles > 0 && proj_path();
    // projection workgroups of 12 waves (one LDS weight image for 12 waves' gathers) when the
    // type table leaves room, else 4
    const int proj_nt = LDPC_PROJ_NT != 256 && proj_lds_bytes(types, LDPC_PROJ_NT / 64) <= 160 * 1024 ? LDPC_PROJ_NT : 256;
    const bool split = !fp32_products && split_path() && mlp2s_lds_bytes(types, false) <= 160 * 1024;
    // degree-1 message tiles first (gnn_mlp2s_kernel) when the combined image fits
    const bool d1t = split && p->n_mtiles_v1 > 0 && mlp2s_lds_bytes(types, true) <= 160 * 1024 && d1_skip();
    // row walk (gnn_mlp2s_kernel RW): check tile groups, per-check sums out of the MLP (w.S set by carve)
    const bool rw = split && w.S && rowwalk_path();
    const bool rwd1 = rw && p->rw_d1 && mlp2s_lds_bytes(types, true) <= 160 * 1024 && d1_skip();
    // the staged check rows need 8 KB per wave beside the images (types up to ~50 at 8 waves)
    const bool pc_lds = rw && LDPC_S6_PCLDS && pclds_path() && mlp2s_rw_lds_bytes(types, true, kMlp2sNt / 64) <= 160 * 1024;
    const size_t proj_lds = proj_lds_bytes(types, proj_nt / 64),
                 mlp2_lds = split ? (pc_lds ? mlp2s_rw_lds_bytes(types, rwd1, kMlp2sNt / 64) : mlp2s_lds_bytes(types, rw ? rwd1 : d1t))
                                  : mlp2_lds_bytes(types);
    const void *proj_fn = fp32_products
                              ? (proj_nt != 256 ? reinterpret_cast<const void *>(gnn_group_proj_kernel<LDPC_PROJ_NT, false, false>)
                                                : reinterpret_cast<const void *>(gnn_group_proj_kernel<256, false, false>))
                              : (proj_nt != 256 ? reinterpret_cast<const void *>(gnn_group_proj_kernel<LDPC_PROJ_NT>)
                                                : reinterpret_cast<const void *>(gnn_group_proj_kernel<256>));
    // the row walk's projection without the generic typed gather (see gnn_group_proj_kernel)
    const void *proj_fn_rw = proj_nt != 256 ? reinterpret_cast<const void *>(gnn_group_proj_kernel<LDPC_PROJ_NT, false, true, false>)
                                            : reinterpret_cast<const void *>(gnn_group_proj_kernel<256, false, true, false>);
    int mlp2_per_cu = 1, proj_per_cu = 1;
    if (proj) {
        if (mlp2_lds > 160 * 1024 || proj_lds > 160 * 1024)
            return fail(LDPC_EUNSUPPORTED, "too many message types for the LDS image");
        proj_per_cu = std::max<int>(1, std::min<int>(3, (int)((160 * 1024) / proj_lds)));
        // workgroups per CU: bounded by LDS and by kMlp2Wps waves per SIMD
        mlp2_per_cu = std::max<int>(1, std::min<int>(4 * kMlp2Wps / (kMlp2Nt / 64), (int)((160 * 1024) / mlp2_lds)));
        LDPC_HIP(hipFuncSetAttribute(proj_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)proj_lds));
        LDPC_HIP(hipFuncSetAttribute(proj_fn_rw, hipFuncAttributeMaxDynamicSharedMemorySize, (int)proj_lds));
        LDPC_HIP(hipFuncSetAttribute(split ? (rw ? (pc_lds ? reinterpret_cast<const void *>(gnn_mlp2s_kernel<kMlp2sNt, kMlp2sWps, false, true, true>)
                                                           : reinterpret_cast<const void *>(gnn_mlp2s_kernel<kMlp2sNt, kMlp2sWps, false, true>))
                                                 : reinterpret_cast<const void *>(gnn_mlp2s_kernel<kMlp2sNt, kMlp2sWps, false>))
                                           : reinterpret_cast<const void *>(gnn_mlp2_kernel<kMlp2Nt, kMlp2Wps>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlp2_lds));
    }
    if (proj && rw) {  // every layer's mean type embedding per check group, once per call
        const int64_t n = (int64_t)layers * p->Gc * 64;
        hipLaunchKernelGGL(gnn_memb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_weights + 2 * H,
                           layer_floats(H, types), d_msg_type, p->cg_ptr, p->cg_mem, p->inv_c, p->Gc, layers, w.memb);
        LDPC_CHECK_LAUNCH("gnn_memb_kernel");
        const int64_t nv = (int64_t)layers * p->Gv * 64;
        hipLaunchKernelGGL(gnn_memb_kernel, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, d_weights + 2 * H,
                           layer_floats(H, types), d_msg_type, p->vg_ptr, p->vg_mem, p->inv_v, p->Gv, layers, w.memb_v);
        LDPC_CHECK_LAUNCH("gnn_memb_kernel");
    }
    // wide H = 96 / 128 on f16 splits: every layer's fused-MLP slice images, once per call
    const bool wfused = wide && !fp32_products && w.wimg && gnn_wide_fused_fits(H, types);
    if (wfused)
        if (int rc = gnn_wide_prep(H, layers, d_weights, layer_floats(H, types), types, w.wimg, w.wexp, s)) return rc;
    if (wide && w.wmemb)
        if (int rc = gnn_wide_memb(p, H, layers, d_weights + 2 * H, layer_floats(H, types), d_msg_type, w.wmemb, s)) return rc;
    // frames [b0, b0 + nb) through every layer on stream st (pointers offset to the range)
    const GnnLayer L0 = L;
    auto run_range = [&](int64_t b0, int64_t nb, hipStream_t st) -> int {
    GnnLayer L = L0;
    L.B = nb;
    L.llr = d_llr + b0 * N;
    L.Mv = w.Mv + b0 * p->Gv * H;
    L.Mc = w.Mc + b0 * p->Gc * H;
    const int64_t xoff = b0 * p->E * H;
    const float *x_in = nullptr;
    for (int l = 0; l < layers; ++l) {
        const float *lw = d_weights + 2 * H + (int64_t)l * layer_floats(H, types);
        L.emb = lw;
        L.w1v = L.emb + (int64_t)types * H;
        L.b1v = L.w1v + 2LL * H * H;
        L.w2v = L.b1v + H;
        L.b2v = L.w2v + (int64_t)H * H;
        L.w1c = L.b2v + H;
        L.b1c = L.w1c + 2LL * H * H;
        L.w2c = L.b1c + H;
        L.b2c = L.w2c + (int64_t)H * H;
        L.wo = L.b2c + H;
        L.bo = L.wo + H;
        L.x_in = x_in;
        L.residual = l > 0;
        L.last = l == layers - 1;
        L.x_out = d_saved ? d_saved + (int64_t)l * B * p->E * H + xoff
                          : L.last ? nullptr : ((l % 2 == 0) ? w.xa : w.xb) + xoff;
        L.msg_out = w.msg_out + b0 * p->E;
        if (wide) {
            GnnWideLayer W{};
            W.plan = p;
            W.H = H; W.T = types; W.N = N; W.B = nb; W.E = p->E;
            W.x_in = x_in;
            W.llr = L.llr; W.msg_type = d_msg_type; W.msg_var = d_msg_var; W.w_in = L.w_in; W.b_in = L.b_in;
            W.emb = L.emb; W.w1v = L.w1v; W.b1v = L.b1v; W.w2v = L.w2v; W.b2v = L.b2v;
            W.w1c = L.w1c; W.b1c = L.b1c; W.w2c = L.w2c; W.b2c = L.b2c; W.wo = L.wo; W.bo = L.bo;
            W.Mv = L.Mv; W.Mc = L.Mc;
            W.Pv = w.Pv + b0 * p->Gv * H; W.Pc = w.Pc + b0 * p->Gc * H;
            W.hbuf = w.hbuf + b0 * p->E * 2 * H;
            W.y = L.x_out ? L.x_out : ((l % 2 == 0) ? w.xa : w.xb) + xoff;  // the last layer: a free buffer
            W.residual = l > 0;
            W.msg_out = L.last ? L.msg_out : nullptr;
            W.f16 = !fp32_products;
            const int64_t roff = b0 * p->E;
            W.xmax_in = l > 0 ? w.xmax[(l - 1) & 1] + roff : nullptr;
            W.xmax_out = w.xmax[l & 1] + roff;
            W.hmax = w.hmax + roff;
            W.gmax_v = w.gmax_v + b0 * p->Gv;
            W.gmax_c = w.gmax_c + b0 * p->Gc;
            W.wimg = wfused ? w.wimg + (int64_t)l * (gnn_wide_fused_bytes(H, 1)) : nullptr;
            W.wexp = wfused ? w.wexp + 2 * l : nullptr;
            W.memb = w.wmemb ? w.wmemb + (int64_t)l * (p->Gv + p->Gc) * H : nullptr;
            if (int rc = gnn_wide_layer(W, st)) return rc;
            x_in = W.y;
            continue;
        }
        const int64_t waves = nb * (int64_t)(p->Gv + p->Gc);
        L.d1 = H == 64 && gm_tiles() && d1_skip() && !p->weighted;
        if (proj) {
            L.d1 = 0;
            if (rw) {
                L.rw_meta = p->rw_meta;
                L.rw_n = p->n_rw;
                L.ntile_v1 = rwd1;
                L.S_in = l > 0 ? w.S + b0 * p->Gc * H : nullptr;
                L.S_out = l + 1 < layers ? w.S + b0 * p->Gc * H : nullptr;
                L.memb = w.memb + (int64_t)l * p->Gc * H;
                L.memb_v = w.memb_v + (int64_t)l * p->Gv * H;
            } else if (d1t) {
                L.tperm = p->mt_perm;
                L.ntile_pf = p->n_mtiles;
                L.ntile_v1 = p->n_mtiles_v1;
            }
            // training with saved projections (d_proj): this layer's projected rows and group means go
            // to d_proj for the backward, every var group's included (the backward's GEMM1 reads them)
            bool skip_v1 = rw ? rwd1 : d1t;
            if (d_proj) {
                const int64_t G = p->Gv + p->Gc;
                float *base = d_proj + (int64_t)l * B * G * 2 * H;
                L.Mv = base + b0 * p->Gv * H;
                L.Mc = base + B * p->Gv * H + b0 * p->Gc * H;
                L.gsave_v = base + B * G * H + b0 * p->Gv * H;
                L.gsave_c = base + B * G * H + B * p->Gv * H + b0 * p->Gc * H;
                skip_v1 = false;
            }
            const ProjTiles T{p->pt_meta, p->pt_grp, p->pt_deg, p->pt_mem, p->n_ptiles, skip_v1 ? p->n_ptiles_v1 : 0};
            const int64_t ptiles = nb * (int64_t)p->n_ptiles;
            const int pw = proj_nt / 64;
            const unsigned pgrid = (unsigned)std::min<int64_t>((ptiles + pw - 1) / pw, (int64_t)g_num_cus * proj_per_cu);
            // the row walk's tiles never take the typed gather: without x_in they read the LLRs, with it
            // the check side reads the sums S_in and the var side the mean embeddings memb_v (set above)
            const bool gen = !(rw && L.memb_v && (!L.x_in || L.S_in));
            if (!fp32_products && !gen && proj_nt != 256)
                hipLaunchKernelGGL((gnn_group_proj_kernel<LDPC_PROJ_NT, false, true, false>), dim3(pgrid), dim3(LDPC_PROJ_NT), proj_lds, st, L, T);
            else if (!fp32_products && !gen)
                hipLaunchKernelGGL((gnn_group_proj_kernel<256, false, true, false>), dim3(pgrid), dim3(256), proj_lds, st, L, T);
            else if (fp32_products && proj_nt != 256)
                hipLaunchKernelGGL((gnn_group_proj_kernel<LDPC_PROJ_NT, false, false>), dim3(pgrid), dim3(LDPC_PROJ_NT), proj_lds, st, L, T);
            else if (fp32_products)
                hipLaunchKernelGGL((gnn_group_proj_kernel<256, false, false>), dim3(pgrid), dim3(256), proj_lds, st, L, T);
            else if (proj_nt != 256)
                hipLaunchKernelGGL(gnn_group_proj_kernel<LDPC_PROJ_NT>, dim3(pgrid), dim3(LDPC_PROJ_NT), proj_lds, st, L, T);
            else
                hipLaunchKernelGGL(gnn_group_proj_kernel<256>, dim3(pgrid), dim3(256), proj_lds, st, L, T);
            LDPC_CHECK_LAUNCH("gnn_group_proj_kernel");
            const int64_t tiles = d1t ? nb * p->n_mtiles : (nb * p->E + 31) / 32;
            constexpr int wpb = kMlp2Nt / 64;
            const unsigned grid = (unsigned)std::min<int64_t>((tiles + wpb - 1) / wpb, (int64_t)g_num_cus * mlp2_per_cu);
            if (rw) {
                const dim3 rgrid((unsigned)std::min<int64_t>((nb * p->n_rw + kMlp2sNt / 64 - 1) / (kMlp2sNt / 64), (int64_t)g_num_cus));
                if (pc_lds)
                    hipLaunchKernelGGL((gnn_mlp2s_kernel<kMlp2sNt, kMlp2sWps, false, true, true>), rgrid, dim3(kMlp2sNt), mlp2_lds, st, L);
                else
                    hipLaunchKernelGGL((gnn_mlp2s_kernel<kMlp2sNt, kMlp2sWps, false, true>), rgrid, dim3(kMlp2sNt), mlp2_lds, st, L);
            }
            else if (split)
                hipLaunchKernelGGL((gnn_mlp2s_kernel<kMlp2sNt, kMlp2sWps, false>),
                                   dim3((unsigned)std::min<int64_t>((tiles + kMlp2sNt / 64 - 1) / (kMlp2sNt / 64), (int64_t)g_num_cus)),
                                   dim3(kMlp2sNt), mlp2_lds, st, L);
            else
                hipLaunchKernelGGL((gnn_mlp2_kernel<kMlp2Nt, kMlp2Wps>), dim3(grid), dim3(kMlp2Nt), mlp2_lds, st, L);
            LDPC_CHECK_LAUNCH("gnn_mlp2_kernel");
            x_in = L.x_out;
            continue;
        }
        if (p->weighted)  // general adjacency: weighted rows, one wave per (frame, message row)
            hipLaunchKernelGGL(gnn_group_mean_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, L, H);
        else if (H == 64 && gm_tiles()) {
            const GtTiles G{p->gt_meta, p->gt_grp, p->gt_mem, p->n_gtiles, L.d1 ? p->n_gtiles_v1 : 0};
            const int64_t twaves = nb * (int64_t)(G.n_tiles - G.first);
            hipLaunchKernelGGL(gnn_group_mean_tile_kernel, dim3((unsigned)((twaves + 3) / 4)), dim3(256), 0, st, L, G);
        } else if (H == 64)
            hipLaunchKernelGGL(gnn_group_mean_h64_kernel, dim3((unsigned)((waves + 15) / 16)), dim3(256), 0, st, L);
        else
            hipLaunchKernelGGL(gnn_group_mean_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, L, H);
        LDPC_CHECK_LAUNCH("gnn_group_mean_kernel");
        if (mfma) {
            const int64_t tiles = (nb * p->E + 31) / 32;
            const int64_t want = (tiles + mt / 64 - 1) / (mt / 64);
            const unsigned grid = (unsigned)std::min<int64_t>(want, (int64_t)g_num_cus);
            hipLaunchKernelGGL(gnn_mlp_mfma_kernel<512>, dim3(grid), dim3(512), mfma_lds, st, L);
            LDPC_CHECK_LAUNCH("gnn_mlp_mfma_kernel");
        } else {
            if (w.wt) {  // tiled: kTiledNM messages per wave over the layer's transposed weights
                GnnLayer T = L;
                T.wt = w.wt + 6LL * H * H * l;
                const int tw = tiled_waves(H);
                const int64_t want = (nb * p->E + (int64_t)tw * kTiledNM - 1) / ((int64_t)tw * kTiledNM);
                const unsigned grid = (unsigned)std::min<int64_t>(want, (int64_t)std::max(1, g_num_cus * 16 / tw));
                const size_t tl = (size_t)tw * kTiledNM * 4 * H * 4;
                if (tl > 64 * 1024)
                    LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(gnn_mlp_tiled_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)tl));
                hipLaunchKernelGGL(gnn_mlp_tiled_kernel, dim3(grid), dim3(64 * tw), (size_t)tw * kTiledNM * 4 * H * 4, st,
                                   T, H);
                LDPC_CHECK_LAUNCH("gnn_mlp_tiled_kernel");
            } else {
                const int64_t want = (nb * p->E + 3) / 4;
                const unsigned grid = (unsigned)std::min<int64_t>(want, (int64_t)g_num_cus * 8);
                hipLaunchKernelGGL(gnn_mlp_generic_kernel, dim3(grid), dim3(256), (size_t)16 * H * 4, st, L, H);
                LDPC_CHECK_LAUNCH("gnn_mlp_generic_kernel");
            }
        }
        x_in = L.x_out;
    }
    return LDPC_OK;
    };
    if (w.wt) {  // the tiled kernel's transposed weights of every layer, on the caller's stream
        for (int l = 0; l < layers; ++l) {
            const float *lw = d_weights + 2 * H + (int64_t)l * layer_floats(H, types);
            const float *w1v = lw + (int64_t)types * H, *w2v = w1v + 2LL * H * H + H;
            const float *w1c = w2v + (int64_t)H * H + H, *w2c = w1c + 2LL * H * H + H;
            hipLaunchKernelGGL(gnn_wt_kernel, dim3((unsigned)((6LL * H * H + 255) / 256)), dim3(256), 0, s, w1v, w2v, w1c,
                               w2c, H, w.wt + 6LL * H * H * l);
            LDPC_CHECK_LAUNCH("gnn_wt_kernel");
        }
    }
    // Two frame halves on two streams (fork / join through events on the caller's stream): every
    // frame's layers stay in order on its stream, and the halves share no data.
    if (gnn_streams() == 2 && B >= 2 * 64) {
        hipStream_t s2;
        hipEvent_t fork, join;
        if (int rc = gnn_side_stream(&s2, &fork, &join)) return rc;
        const int64_t b1 = B / 2;
        LDPC_HIP(hipEventRecord(fork, s));
        LDPC_HIP(hipStreamWaitEvent(s2, fork, 0));
        if (int rc = run_range(0, b1, s)) return rc;
        if (int rc = run_range(b1, B - b1, s2)) return rc;
        LDPC_HIP(hipEventRecord(join, s2));
        LDPC_HIP(hipStreamWaitEvent(s, join, 0));
    } else if (int rc = run_range(0, B, s)) {
        return rc;
    }
    if (int rc = gnn_output(w.msg_out, w.csr, d_llr, p->E, N, B, nullptr, d_probs, s)) return rc;
    return LDPC_OK;
}

int ldpc::gnn_project_groups(const ldpc_gnn_plan *p, int types, const float *d_weights, int layer, const float *d_x,
                             const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N,
                             int64_t B, float *d_pv, float *d_pc, float *d_gv, float *d_gc, hipStream_t s) {
    constexpr int H = kMfmaH;
    if (p->weighted || p->n_ptiles <= 0) return fail(LDPC_EUNSUPPORTED, "group projection needs a group plan");
    if (!g_num_cus) {
        int dev = 0;
        LDPC_HIP(hipGetDevice(&dev));
        LDPC_HIP(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    GnnLayer L{};
    L.x_in = d_x;
    L.llr = d_llr;
    L.msg_var = d_msg_var;
    L.w_in = d_weights;
    L.b_in = d_weights + H;
    L.N = N;
    L.T = types;
    L.msg_type = d_msg_type;
    L.vgroup = p->vgroup; L.cgroup = p->cgroup;
    L.vg_ptr = p->vg_ptr; L.vg_mem = p->vg_mem; L.cg_ptr = p->cg_ptr; L.cg_mem = p->cg_mem;
    L.inv_v = p->inv_v; L.inv_c = p->inv_c;
    L.Gv = p->Gv; L.Gc = p->Gc;
    L.E = p->E; L.B = B;
    L.Mv = d_pv; L.Mc = d_pc;
    L.gsave_v = d_gv; L.gsave_c = d_gc;
    L.vside = 1;
    const float *lw = d_weights + 2 * H + (int64_t)layer * layer_floats(H, types);
    L.emb = lw;
    L.w1v = L.emb + (int64_t)types * H;
    L.b1v = L.w1v + 2LL * H * H;
    L.w2v = L.b1v + H;
    L.b2v = L.w2v + (int64_t)H * H;
    L.w1c = L.b2v + H;
    L.b1c = L.w1c + 2LL * H * H;
    L.w2c = L.b1c + H;
    const int proj_nt = LDPC_PROJ_NT != 256 && proj_lds_bytes(types, LDPC_PROJ_NT / 64) <= 160 * 1024 ? LDPC_PROJ_NT : 256;
    const size_t proj_lds = proj_lds_bytes(types, proj_nt / 64);
    if (proj_lds > 160 * 1024) return fail(LDPC_EUNSUPPORTED, "too many message types for the LDS image");
    const void *proj_fn = proj_nt != 256 ? reinterpret_cast<const void *>(gnn_group_proj_kernel<LDPC_PROJ_NT>)
                                         : reinterpret_cast<const void *>(gnn_group_proj_kernel<256>);
    LDPC_HIP(hipFuncSetAttribute(proj_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)proj_lds));
    const int per_cu = std::max<int>(1, std::min<int>(3, (int)((160 * 1024) / proj_lds)));
    const ProjTiles T{p->pt_meta, p->pt_grp, p->pt_deg, p->pt_mem, p->n_ptiles, 0};
    const int64_t ptiles = B * (int64_t)p->n_ptiles;
    const int pw = proj_nt / 64;
    const unsigned pgrid = (unsigned)std::min<int64_t>((ptiles + pw - 1) / pw, (int64_t)g_num_cus * per_cu);
    if (proj_nt != 256)
        hipLaunchKernelGGL(gnn_group_proj_kernel<LDPC_PROJ_NT>, dim3(pgrid), dim3(LDPC_PROJ_NT), proj_lds, s, L, T);
    else
        hipLaunchKernelGGL(gnn_group_proj_kernel<256>, dim3(pgrid), dim3(256), proj_lds, s, L, T);
    LDPC_CHECK_LAUNCH("gnn_group_proj_kernel (training backward)");
    return LDPC_OK;
}

extern "C" int ldpc_gnn_forward_ex(const ldpc_gnn_plan *p, int hidden, int types, int layers, const float *d_weights,
                                   const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N,
                                   int64_t B, int precision, int flags, float *d_probs, int32_t *d_iters,
                                   void *d_work, int64_t work_bytes, void *stream) {
    if (!p) return fail(LDPC_EINVAL, "plan is NULL");
    if (hidden <= 0 || types <= 0 || layers <= 0 || N <= 0 || B < 0) return fail(LDPC_EINVAL, "bad dimensions");
    if (precision != 0 && precision != 1) return fail(LDPC_EINVAL, "precision must be 0 (fp32) or 1 (bf16)");
    if (precision == 1 && hidden != kMfmaH) return fail(LDPC_EUNSUPPORTED, "bf16 path needs hidden_dim 64");
    if (flags & ~(LDPC_GNN_EARLY_STOP | LDPC_GNN_FP32_PRODUCTS)) return fail(LDPC_EINVAL, "unknown flags");
    if ((flags & LDPC_GNN_EARLY_STOP) && precision != 1)
        return fail(LDPC_EUNSUPPORTED, "early termination is implemented on the bf16 path (precision 1)");
    if (B == 0) return LDPC_OK;
    if (!d_weights || !d_msg_type || !d_msg_var || !d_llr || !d_probs) return fail(LDPC_EINVAL, "NULL tensor");
    if (precision == 1 && p->weighted)
        return fail(LDPC_EUNSUPPORTED, "the bf16 path needs a group plan (clique adjacencies); use precision 0");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (precision == 1)
        return gnn_bf16_forward(p, types, layers, d_weights, d_msg_type, d_msg_var, d_llr, N, B, flags, d_probs,
                                d_iters, d_work, work_bytes, s);
    if (d_iters) {  // no early termination: every frame runs every layer
        hipLaunchKernelGGL(gnn_fill_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, d_iters, B, layers);
        LDPC_CHECK_LAUNCH("gnn_fill_kernel");
    }
    return gnn_fp32_forward(p, hidden, types, layers, d_weights, d_msg_type, d_msg_var, d_llr, N, B, d_probs,
                            nullptr, d_work, work_bytes, s, nullptr, (flags & LDPC_GNN_FP32_PRODUCTS) != 0);
}

extern "C" int ldpc_gnn_forward(const ldpc_gnn_plan *p, int hidden, int types, int layers, const float *d_weights,
                                const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N,
                                int64_t B, int precision, float *d_probs, void *d_work, int64_t work_bytes,
                                void *stream) {
    return ldpc_gnn_forward_ex(p, hidden, types, layers, d_weights, d_msg_type, d_msg_var, d_llr, N, B, precision, 0,
                               d_probs, nullptr, d_work, work_bytes, stream);
}

// ------------------------------------------------------------------------ hybrid GNN host side
extern "C" int64_t ldpc_gnn_custom_var_workspace_size(const ldpc_gnn_plan *p, int hidden, int N, int64_t B, int layers) {
    if (!p || hidden <= 0 || N <= 0 || B < 0 || layers <= 0) return fail(LDPC_EINVAL, "bad arguments");
    // carve() with at least 3 layers keeps both feature buffers (H != 64: the tiled kernel's
    // transposed weights, never the wide path); + v2c (B, E)
    return carve(p, hidden, N, B, std::max(layers, 3), 0, nullptr, hidden != kMfmaH).bytes + (B * p->E * 4 + 255) / 256 * 256;
}

namespace ldpc {
namespace {
// The hybrid GNN at H != 64 (up to kTiledMaxH): the check side of the generic kernels -- weighted-free
// group means of the check groups (gnn_group_mean_kernel, vside 0), the tiled MLP over [c; b] with
// the layer's own output head, then the same variable update and output as H = 64.
int custom_var_forward_any(const ldpc_gnn_plan *p, int H, int types, int layers, const float *d_weights,
                           const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N, int64_t B,
                           float *d_probs, void *d_work, hipStream_t s) {
    Ws w = carve(p, H, N, B, std::max(layers, 3), 0, d_work, true);
    float *v2c = reinterpret_cast<float *>(static_cast<char *>(d_work) + w.bytes);
    if (!w.wt) return fail(LDPC_EUNSUPPORTED, "hidden_dim too wide for the hybrid GNN");
    if (!g_num_cus) {
        int dev = 0;
        LDPC_HIP(hipGetDevice(&dev));
        LDPC_HIP(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    if (int rc = gnn_build_var_csr(d_msg_var, p->E, N, w.csr, s)) return rc;
    GnnLayer L{};
    L.llr = d_llr; L.msg_var = d_msg_var; L.w_in = d_weights; L.b_in = d_weights + H; L.N = N; L.T = types;
    L.msg_type = d_msg_type;
    L.vgroup = p->vgroup; L.cgroup = p->cgroup; L.vg_ptr = p->vg_ptr; L.vg_mem = p->vg_mem;
    L.cg_ptr = p->cg_ptr; L.cg_mem = p->cg_mem; L.inv_v = p->inv_v; L.inv_c = p->inv_c;
    L.Gv = p->Gv; L.Gc = p->Gc; L.E = p->E; L.B = B; L.Mv = w.Mv; L.Mc = w.Mc;
    L.vside = 0; L.residual = 0; L.last = 1; L.d1 = 0;
    L.msg_out = w.msg_out;
    const int64_t R = B * p->E;
    const int tw = tiled_waves(H);
    const size_t tl = (size_t)tw * kTiledNM * 4 * H * 4;
    if (tl > 64 * 1024)
        LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(gnn_mlp_tiled_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)tl));
    const float *x_in = nullptr;
    for (int l = 0; l < layers; ++l) {
        const float *lw = d_weights + 2 * H + (int64_t)l * layer_floats(H, types);
        L.emb = lw;
        L.w1v = L.emb + (int64_t)types * H; L.b1v = L.w1v + 2LL * H * H; L.w2v = L.b1v + H; L.b2v = L.w2v + (int64_t)H * H;
        L.w1c = L.b2v + H; L.b1c = L.w1c + 2LL * H * H; L.w2c = L.b1c + H; L.b2c = L.w2c + (int64_t)H * H;
        L.wo = L.b2c + H; L.bo = L.wo + H;
        L.x_in = x_in;
        L.hv2c = l > 0 ? v2c : nullptr;        // layers >= 1 read x = (v2c w_in + b_in) + F_{l-1}
        L.x_out = (l % 2 == 0) ? w.xa : w.xb;  // F
        L.wt = w.wt + 6LL * H * H * l;
        hipLaunchKernelGGL(gnn_wt_kernel, dim3((unsigned)((6LL * H * H + 255) / 256)), dim3(256), 0, s, L.w1v, L.w2v,
                           L.w1c, L.w2c, H, w.wt + 6LL * H * H * l);
        LDPC_CHECK_LAUNCH("gnn_wt_kernel (hybrid)");
        const int64_t waves = B * (int64_t)(p->Gv + p->Gc);
        hipLaunchKernelGGL(gnn_group_mean_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, L, H);
        LDPC_CHECK_LAUNCH("gnn_group_mean_kernel (hybrid check side)");
        const int64_t want = (R + (int64_t)tw * kTiledNM - 1) / ((int64_t)tw * kTiledNM);
        const unsigned grid = (unsigned)std::min<int64_t>(want, (int64_t)std::max(1, g_num_cus * 16 / tw));
        hipLaunchKernelGGL(gnn_mlp_tiled_kernel, dim3(grid), dim3(64 * tw), tl, s, L, H);
        LDPC_CHECK_LAUNCH("gnn_mlp_tiled_kernel (hybrid check side)");
        hipLaunchKernelGGL(custom_var_llr_kernel, dim3((unsigned)((B * N + 255) / 256)), dim3(256), 0, s, w.msg_out, w.csr,
                           d_llr, p->E, N, B, v2c);
        LDPC_CHECK_LAUNCH("hybrid GNN variable update");
        if (l == layers - 1) {
            hipLaunchKernelGGL(custom_combine_any_kernel, dim3((unsigned)((R * 16 + 255) / 256)), dim3(256), 0, s, L.x_out,
                               v2c, d_weights, d_weights + H, H, R, L.wo, L.bo, w.msg_out);
            LDPC_CHECK_LAUNCH("hybrid GNN output head");
        }
        x_in = L.x_out;
    }
    hipLaunchKernelGGL(custom_output_kernel, dim3((unsigned)((B * N + 255) / 256)), dim3(256), 0, s, w.msg_out, w.csr, d_llr,
                       p->E, N, B * N, d_probs);
    LDPC_CHECK_LAUNCH("custom_output_kernel");
    return LDPC_OK;
}
}  // namespace
}  // namespace ldpc

extern "C" int ldpc_gnn_custom_var_forward(const ldpc_gnn_plan *p, int hidden, int types, int layers,
                                           const float *d_weights, const int32_t *d_msg_type,
                                           const int32_t *d_msg_var, const float *d_llr, int N, int64_t B,
                                           float *d_probs, void *d_work, int64_t work_bytes, void *stream) {
    if (!p) return fail(LDPC_EINVAL, "plan is NULL");
    if (hidden <= 0 || hidden > kTiledMaxH) return fail(LDPC_EUNSUPPORTED, "the hybrid GNN runs at hidden_dim <= 1024");
    if (p->weighted || p->n_ptiles == 0) return fail(LDPC_EUNSUPPORTED, "the hybrid GNN needs a group plan");
    if (types <= 0 || layers <= 0 || N <= 0 || B < 0) return fail(LDPC_EINVAL, "bad dimensions");
    if (B == 0) return LDPC_OK;
    if (!d_weights || !d_msg_type || !d_msg_var || !d_llr || !d_probs) return fail(LDPC_EINVAL, "NULL tensor");
    const int64_t need = ldpc_gnn_custom_var_workspace_size(p, hidden, N, B, layers);
    if (!d_work || work_bytes < need) return fail(LDPC_EINVAL, "workspace too small: need " + std::to_string(need) + " bytes");
    if (B * p->E >= (1LL << 31) / 16) return fail(LDPC_EUNSUPPORTED, "batch too large for one launch (chunk it)");
    if (hidden != kMfmaH)
        return custom_var_forward_any(p, hidden, types, layers, d_weights, d_msg_type, d_msg_var, d_llr, N, B, d_probs,
                                      d_work, static_cast<hipStream_t>(stream));
    const int H = kMfmaH;
    hipStream_t s = static_cast<hipStream_t>(stream);
    Ws w = carve(p, H, N, B, std::max(layers, 3), 0, d_work);
    float *v2c = reinterpret_cast<float *>(static_cast<char *>(d_work) + w.bytes);
    if (!g_num_cus) {
        int dev = 0;
        LDPC_HIP(hipGetDevice(&dev));
        LDPC_HIP(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const bool split = split_path() && mlp2s_lds_bytes(types, false) <= 160 * 1024;
    const size_t proj_lds = proj_lds_bytes(types, 4), mlp2_lds = split ? mlp2s_lds_bytes(types, false) : mlp2_lds_bytes(types);
    if (proj_lds > 160 * 1024 || mlp2_lds > 160 * 1024) return fail(LDPC_EUNSUPPORTED, "too many message types for the LDS image");
    LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(gnn_group_proj_kernel<256, true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)proj_lds));
    LDPC_HIP(hipFuncSetAttribute(split ? reinterpret_cast<const void *>(gnn_mlp2s_kernel<kMlp2sNt, kMlp2sWps, true>)
                                       : reinterpret_cast<const void *>(gnn_mlp2_kernel<kMlp2Nt, kMlp2Wps, true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlp2_lds));
    const int mlp2_per_cu = std::max<int>(1, std::min<int>(4 * kMlp2Wps / (kMlp2Nt / 64), (int)((160 * 1024) / mlp2_lds)));
    const int proj_per_cu = std::max<int>(1, std::min<int>(3, (int)((160 * 1024) / proj_lds)));
    if (int rc = gnn_build_var_csr(d_msg_var, p->E, N, w.csr, s)) return rc;
    GnnLayer L{};
    L.llr = d_llr; L.msg_var = d_msg_var; L.w_in = d_weights; L.b_in = d_weights + H; L.N = N; L.T = types;
    L.msg_type = d_msg_type;
    L.vgroup = p->vgroup; L.cgroup = p->cgroup; L.vg_ptr = p->vg_ptr; L.vg_mem = p->vg_mem;
    L.cg_ptr = p->cg_ptr; L.cg_mem = p->cg_mem; L.inv_v = p->inv_v; L.inv_c = p->inv_c;
    L.Gv = p->Gv; L.Gc = p->Gc; L.E = p->E; L.B = B; L.Mv = w.Mv; L.Mc = w.Mc;
    L.vside = 0; L.residual = 0; L.last = 1; L.d1 = 0;
    L.msg_out = w.msg_out;
    const ProjTiles T{p->pt_meta, p->pt_grp, p->pt_deg, p->pt_mem, p->n_ptiles, p->n_ptiles_v};
    const int64_t R = B * p->E;
    const float *x_in = nullptr;
    for (int l = 0; l < layers; ++l) {
        const float *lw = d_weights + 2 * H + (int64_t)l * layer_floats(H, types);
        L.emb = lw;
        L.w1v = L.emb + (int64_t)types * H; L.b1v = L.w1v + 2LL * H * H; L.w2v = L.b1v + H; L.b2v = L.w2v + (int64_t)H * H;
        L.w1c = L.b2v + H; L.b1c = L.w1c + 2LL * H * H; L.w2c = L.b1c + H; L.b2c = L.w2c + (int64_t)H * H;
        L.wo = L.b2c + H; L.bo = L.wo + H;
        L.x_in = x_in;
        L.hv2c = l > 0 ? v2c : nullptr;        // layers >= 1 read x = (v2c w_in + b_in) + F_{l-1}
        L.x_out = (l % 2 == 0) ? w.xa : w.xb;  // F
        const int64_t ptiles = B * (int64_t)(T.n_tiles - T.first);
        hipLaunchKernelGGL((gnn_group_proj_kernel<256, true>), dim3((unsigned)std::min<int64_t>((ptiles + 3) / 4, (int64_t)g_num_cus * proj_per_cu)),
                           dim3(256), proj_lds, s, L, T);
        LDPC_CHECK_LAUNCH("gnn_group_proj_kernel (check side)");
        constexpr int wpb = kMlp2Nt / 64;
        const int64_t tiles = (R + 31) / 32;
        const dim3 mgrid((unsigned)std::min<int64_t>((tiles + wpb - 1) / wpb, (int64_t)g_num_cus * mlp2_per_cu));
        if (split)
            hipLaunchKernelGGL((gnn_mlp2s_kernel<kMlp2sNt, kMlp2sWps, true>),
                               dim3((unsigned)std::min<int64_t>((tiles + kMlp2sNt / 64 - 1) / (kMlp2sNt / 64), (int64_t)g_num_cus)),
                               dim3(kMlp2sNt), mlp2_lds, s, L);
        else
            hipLaunchKernelGGL((gnn_mlp2_kernel<kMlp2Nt, kMlp2Wps, true>), mgrid, dim3(kMlp2Nt), mlp2_lds, s, L);
        LDPC_CHECK_LAUNCH("gnn_mlp2_kernel (check side)");
        hipLaunchKernelGGL(custom_var_llr_kernel, dim3((unsigned)((B * N + 255) / 256)), dim3(256), 0, s, w.msg_out, w.csr,
                           d_llr, p->E, N, B, v2c);
        LDPC_CHECK_LAUNCH("hybrid GNN variable update");
        if (l == layers - 1)  // x_L and the decoder's output head, the last layer's (:855)
            hipLaunchKernelGGL(custom_combine_kernel, dim3((unsigned)((R * 16 + 255) / 256)), dim3(256), 0, s, L.x_out,
                               v2c, d_weights, d_weights + H, R, L.wo, L.bo, w.msg_out);
        LDPC_CHECK_LAUNCH("hybrid GNN output head");
        x_in = L.x_out;
    }
    hipLaunchKernelGGL(custom_output_kernel, dim3((unsigned)((B * N + 255) / 256)), dim3(256), 0, s, w.msg_out, w.csr, d_llr,
                       p->E, N, B * N, d_probs);
    LDPC_CHECK_LAUNCH("custom_output_kernel");
    return LDPC_OK;
}
