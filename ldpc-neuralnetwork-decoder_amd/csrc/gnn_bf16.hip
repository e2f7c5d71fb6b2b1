// gnn_bf16.hip -- message-GNN forward, bf16 features on v_mfma_f32_32x32x16_bf16 (precision 1).
//
// Same layer as gnn.hip (message_gnn_decoder.py:51-129, :190-317), re-associated so that the
// per-message work is MFMA + a few VALU ops:
//
//   MLP_s([c; g]) with c = x + emb[type] and g the group mean of c (s = var side / check side)
//     W1_s [c; g] + b1_s = W1_s,left x  +  (W1_s,left emb[type] + b1_s)  +  W1_s,right g
//   The bracket depends only on (layer, type, side): a "type constant" K[t][s], computed once
//   per forward by gnn_bf16_kconst_kernel and used as the GEMM1 accumulator's initial value.
//   Layer 0 has x = w_in llr + b_in, so W1_s,left x = llr * (W1_s,left w_in) + W1_s,left b_in:
//   two more constant vectors (U, V) and GEMM1 over x disappears.
//   The group means keep the emb part: g = mean(x) + mean(emb[type]) where the second term is
//   a per-(layer, group) constant (gnn_bf16_memb_kernel).
//   A var group of degree 1 (1216 of 1664 at BG2 Z = 32) has g = c = x + emb[type]: from layer 1
//   on its message skips the group-mean row altogether and feeds its own x as g, with
//   W1_v,right emb[type] folded into a third type constant D1[t] (no Mv write, no Mv gather).
//
// Feature storage order.  A 64-feature row is stored permuted: stored position p = 16 s + 8 h + i
// holds logical unit pi(p) = 32 (s>>1) + 16 (s&1) + 8 (i>>2) + 4 h + (i&3).  Then the 16-byte
// chunk s that lane (j, h) loads as the k-step-s B operand of GEMM1 holds exactly the units that
// the same lane owns in its 32x32 accumulator (row tile s>>1, registers 8 (s&1) .. +7).  So the
// residual add needs no reload and no shuffle, and the output row is written as four 16-B
// chunks straight from the accumulators.  W1's columns are permuted to match; Mv/Mc rows use
// the same order; the logical order never appears in memory.
//
// Kernels per layer:
//   gnn_bf16_gm_kernel   group means (bf16 rows).  One wave sums 8 groups of one degree (a
//                        "group tile", see gnn.hpp), 8 lanes x 16 B per 128-B row.
//   gnn_bf16_mlp_kernel  persistent, weights (bf16) + type constants in LDS; one wave per
//                        32-message tile: GEMM1 (K = 64 x-part + 64 group-part) -> ReLU -> GEMM2
//                        for both sides into one accumulator, + b2v + b2c + residual, bf16 out.
//                        Last layer: output projection + per-variable sum instead.
//   gnn_bf16_syndrome_kernel  (early termination, cfg5) per frame, after every layer but the
//                        last: hard decision through the last layer's output projection on the
//                        current features, parity checks; a satisfied frame writes its probs
//                        and every later kernel skips it.
#include <cstdint>
#include <string>

#include "common.hpp"
#include "gnn.hpp"

namespace ldpc {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int H = 64;
constexpr int kMlpThreads = 512;  // the MLP kernel's workgroup (8 waves): one per CU, 2 waves per SIMD

__host__ __device__ constexpr int pi_unit(int p) {
    return 32 * (p >> 5) + 16 * ((p >> 4) & 1) + 8 * ((p >> 2) & 1) + 4 * ((p >> 3) & 1) + (p & 3);
}
// accumulator order: index a = 32 rt + 16 h + r (row tile rt, lane half h, register r) -> unit
__host__ __device__ constexpr int acc_unit(int a) {
    return 32 * (a >> 5) + (a & 3) + 8 * ((a >> 2) & 3) + 4 * ((a >> 4) & 1);
}

struct LayerW {
    const float *emb, *w1v, *b1v, *w2v, *b2v, *w1c, *b1c, *w2c, *b2c, *wo, *bo;
};
__host__ __device__ inline int64_t layer_floats(int T) { return (int64_t)T * H + 2 * (2 * H * H + H + H * H + H) + H + 1; }
__host__ __device__ inline LayerW layer_w(const float *blob, int T, int l) {
    LayerW w;
    w.emb = blob + 2 * H + (int64_t)l * layer_floats(T);
    w.w1v = w.emb + (int64_t)T * H;
    w.b1v = w.w1v + 2 * H * H;
    w.w2v = w.b1v + H;
    w.b2v = w.w2v + H * H;
    w.w1c = w.b2v + H;
    w.b1c = w.w1c + 2 * H * H;
    w.w2c = w.b1c + H;
    w.b2c = w.w2c + H * H;
    w.wo = w.b2c + H;
    w.bo = w.wo + H;
    return w;
}

// derived constants per layer (floats): K[T + 2][2 sides][64 acc order] (rows T, T+1 = U, V of
// layer 0), then b2v + b2c [64 acc], wo [64 acc], then D1[T][64 acc] = K[t][var side] +
// W1_v,right emb[t] (degree-1 var groups)
__host__ __device__ inline int64_t kd_floats(int T) { return (int64_t)(T + 2) * 128 + 128 + (int64_t)T * 64; }
__host__ __device__ inline int64_t kd_d1(int T) { return (int64_t)(T + 3) * 128; }

__global__ __launch_bounds__(128) void gnn_bf16_kconst_kernel(const float *blob, int T, float *kd) {
    const int l = blockIdx.x, t = blockIdx.y, side = threadIdx.x >> 6, a = threadIdx.x & 63;
    const int u = acc_unit(a);
    const LayerW w = layer_w(blob, T, l);
    const float *W1 = (side ? w.w1c : w.w1v) + u * 2 * H;  // row u, left half = columns 0..63
    const float *v = t < T ? w.emb + t * H : t == T ? blob : blob + H;  // emb[t] | w_in | b_in
    float s = t < T ? (side ? w.b1c : w.b1v)[u] : 0.0f;
    for (int k = 0; k < H; ++k) s = fmaf(W1[k], v[k], s);
    float *out = kd + (int64_t)l * kd_floats(T);
    out[(int64_t)t * 128 + side * 64 + a] = s;
    if (t < T && side == 0) {
        float d = s;
        for (int k = 0; k < H; ++k) d = fmaf(W1[H + k], v[k], d);
        out[kd_d1(T) + (int64_t)t * 64 + a] = d;
    }
    if (t == 0 && side == 0) {
        out[(int64_t)(T + 2) * 128 + a] = w.b2v[u] + w.b2c[u];
        out[(int64_t)(T + 2) * 128 + 64 + a] = w.wo[u];
    }
}

// Per tile slot i = 32 k + j (lane j of a frame's tile k, gnn.hpp ct_m0):
//   info[i] = {var group, or ~var group (< 0) for a degree-1 var group when `d1` (see header),
//              check group, type, variable} of the slot's message
//   slot[i] = {message, or ~message of the tile's last one for a padding slot; mask of the tile
//              slots holding the message's check group (aligned tiles), 0 for padding}
__global__ void gnn_bf16_info_kernel(int nslots, const int32_t *ct_m0, int aligned, const int32_t *vgroup,
                                     const int32_t *vg_ptr, int d1, const int32_t *cgroup, const int32_t *cg_ptr,
                                     const int32_t *cg_mem, const int32_t *msg_type, const int32_t *msg_var,
                                     int4 *info, int2 *slot) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nslots) return;
    const int k = i >> 5, j = i & 31;
    const int m0 = ct_m0[k], n = ct_m0[k + 1] - m0;
    const int m = m0 + (j < n ? j : n - 1);
    const int g = vgroup[m], cg = cgroup[m];
    const bool one = d1 && vg_ptr[g + 1] - vg_ptr[g] == 1;
    info[i] = make_int4(one ? ~g : g, cg, msg_type[m], msg_var[m]);
    uint32_t mask = 0;
    if (aligned && j < n) {
        const int d = cg_ptr[cg + 1] - cg_ptr[cg], s = cg_mem[cg_ptr[cg]] - m0;
        mask = (d >= 32 ? 0xFFFFFFFFu : ((1u << d) - 1u)) << s;
    }
    slot[i] = make_int2(j < n ? m : ~m, (int)mask);
}

struct GtArgs {
    const int2 *meta;
    const int32_t *grp, *mem;
    int n_tiles;
    int first;  // group-mean launches start at this tile (skipping degree-1 var tiles)
};

// memb[l][g][p] = mean over group g's messages of emb_l[type][pi(p)]  (one wave per (l, tile));
// memb16: the same rows in bf16 (the MLP's in-tile check means: 16 instead of 32 registers per
// prefetched tile)
__global__ __launch_bounds__(256) void gnn_bf16_memb_kernel(const float *blob, int T, int L, const int32_t *msg_type,
                                                            GtArgs G, int Gtot, float *memb, __bf16 *memb16) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= (int64_t)L * G.n_tiles) return;
    const int l = (int)(w / G.n_tiles), t = (int)(w - (int64_t)l * G.n_tiles);
    const int lane = threadIdx.x & 63, q = lane >> 3, p0 = 8 * (lane & 7);
    const int g = G.grp[8 * t + q];
    if (g < 0) return;
    const int2 md = G.meta[t];
    const float *emb = layer_w(blob, T, l).emb;
    float acc[8] = {};
    for (int i = 0; i < md.x; ++i) {
        const float *e = emb + msg_type[G.mem[md.y + 8 * i + q]] * H;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += e[pi_unit(p0 + k)];
    }
    float *o = memb + ((int64_t)l * Gtot + g) * H + p0;
    bf16x8 o16;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        o[k] = acc[k] / (float)md.x;
        o16[k] = (__bf16)o[k];
    }
    *reinterpret_cast<bf16x8 *>(memb16 + ((int64_t)l * Gtot + g) * H + p0) = o16;
}

// ------------------------------------------------------------------------ group means
struct GmArgs {
    const __bf16 *x_in;  // (B, E, 64) stored order; null at layer 0 (x = w_in llr + b_in)
    const float *llr;
    const int32_t *msg_var;
    const float *w_in, *b_in;
    const float *memb;   // this layer (Gv + Gc, 64) fp32
    GtArgs G;
    __bf16 *Mv, *Mc;
    const uint8_t *active;  // early termination: frames still decoding (null = all)
    // early termination after the first syndrome pass: the frames still decoding, ascending
    // (list[0 .. *count)); null = every frame of the range
    const int32_t *list, *count;
    int Gv, Gc, E, N;
    int64_t B;
};

__device__ __forceinline__ void gm_item(const GmArgs &A, uint32_t w, uint32_t nt);
__global__ __launch_bounds__(256) void gnn_bf16_gm_kernel(GmArgs A) {
    const uint32_t w0 = (uint32_t)(xcd_block(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6));
    const uint32_t nt = (uint32_t)(A.G.n_tiles - A.G.first);
    const uint32_t nact = A.count ? (uint32_t)__builtin_amdgcn_readfirstlane(*A.count) : (uint32_t)A.B;
    // a grid smaller than the work (listed layers with LDPC_GNN_GM_CAP): waves stride over it
    for (uint32_t w = w0; w < nact * nt; w += gridDim.x * 4) gm_item(A, w, nt);
}

__device__ __forceinline__ void gm_item(const GmArgs &A, uint32_t w, uint32_t nt) {
    const uint32_t slot = w / nt, t = w - slot * nt + (uint32_t)A.G.first;
    const uint32_t b = A.list ? (uint32_t)A.list[slot] : slot;
    if (A.active && !A.active[b]) return;
    const int lane = threadIdx.x & 63, q = lane >> 3, p0 = 8 * (lane & 7);
    const int2 md = A.G.meta[t];
    const int g = A.G.grp[8 * t + q];
    const int32_t *mem = A.G.mem + md.y + q;
    float acc[8] = {};
    if (A.x_in) {
        const __bf16 *xb = A.x_in + (int64_t)b * A.E * H + p0;
        int i = 0;
        for (; i + 4 <= md.x; i += 4) {
            const int m0 = mem[8 * i], m1 = mem[8 * i + 8], m2 = mem[8 * i + 16], m3 = mem[8 * i + 24];
            const bf16x8 v0 = *reinterpret_cast<const bf16x8 *>(xb + (int64_t)m0 * H);
            const bf16x8 v1 = *reinterpret_cast<const bf16x8 *>(xb + (int64_t)m1 * H);
            const bf16x8 v2 = *reinterpret_cast<const bf16x8 *>(xb + (int64_t)m2 * H);
            const bf16x8 v3 = *reinterpret_cast<const bf16x8 *>(xb + (int64_t)m3 * H);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += ((float)v0[k] + (float)v1[k]) + ((float)v2[k] + (float)v3[k]);
        }
        for (; i < md.x; ++i) {
            const bf16x8 v = *reinterpret_cast<const bf16x8 *>(xb + (int64_t)mem[8 * i] * H);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += (float)v[k];
        }
    } else {
        float ls = 0.0f;
        for (int i = 0; i < md.x; ++i) ls += A.llr[(int64_t)b * A.N + A.msg_var[mem[8 * i]]];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int u = pi_unit(p0 + k);
            acc[k] = fmaf(A.w_in[u], ls, (float)md.x * A.b_in[u]);
        }
    }
    if (g < 0) return;
    const float inv = 1.0f / (float)md.x;
    const float4 e0 = *reinterpret_cast<const float4 *>(A.memb + (int64_t)g * H + p0);
    const float4 e1 = *reinterpret_cast<const float4 *>(A.memb + (int64_t)g * H + p0 + 4);
    const float e[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (__bf16)fmaf(acc[k], inv, e[k]);
    __bf16 *dst = g < A.Gv ? A.Mv + ((int64_t)b * A.Gv + g) * H : A.Mc + ((int64_t)b * A.Gc + (g - A.Gv)) * H;
    *reinterpret_cast<bf16x8 *>(dst + p0) = o;
}

__device__ __forceinline__ bf16x8 ld8(const char *p) { return *reinterpret_cast<const bf16x8 *>(p); }
__device__ __forceinline__ f32x16 ld16(const float *p) {
    f32x16 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 f = reinterpret_cast<const float4 *>(p)[q];
        v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
    }
    return v;
}
// ReLU of 8 accumulators as bf16 (torch.relu semantics: a NaN stays NaN): v_maximum3_f32 with 0
// (IEEE maximum), then round.  The integer max on the bf16 bits this replaced (v_pk_max_i16, half the
// instructions) mapped a negative-signed NaN to 0; max on the bits viewed as f16 (v_pk_maximum3_f16)
// keeps -inf and quiets f16-signalling patterns (1407 of the 65536 bf16 patterns wrong,
// tools/ubench/relu_bf16.hip).
__device__ __forceinline__ bf16x8 relu8(const f32x16 &a, int half) {
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (__bf16)relu_nan(a[8 * half + i]);
    return o;
}
__device__ __forceinline__ bf16x8 pack8(const f32x16 &a, int half) {
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (__bf16)a[8 * half + i];
    return o;
}

// ------------------------------------------------------------------------ fused MLP
// LDS image (bytes): W1v, W1c bf16 [64 u][136] (128 stored columns + 8 pad: conflict-free
// ds_read_b128), W2v, W2c bf16 [64 o][72] (columns in GEMM1-accumulator order), then fp32:
// K [T + 2][132] (two sides x 64 + 4 pad, so that lanes reading different types' rows spread
// over the banks), b2 [64], wo [64].
constexpr int kW1B = 64 * 136 * 2, kW2B = 64 * 72 * 2;
constexpr int kOffW1v = 0, kOffW1c = kW1B, kOffW2v = 2 * kW1B, kOffW2c = 2 * kW1B + kW2B;
constexpr int kOffK = 2 * kW1B + 2 * kW2B;
constexpr int kKStride = 132;
// D1 rows: 68 floats apart (a row stride of 64 put every type's row on the same LDS banks: the
// 16-lane groups of a ds_read_b128 with lanes of different types serialised up to 16-way)
#ifndef LDPC_BF16_D1_STRIDE
#define LDPC_BF16_D1_STRIDE 68
#endif
constexpr int kD1Stride = LDPC_BF16_D1_STRIDE;
// then (MODE bit 2) one 4 KB staging tile per wave for the in-tile check sums
constexpr int kCTileB = 32 * 128;
__host__ __device__ inline size_t mlp_tables_bytes(int T, bool d1) {
    return (size_t)kOffK + ((size_t)(T + 2) * kKStride + 192 + (d1 ? (size_t)T * kD1Stride : 0)) * 4;
}
inline size_t mlp_lds_bytes(int T, bool d1) {
    return (mlp_tables_bytes(T, d1) + 15) / 16 * 16 + (size_t)(kMlpThreads / 64) * kCTileB;
}
// byte offset of (message row, byte b of its 128-B feature row) in a staging tile: 16-B chunks
// XOR-swizzled by the row so that the four ds_write_b128 of a tile and the eight
// ds_read_b64_tr_b16 that transpose it are all conflict-free (64-bank model of the LDS table in
// MI355X_MICROARCH.md)
__device__ __forceinline__ int ctile_off(int row, int b) {
    return row * 128 + 16 * ((b >> 4) ^ (((row & 3) << 1) | ((row >> 2) & 1))) + (b & 15);
}
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct MlpArgs {
    const __bf16 *x_in;  // null at layer 0
    __bf16 *x_out;       // null at the last layer
    const __bf16 *Mv, *Mc;               // group-mean rows (Mc: layer 0, or tiles not check-aligned)
    const int4 *info;                    // per tile slot (gnn_bf16_info_kernel)
    const int2 *slot;                    // per tile slot {message, check member mask}
    const float *inv_c;                  // 1 / |check group|
    const __bf16 *memb_c;                // this layer's mean type embedding per check group (Gc, 64), bf16
    const float *llr;
    const float *w1v, *w1c, *w2v, *w2c;  // this layer, nn.Linear layout, fp32
    const float *kd;                     // this layer's derived constants
    const float *bo;                     // output_projection bias (device)
    int T, Gv, Gc, E, N, tpf;            // tpf = message tiles per frame (gnn.hpp ct_m0)
    int d1;                              // degree-1 var groups use D1 (info.x < 0), layers >= 1
    int64_t B;
    float *msg_out;                      // last layer / early termination: (B, E) projected LLRs
    const uint8_t *active;               // early termination: frames still decoding (null = all)
    const int32_t *list, *count;         // early termination: the frames still decoding (see GmArgs)
    const float *kd_last, *bo_last;      // early termination: the last layer's output projection
};

// Per-tile inputs of one lane (message j of the tile, lane half h).
struct TileIn {
    bf16x8 xf[4], af[4], cf[4];
    bf16x8 mb[4];     // in-tile check means: the check group's mean type embedding, stored positions 16 s + 8 h + i
    float cinv;       // ... 1 / |check group|
    uint32_t cmask;   // ... the tile slots of the check group
    float l;
    int ty, var;
    bool one;  // degree-1 var group (D1 constant instead of K[ty][var side])
    int64_t row, b;
    bool ok, on;  // on: the frame is still decoding (early termination)
};
// Per-tile items fetched two tiles ahead: the slot's static info and the frame's id and flag
struct TileCtl {
    int4 inf;
    int2 sl;
    int64_t frame;
    bool on;
};
struct TilePos { int64_t t, b, k; };

// MODE bit 0: layer 0 (x from the LLRs, no GEMM1 over x, no residual); bit 1: last layer
// (output projection + per-variable sum instead of writing x); bit 2: check means in-tile (the
// tiles hold whole check groups: the check side's group mean is formed here from the tile's own
// feature rows, message_gnn_decoder.py:116-118, instead of read from a group-mean pass):
//   sum_c(m) = X S   as v_mfma_f32_32x32x16_bf16: A = the tile's feature rows transposed through
//                    a swizzled LDS tile by ds_read_b64_tr_b16 (rows permuted so that the
//                    accumulator holds exactly the stored positions GEMM1's B operand takes), B =
//                    S[k][j] = 1 when slots k and j share a check (bf16 1.0 / 0, exact)
//   g_c(m) = bf16(sum_c(m) / |group| + mean of the group's type embeddings)  (fp32 math, as the
//                    group-mean kernel: the same value up to the summation order of the sum)
// The next tile's rows are prefetched into registers one tile ahead, the small per-tile items two
// tiles ahead.
template <int MODE>
__global__ __launch_bounds__(kMlpThreads, 2) void gnn_bf16_mlp_kernel(MlpArgs A) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
    constexpr int NT = kMlpThreads;
    constexpr int oW1v = kOffW1v, oW1c = kOffW1c, oW2v = kOffW2v, oW2c = kOffW2c;
    constexpr int w1row = 272;  // bytes per W1 image row
    for (int i = tid; i < 64 * 128; i += NT) {
        const int u = i >> 7, p = i & 127;
        const int k = p < 64 ? pi_unit(p) : 64 + pi_unit(p - 64);
        reinterpret_cast<__bf16 *>(smem + kOffW1v)[u * 136 + p] = (__bf16)A.w1v[u * 128 + k];
        reinterpret_cast<__bf16 *>(smem + kOffW1c)[u * 136 + p] = (__bf16)A.w1c[u * 128 + k];
    }
    for (int i = tid; i < 64 * 64; i += NT) {
        const int o = i >> 6, q = i & 63;
        const int u = pi_unit(q);  // GEMM2's k index = GEMM1 accumulator registers (see header)
        reinterpret_cast<__bf16 *>(smem + oW2v)[o * 72 + q] = (__bf16)A.w2v[o * 64 + u];
        reinterpret_cast<__bf16 *>(smem + oW2c)[o * 72 + q] = (__bf16)A.w2c[o * 64 + u];
    }
    float *Ks = reinterpret_cast<float *>(smem + kOffK);
    const int nk = (A.T + 2) * 128;
    for (int i = tid; i < nk; i += NT) Ks[(i >> 7) * kKStride + (i & 127)] = A.kd[i];
    float *tail = Ks + (A.T + 2) * kKStride;  // b2 [64], wo [64]
    if (tid < 128) tail[tid] = A.kd[nk + tid];
    if (A.kd_last && tid < 64) tail[128 + tid] = A.kd_last[nk + 64 + tid];  // wo of the last layer
    float *D1s = tail + 192;  // D1 [T][kD1Stride]
    if (A.d1)
        for (int i = tid; i < A.T * 64; i += NT) D1s[(i >> 6) * kD1Stride + (i & 63)] = A.kd[nk + 128 + i];
    __syncthreads();

    const int lane = tid & 63, j = lane & 31, h = lane >> 5, wave = tid >> 6;
    constexpr bool layer0 = (MODE & 1) != 0, last = (MODE & 2) != 0, itc = (MODE & 4) != 0;
    // the output head's bias, read once (a load inside the tile loop would wait for the
    // prefetched rows before its store)
    const float bo_out = last ? A.bo[0] : A.kd_last ? A.bo_last[0] : 0.0f;
    char *ctile = smem + (mlp_tables_bytes(A.T, A.d1 != 0) + 15) / 16 * 16 + wave * kCTileB;
    // tiles of the frames still decoding: slot-major (slot s = the s-th listed frame)
    const int64_t nact = A.count ? (int64_t)__builtin_amdgcn_readfirstlane(*A.count) : A.B;
    const int64_t ntiles = nact * A.tpf;
    const TileWalk tw = xcd_tiles(ntiles, NT / 64, wave);
    // frame / in-frame tile counters, advanced without divisions
    const int64_t sb = tw.stride / A.tpf, sk = tw.stride - sb * A.tpf;
    const int64_t fb = tw.first / A.tpf, fk = tw.first - fb * A.tpf;
    auto next = [&](TilePos p) {
        p.t += tw.stride;
        p.b += sb;
        p.k += sk;
        if (p.k >= A.tpf) { p.k -= A.tpf; ++p.b; }
        return p;
    };

    // Everything below is branch-free per lane: a load in one arm of a branch whose other arm
    // writes the same registers makes the compiler wait for the load at the join, and then the
    // next tile's rows are no longer in flight while this tile computes.
    // Tile p's slot info, frame (list entry) and still-decoding flag, fetched two tiles ahead.
    auto ctl_of = [&](const TilePos &p) {
        TileCtl c;
        c.inf = A.info[p.k * 32 + j];
        c.sl = A.slot[p.k * 32 + j];
        const int64_t slot = p.t < tw.end ? p.b : fb;  // past the end: any valid frame
        const int32_t *lp = A.list ? A.list + slot : reinterpret_cast<const int32_t *>(A.slot);
        const int64_t lv = *lp;
        c.frame = A.list ? lv : slot;
        const bool chk = A.active && !A.list;  // listed frames are active by construction
        const uint8_t *ap = chk ? A.active + c.frame : reinterpret_cast<const uint8_t *>(A.slot);
        const uint8_t av = *ap;
        c.on = !chk || av != 0;
        return c;
    };
    auto load = [&](const TileCtl &c, const TilePos &p) {
        TileIn I;
        const int4 inf = c.inf;
        I.ok = c.sl.x >= 0 && p.t < tw.end;
        const int m = c.sl.x >= 0 ? c.sl.x : ~c.sl.x;
        const int64_t bb = c.frame;
        I.ty = inf.z;
        I.var = inf.w;
        I.one = !layer0 && A.d1 && inf.x < 0;
        I.row = bb * A.E + m;
        I.b = bb;
        I.on = c.on;
        // A terminated frame (uniform over the tile) loads frame 0's rows instead of its own:
        // L2 hits, and no branch around the loads.
        const int64_t lb = I.on ? bb : 0;
        const int vg = inf.x < 0 ? ~inf.x : inf.x;
        const char *mv = reinterpret_cast<const char *>(A.Mv + (lb * A.Gv + vg) * H) + 16 * h;
        if constexpr (!layer0) {
            const char *xr = reinterpret_cast<const char *>(A.x_in + (lb * A.E + m) * H) + 16 * h;
            // a degree-1 var group's g is x itself (its emb part is in D1): the same rows again
            const char *ma = I.one ? xr : mv;
#pragma unroll
            for (int s = 0; s < 4; ++s) I.xf[s] = ld8(xr + 32 * s);
#pragma unroll
            for (int s = 0; s < 4; ++s) I.af[s] = ld8(ma + 32 * s);
            I.l = 0.0f;
        } else {
            I.l = A.llr[lb * A.N + I.var];
#pragma unroll
            for (int s = 0; s < 4; ++s) I.af[s] = ld8(mv + 32 * s);
        }
        if constexpr (itc) {
            I.cmask = (uint32_t)c.sl.y;
            I.cinv = A.inv_c[inf.y];
            const char *mbr = reinterpret_cast<const char *>(A.memb_c + (int64_t)inf.y * H) + 16 * h;
#pragma unroll
            for (int s = 0; s < 4; ++s) I.mb[s] = ld8(mbr + 32 * s);
        } else {
            const char *mc = reinterpret_cast<const char *>(A.Mc + (lb * A.Gc + inf.y) * H) + 16 * h;
#pragma unroll
            for (int s = 0; s < 4; ++s) I.cf[s] = ld8(mc + 32 * s);
        }
        return I;
    };

    // In-tile check means (MODE bit 2): g_c of this lane's message from the tile's feature rows
    auto check_means = [&](TileIn &I) {
#pragma unroll
        for (int s = 0; s < 4; ++s) *reinterpret_cast<bf16x8 *>(ctile + ctile_off(j, 32 * s + 16 * h)) = I.xf[s];
        __builtin_amdgcn_wave_barrier();
        // A fragment (row tile rt, k-step ks): lane (r, h) <- stored position sigma(32 rt + r) of
        // slots 16 ks + 8 h + 0..7 (sigma swaps bits 2 and 3 of r: the accumulator's register
        // 8 (s & 1) + i of tile s >> 1 then holds stored position 16 s + 8 h + i).  One
        // ds_read_b64_tr_b16 per four slots: group lane 4q + p addresses slot row q, 4 stored
        // positions; lane i of the 16-lane group receives column i (MI355X: T10).
        const int g16 = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3, hh = g16 >> 1;
        const int col0 = 16 * (g16 & 1) + 4 * (2 * (p & 1) + (p >> 1));
        f32x16 sum[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) sum[rt] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            // B = S: element e of lane (j, h) is slot 16 ks + 8 h + e in j's check (bf16 1.0 / 0)
            const uint32_t bits = (I.cmask >> (16 * ks + 8 * h)) & 0xFFu;
            uint32_t sw[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
                const uint32_t t = (bits >> (2 * e2)) & 3u;
                sw[e2] = ((t | (t << 15)) & 0x10001u) * 0x3F80u;
            }
            const bf16x8 sop = __builtin_bit_cast(bf16x8, (uint32_t __attribute__((ext_vector_type(4)))){sw[0], sw[1], sw[2], sw[3]});
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                const int col = 32 * rt + col0, row = 16 * ks + 8 * hh + q;
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4 *)(ctile + ctile_off(row, 2 * col)));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4 *)(ctile + ctile_off(row + 4, 2 * col)));
                const s16x4 a8[2] = {lo, hi};
                const bf16x8 afr = __builtin_bit_cast(bf16x8, a8);
                sum[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afr, sop, sum[rt], 0, 0, 0);
            }
        }
        __builtin_amdgcn_wave_barrier();  // the next tile's staging writes wait for these reads
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            bf16x8 o;
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = (__bf16)fmaf(sum[s >> 1][8 * (s & 1) + i], I.cinv, (float)I.mb[s][i]);
            I.cf[s] = o;
        }
    };

    auto compute = [&](TileIn &I) {
        if (!I.on) return;
        if constexpr (itc) check_means(I);
        const float *Kt = Ks + I.ty * kKStride;
        f32x16 y0 = ld16(tail + 16 * h), y1 = ld16(tail + 32 + 16 * h);  // b2v + b2c
        int wbase = j * w1row + 16 * h, w2base = j * 144 + 16 * h;
        asm volatile("" : "+v"(wbase), "+v"(w2base));
        // GEMM1 of one side into (h0, h1), then ReLU + GEMM2 into y
        auto gemm1 = [&](int side, f32x16 &h0, f32x16 &h1) {
            const char *W1 = smem + (side == 0 ? oW1v : oW1c);
            const float *K0 = side == 0 && I.one ? D1s + I.ty * kD1Stride : Kt + side * 64;
            h0 = ld16(K0 + 16 * h);
            h1 = ld16(K0 + 32 + 16 * h);
            if constexpr (layer0) {  // + llr * (W1 w_in) + W1 b_in
                const float *U = Ks + A.T * kKStride + side * 64 + 16 * h, *V = U + kKStride;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    h0[r] += fmaf(I.l, U[r], V[r]);
                    h1[r] += fmaf(I.l, U[32 + r], V[32 + r]);
                }
            } else {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    h0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld8(W1 + wbase + 32 * s), I.xf[s], h0, 0, 0, 0);
                    h1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld8(W1 + 32 * w1row + wbase + 32 * s), I.xf[s], h1, 0, 0, 0);
                }
            }
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const bf16x8 g = side == 0 ? I.af[s] : I.cf[s];
                h0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld8(W1 + wbase + 32 * (4 + s)), g, h0, 0, 0, 0);
                h1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld8(W1 + 32 * 272 + wbase + 32 * (4 + s)), g, h1, 0, 0, 0);
            }
        };
        auto gemm2 = [&](int side, const f32x16 &h0, const f32x16 &h1) {
            const char *W2 = smem + (side == 0 ? oW2v : oW2c);
            const bf16x8 p00 = relu8(h0, 0), p01 = relu8(h0, 1), p10 = relu8(h1, 0), p11 = relu8(h1, 1);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bf16x8 bop = q == 0 ? p00 : q == 1 ? p01 : q == 2 ? p10 : p11;
                const int qb = w2base + 32 * q;
                y0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld8(W2 + qb), bop, y0, 0, 0, 0);
                y1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld8(W2 + 32 * 144 + qb), bop, y1, 0, 0, 0);
            }
        };
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            f32x16 h0, h1;
            gemm1(side, h0, h1);
            gemm2(side, h0, h1);
        }
        if constexpr (!layer0) {  // residual (message_gnn_decoder.py:261): chunk s <-> y_{s>>1}[8 (s&1) ..]
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                y0[i] += (float)I.xf[0][i];
                y0[8 + i] += (float)I.xf[1][i];
                y1[i] += (float)I.xf[2][i];
                y1[8 + i] += (float)I.xf[3][i];
            }
        }
        if constexpr (last) {
            const float *wo = tail + 64;
            float part = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                part = fmaf(y0[r], wo[16 * h + r], part);
                part = fmaf(y1[r], wo[32 + 16 * h + r], part);
            }
            part += __shfl_xor(part, 32, 64);
            if (I.ok && h == 0) A.msg_out[I.row] = part + bo_out;
        } else {
            if (A.kd_last) {  // early termination: project with the last layer's output head
                const float *wo = tail + 128;
                float part = 0.0f;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    part = fmaf(y0[r], wo[16 * h + r], part);
                    part = fmaf(y1[r], wo[32 + 16 * h + r], part);
                }
                part += __shfl_xor(part, 32, 64);
                if (I.ok && h == 0) A.msg_out[I.row] = part + bo_out;
            }
            if (!I.ok) return;
            char *xo = reinterpret_cast<char *>(A.x_out + I.row * H) + 16 * h;
            *reinterpret_cast<bf16x8 *>(xo) = pack8(y0, 0);
            *reinterpret_cast<bf16x8 *>(xo + 32) = pack8(y0, 1);
            *reinterpret_cast<bf16x8 *>(xo + 64) = pack8(y1, 0);
            *reinterpret_cast<bf16x8 *>(xo + 96) = pack8(y1, 1);
        }
    };

    if (tw.first >= tw.end) return;
    // rows one tile ahead, the per-tile items two tiles ahead; unrolled by two so that the tile
    // in flight lives in its own registers (no copies that would wait for its loads)
    TilePos p0{tw.first, fb, fk};
    TilePos p1 = next(p0);
    TileIn ta = load(ctl_of(p0), p0), tb;
    TileCtl c1 = ctl_of(p1);
    for (;;) {
        const TilePos p2 = next(p1);
        const TileCtl c2 = ctl_of(p2);
        tb = load(c1, p1);
        compute(ta);
        if (p1.t >= tw.end) break;
        const TilePos p3 = next(p2);
        c1 = ctl_of(p3);
        ta = load(c2, p2);
        compute(tb);
        if (p2.t >= tw.end) break;
        p1 = p3;
    }
}

// Early termination (cfg5; no reference counterpart).  One workgroup per frame still decoding,
// after layer `layer` < L - 1: bit_v = [llr_v + sum_{m -> v} (wo_L . x_m + bo_L) > 0] (the
// decoder's P(bit = 1) > 0.5, message_gnn_decoder.py:298-307, with the last layer's head as the
// output stage, :270); if every check group has even parity the frame is done: its probs are
// written now, its layer count recorded, and every later kernel skips it.  A frame that goes on is
// appended to out_list (one atomic per frame): the next layer's kernels walk that list, so no
// separate compaction pass is needed (the list order varies run to run; no result depends on it).
// ZS: the variable sums are kept in LDS for the probs of a finished frame ((N + 31) / 32 + N words;
// syndrome_lds_bytes); without ZS (codes whose N does not fit) they are summed again, in the same
// order, only for a finished frame.
template <bool ZS>
__global__ __launch_bounds__(256) void gnn_bf16_syndrome_kernel(const float *__restrict__ msg_out,
                                                                const int32_t *__restrict__ csr, int64_t E,
                                                                const float *__restrict__ llr, int N,
                                                                const int32_t *__restrict__ cg_ptr,
                                                                const int32_t *__restrict__ cg_var, int Gc, int layer,
                                                                uint8_t *__restrict__ active,
                                                                const int32_t *__restrict__ list,
                                                                const int32_t *__restrict__ count,
                                                                int32_t *__restrict__ iters, float *__restrict__ probs,
                                                                int32_t *__restrict__ out_list,
                                                                int32_t *__restrict__ out_count) {
    extern __shared__ uint32_t bits[];  // [(N + 31) / 32] decision bits, then (ZS) zs [N]
    float *zs = reinterpret_cast<float *>(bits + (N + 31) / 32);
    const int32_t *vptr = csr_ptr(csr), *vmem = csr_mem(csr, N);
    auto zsum = [&](const float *mo, const float *lr, int v) {
        float sum = 0.0f;  // the output stage's own sum order (gnn_output)
        for (int q = vptr[v]; q < vptr[v + 1]; ++q) sum += mo[vmem[q]];
        return sum + lr[v];
    };
    __shared__ int odd;
    if (count && (int)blockIdx.x >= *count) return;
    const int64_t b = list ? list[blockIdx.x] : blockIdx.x;
    if (!active[b]) return;
    const float *mo = msg_out + b * E, *lr = llr + b * N;
    for (int i = threadIdx.x; i < (N + 31) / 32; i += blockDim.x) bits[i] = 0u;
    if (threadIdx.x == 0) odd = 0;
    __syncthreads();
    for (int v = threadIdx.x; v < N; v += blockDim.x) {
        const float zv = zsum(mo, lr, v);
        if constexpr (ZS) zs[v] = zv;
        if (zv > 0.0f) atomicOr(&bits[v >> 5], 1u << (v & 31));
        if ((__float_as_uint(zv) & 0x7f800000u) == 0x7f800000u) odd = 1;  // inf / NaN: never a decision;
        // the frame runs on to gnn_output, which makes all of it NaN (the reference's dense bmm)
    }
    __syncthreads();
    for (int g = threadIdx.x; g < Gc; g += blockDim.x) {
        uint32_t p = 0;
        for (int q = cg_ptr[g]; q < cg_ptr[g + 1]; ++q) {  // cg_var[q] = the variable of member q
            const int v = cg_var[q];
            p ^= bits[v >> 5] >> (v & 31);
        }
        if (p & 1u) odd = 1;
    }
    __syncthreads();
    if (odd) {  // still decoding: onto the next layer's list (any order: frames are independent)
        if (out_list && threadIdx.x == 0) out_list[atomicAdd(out_count, 1)] = (int32_t)b;
        return;
    }
    if (threadIdx.x == 0) {
        active[b] = 0;
        if (iters) iters[b] = layer + 1;
    }
    for (int v = threadIdx.x; v < N; v += blockDim.x)
        probs[b * N + v] = 1.0f / (1.0f + expf(-(ZS ? zs[v] : zsum(mo, lr, v))));
}

// dynamic LDS of gnn_bf16_syndrome_kernel<ZS>
inline size_t syndrome_lds_bytes(int N, bool zs) { return (size_t)((N + 31) / 32 + (zs ? N : 0)) * 4; }
constexpr size_t kSyndromeLdsMax = 64 * 1024;  // the z cache only while several workgroups fit a CU

// cg_var[q] = msg_var[cg_mem[q]]: the variable of every check-group member (syndrome tables)
__global__ void gnn_bf16_cgvar_kernel(const int32_t *__restrict__ cg_mem, const int32_t *__restrict__ msg_var,
                                      int64_t n, int32_t *__restrict__ cg_var) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n) cg_var[q] = msg_var[cg_mem[q]];
}

__global__ void fill_i32_kernel(int32_t *p, int64_t n, int32_t v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

struct Bf16Ws {
    float *kd, *memb, *msg_out;
    __bf16 *memb16;
    int32_t *csr, *alist, *acount, *cg_var;
    int4 *info;
    int2 *slot;
    uint8_t *active;
    __bf16 *xa, *xb, *Mv, *Mc;
    int64_t bytes;
};

Bf16Ws carve_bf16(const ldpc_gnn_plan *p, int N, int64_t B, int T, int L, void *base) {
    auto al = [](int64_t x) { return (x + 255) / 256 * 256; };
    const int64_t kd = al(L * kd_floats(T) * 4), memb = al((int64_t)L * (p->Gv + p->Gc) * H * 4) * 3 / 2;
    const int64_t xa = L > 1 ? al(B * p->E * H * 2) : 0, xb = L > 2 ? xa : 0;
    const int64_t mv = al(B * p->Gv * H * 2), mc = al(B * p->Gc * H * 2), vs = al(B * p->E * 4);
    const int64_t nslot = (int64_t)p->n_ctiles * 32;
    const int64_t inf = al(nslot * 16) + al(nslot * 8), act = al(B), cs = al(gnn_csr_ints(p->E, N) * 4);
    const int64_t alb = al(2 * B * 4) + 256;  // two active lists [B] + the two ranges' two counts
    char *c = static_cast<char *>(base);
    Bf16Ws w;
    w.info = reinterpret_cast<int4 *>(c + kd + memb + xa + xb + mv + mc + vs);
    w.slot = reinterpret_cast<int2 *>(c + kd + memb + xa + xb + mv + mc + vs + al(nslot * 16));
    w.active = reinterpret_cast<uint8_t *>(c + kd + memb + xa + xb + mv + mc + vs + inf);
    w.csr = reinterpret_cast<int32_t *>(c + kd + memb + xa + xb + mv + mc + vs + inf + act);
    w.kd = reinterpret_cast<float *>(c);
    w.memb = reinterpret_cast<float *>(c + kd);
    w.memb16 = reinterpret_cast<__bf16 *>(c + kd + al((int64_t)L * (p->Gv + p->Gc) * H * 4));
    w.xa = reinterpret_cast<__bf16 *>(c + kd + memb);
    w.xb = reinterpret_cast<__bf16 *>(c + kd + memb + xa);
    w.Mv = reinterpret_cast<__bf16 *>(c + kd + memb + xa + xb);
    w.Mc = reinterpret_cast<__bf16 *>(c + kd + memb + xa + xb + mv);
    w.msg_out = reinterpret_cast<float *>(c + kd + memb + xa + xb + mv + mc);
    w.alist = reinterpret_cast<int32_t *>(c + kd + memb + xa + xb + mv + mc + vs + inf + act + cs);
    w.acount = reinterpret_cast<int32_t *>(c + kd + memb + xa + xb + mv + mc + vs + inf + act + cs + al(2 * B * 4));
    w.cg_var = reinterpret_cast<int32_t *>(c + kd + memb + xa + xb + mv + mc + vs + inf + act + cs + alb);
    w.bytes = kd + memb + xa + xb + mv + mc + vs + inf + act + cs + alb + al(p->E * 4);
    return w;
}

int g_cus = 0;

template <int MODE>
int launch_mlp_t(int64_t tiles, size_t lds, hipStream_t s, const MlpArgs &m) {
    const void *fn = reinterpret_cast<const void *>(gnn_bf16_mlp_kernel<MODE>);
    LDPC_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int per_cu = 4 * 2 / (kMlpThreads / 64);  // workgroups per CU at 2 waves per SIMD
    const unsigned grid = (unsigned)std::min<int64_t>((tiles + kMlpThreads / 64 - 1) / (kMlpThreads / 64),
                                                      (int64_t)g_cus * per_cu);
    hipLaunchKernelGGL((gnn_bf16_mlp_kernel<MODE>), dim3(grid), dim3(kMlpThreads), lds, s, m);
    return LDPC_OK;
}

// the MLP kernel per layer mode (bit 0 layer 0, bit 1 last layer, bit 2 in-tile check means): one
// 512-thread workgroup per CU, 2 waves per SIMD, next tile prefetched into registers (measured
// against 3-4 waves per SIMD and deeper prefetch: all within 2 % or slower)
int launch_mlp(int mode, int64_t tiles, size_t lds, hipStream_t s, const MlpArgs &m) {
    switch (mode) {
        case 0: return launch_mlp_t<0>(tiles, lds, s, m);
        case 1: return launch_mlp_t<1>(tiles, lds, s, m);
        case 2: return launch_mlp_t<2>(tiles, lds, s, m);
        case 3: return launch_mlp_t<3>(tiles, lds, s, m);
        case 4: return launch_mlp_t<4>(tiles, lds, s, m);
        case 6: return launch_mlp_t<6>(tiles, lds, s, m);
        default: return fail(LDPC_EINVAL, "bad MLP mode");
    }
}

// LDPC_GNN_STREAMS=1: one frame range on the caller's stream; default two halves on two streams
// (gnn.hip), so one half's group means and syndrome checks overlap the other half's MLP.
int gnn_streams_bf16() {
    static int t = [] {
        const char *e = std::getenv("LDPC_GNN_STREAMS");
        return (e && std::atoi(e) == 1) ? 1 : 2;
    }();
    return t;
}

// LDPC_GNN_ET_COMPACT=0: after a syndrome pass the kernels still walk every frame and skip the
// finished ones (A/B); default: they walk the list of frames still decoding that the pass appended
int compact_env() {
    const char *e = std::getenv("LDPC_GNN_ET_COMPACT");  // read per call (tests toggle it)
    return e ? std::atoi(e) : 1;
}

// LDPC_GNN_GM_CAP=n: after the first syndrome pass the group-mean kernel runs at most n workgroups
// per CU, striding over the frames still decoding, instead of one wave per (frame, tile) of the
// whole range (whose early-exiting waves cost ~0.1 ms per layer once few frames are left).  Default
// 256 (+2.3 % on cfg5 random codewords; 64: -1.2 %; profiles/r03ah); 0 = the full grid.  Read per call.
int gm_cap() {
    const char *e = std::getenv("LDPC_GNN_GM_CAP");
    return e ? std::atoi(e) : 256;
}

}  // namespace

int64_t gnn_bf16_workspace(const ldpc_gnn_plan *p, int N, int64_t B, int layers) {
    return carve_bf16(p, N, B, kBf16MaxTypes, layers, nullptr).bytes;
}

int gnn_bf16_forward(const ldpc_gnn_plan *p, int T, int L, const float *d_weights, const int32_t *d_msg_type,
                     const int32_t *d_msg_var, const float *d_llr, int N, int64_t B, int flags, float *d_probs,
                     int32_t *d_iters, void *d_work, int64_t work_bytes, hipStream_t s) {
    const bool et = (flags & LDPC_GNN_EARLY_STOP) && L > 1;
    if (!p->n_gtiles) return fail(LDPC_EUNSUPPORTED, "plan has no group tiles");
    Bf16Ws w = carve_bf16(p, N, B, T, L, d_work);
    if (!d_work || work_bytes < w.bytes)
        return fail(LDPC_EINVAL, "workspace too small: need " + std::to_string(w.bytes) + " bytes");
    const int64_t tpf = p->n_ctiles;  // message tiles per frame (gnn.hpp ct_m0)
    if (tpf <= 0) return fail(LDPC_EUNSUPPORTED, "plan has no message tiles");
    if (B * tpf >= (1LL << 31) || B * p->n_gtiles >= (1LL << 31) || p->E >= (1LL << 31))
        return fail(LDPC_EUNSUPPORTED, "batch too large for one launch (chunk it)");
    // degree-1 skip when its D1 table still fits the LDS image
    const bool d1 = p->n_gtiles_v1 > 0 && mlp_lds_bytes(T, true) <= 160 * 1024;
    const size_t lds = mlp_lds_bytes(T, d1);
    if (T > kBf16MaxTypes || lds > 160 * 1024)
        return fail(LDPC_EUNSUPPORTED, "too many message types for the bf16 LDS image");
    if (!g_cus) {
        int dev = 0;
        LDPC_HIP(hipGetDevice(&dev));
        LDPC_HIP(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const GtArgs G{p->gt_meta, p->gt_grp, p->gt_mem, p->n_gtiles, 0};
    const int Gtot = p->Gv + p->Gc;
    {
        const int nslot = (int)(tpf * 32);
        hipLaunchKernelGGL(gnn_bf16_info_kernel, dim3((unsigned)((nslot + 255) / 256)), dim3(256), 0, s, nslot,
                           p->ct_m0, p->ct_aligned ? 1 : 0, p->vgroup, p->vg_ptr, d1 ? 1 : 0, p->cgroup, p->cg_ptr,
                           p->cg_mem, d_msg_type, d_msg_var, w.info, w.slot);
        LDPC_CHECK_LAUNCH("gnn_bf16_info_kernel");
    }
    hipLaunchKernelGGL(gnn_bf16_kconst_kernel, dim3(L, T + 2), dim3(128), 0, s, d_weights, T, w.kd);
    LDPC_CHECK_LAUNCH("gnn_bf16_kconst_kernel");
    hipLaunchKernelGGL(gnn_bf16_memb_kernel, dim3((unsigned)(((int64_t)L * p->n_gtiles + 3) / 4)), dim3(256), 0, s,
                       d_weights, T, L, d_msg_type, G, Gtot, w.memb, w.memb16);
    LDPC_CHECK_LAUNCH("gnn_bf16_memb_kernel");
    if (int rc = gnn_build_var_csr(d_msg_var, p->E, N, w.csr, s)) return rc;
    if (d_iters) {
        hipLaunchKernelGGL(fill_i32_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, d_iters, B, L);
        LDPC_CHECK_LAUNCH("fill_i32_kernel");
    }
    if (et) {
        LDPC_HIP(hipMemsetAsync(w.active, 1, (size_t)B, s));
        hipLaunchKernelGGL(gnn_bf16_cgvar_kernel, dim3((unsigned)((p->E + 255) / 256)), dim3(256), 0, s, p->cg_mem,
                           d_msg_var, p->E, w.cg_var);
        LDPC_CHECK_LAUNCH("gnn_bf16_cgvar_kernel");
    }
    const uint8_t *active = et ? w.active : nullptr;
    const float *kd_last = w.kd + (int64_t)(L - 1) * kd_floats(T);
    const float *bo_last = layer_w(d_weights, T, L - 1).bo;

    // frames [b0, b0 + nb) through every layer on stream st (pointers offset to the range)
    auto run_range = [&](int64_t b0, int64_t nb, hipStream_t st, int slot) -> int {
    const int64_t xoff = b0 * p->E * H;
    uint8_t *act = et ? w.active + b0 : nullptr;
    // active lists: the syndrome pass after layer l appends the frames still decoding to one list
    // while the layer walked the other (double-buffered, counts zeroed before each pass)
    int32_t *lists[2] = {w.alist + b0, w.alist + B + b0}, *counts[2] = {w.acount + 2 * slot, w.acount + 2 * slot + 1};
    int cur = 0;
    int32_t *alist = lists[0], *acount = counts[0];
    bool listed = false;  // after the first syndrome pass the kernels walk the active list
    const __bf16 *x_in = nullptr;
    for (int l = 0; l < L; ++l) {
        const LayerW lw = layer_w(d_weights, T, l);
        // layers >= 1 on check-aligned tiles: the MLP forms the check means itself, the group-mean
        // pass does the var groups alone (layer 0's means come from the LLRs: both sides here)
        const bool itc = p->ct_aligned && l > 0;
        GmArgs gm{};
        gm.x_in = x_in;
        gm.llr = d_llr + b0 * N;
        gm.msg_var = d_msg_var;
        gm.w_in = d_weights;
        gm.b_in = d_weights + H;
        gm.memb = w.memb + (int64_t)l * Gtot * H;
        gm.G = G;
        if (d1 && l > 0) gm.G.first = p->n_gtiles_v1;
        if (itc) gm.G.n_tiles = p->n_gtiles_v;
        gm.Mv = w.Mv + b0 * p->Gv * H;
        gm.Mc = w.Mc + b0 * p->Gc * H;
        gm.Gv = p->Gv;
        gm.Gc = p->Gc;
        gm.E = (int)p->E;
        gm.N = N;
        gm.B = nb;
        gm.active = act;
        gm.list = listed ? alist : nullptr;
        gm.count = listed ? acount : nullptr;
        if (gm.G.n_tiles > gm.G.first) {
            const int64_t gwaves = nb * (gm.G.n_tiles - gm.G.first);
            int64_t gblocks = (gwaves + 3) / 4;
            if (gm.count && gm_cap() > 0) gblocks = std::min<int64_t>(gblocks, (int64_t)g_cus * gm_cap());
            hipLaunchKernelGGL(gnn_bf16_gm_kernel, dim3((unsigned)gblocks), dim3(256), 0, st, gm);
            LDPC_CHECK_LAUNCH("gnn_bf16_gm_kernel");
        }

        MlpArgs m{};
        m.x_in = x_in;
        m.x_out = l == L - 1 ? nullptr : (l % 2 == 0 ? w.xa : w.xb) + xoff;
        m.Mv = w.Mv + b0 * p->Gv * H;
        m.Mc = w.Mc + b0 * p->Gc * H;
        m.info = w.info;
        m.slot = w.slot;
        m.inv_c = p->inv_c;
        m.memb_c = w.memb16 + ((int64_t)l * Gtot + p->Gv) * H;
        m.llr = d_llr + b0 * N;
        m.w1v = lw.w1v;
        m.w1c = lw.w1c;
        m.w2v = lw.w2v;
        m.w2c = lw.w2c;
        m.kd = w.kd + (int64_t)l * kd_floats(T);
        m.bo = lw.bo;
        m.T = T;
        m.Gv = p->Gv;
        m.Gc = p->Gc;
        m.E = (int)p->E;
        m.N = N;
        m.tpf = (int)tpf;
        m.d1 = d1 ? 1 : 0;
        m.B = nb;
        m.msg_out = w.msg_out + b0 * p->E;
        m.active = act;
        m.list = listed ? alist : nullptr;
        m.count = listed ? acount : nullptr;
        m.kd_last = et && l < L - 1 ? kd_last : nullptr;
        m.bo_last = bo_last;
        const int mode = (l == 0 ? 1 : 0) | (l == L - 1 ? 2 : 0) | (itc ? 4 : 0);
        const int rc = launch_mlp(mode, nb * tpf, lds, st, m);
        if (rc != LDPC_OK) return rc;
        LDPC_CHECK_LAUNCH("gnn_bf16_mlp_kernel");
        if (m.kd_last) {
            const bool cmp = compact_env();
            int32_t *olist = lists[cur ^ 1], *ocount = counts[cur ^ 1];
            if (cmp) LDPC_HIP(hipMemsetAsync(ocount, 0, 4, st));
            const bool zs = syndrome_lds_bytes(N, true) <= kSyndromeLdsMax;
            const size_t slds = syndrome_lds_bytes(N, zs);
            if (slds > 160 * 1024) return fail(LDPC_EUNSUPPORTED, "early termination: N too large for the syndrome pass");
            auto synd = zs ? gnn_bf16_syndrome_kernel<true> : gnn_bf16_syndrome_kernel<false>;
            if (slds > kSyndromeLdsMax)
                LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(synd),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)slds));
            hipLaunchKernelGGL(synd, dim3((unsigned)nb), dim3(256), slds, st, w.msg_out + b0 * p->E, w.csr, p->E,
                               d_llr + b0 * N, N, p->cg_ptr, w.cg_var, p->Gc, l, act, listed ? alist : nullptr, listed ? acount : nullptr,
                               d_iters ? d_iters + b0 : nullptr, d_probs + b0 * N, cmp ? olist : nullptr, ocount);
            LDPC_CHECK_LAUNCH("gnn_bf16_syndrome_kernel");
            if (cmp) {
                cur ^= 1;
                alist = olist;
                acount = ocount;
                listed = true;
            }
        }
        x_in = m.x_out;
    }
    return LDPC_OK;
    };
    if (gnn_streams_bf16() == 2 && B >= 2 * 64) {
        hipStream_t s2;
        hipEvent_t fork, join;
        if (int rc = gnn_side_stream(&s2, &fork, &join)) return rc;
        const int64_t b1 = B / 2;
        LDPC_HIP(hipEventRecord(fork, s));
        LDPC_HIP(hipStreamWaitEvent(s2, fork, 0));
        if (int rc = run_range(0, b1, s, 0)) return rc;
        if (int rc = run_range(b1, B - b1, s2, 1)) return rc;
        LDPC_HIP(hipEventRecord(join, s2));
        LDPC_HIP(hipStreamWaitEvent(s, join, 0));
    } else if (int rc = run_range(0, B, s, 0)) {
        return rc;
    }
    return gnn_output(w.msg_out, w.csr, d_llr, p->E, N, B, active, d_probs, s);
}

}  // namespace ldpc
