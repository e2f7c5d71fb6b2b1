// gnn.hpp -- message-GNN plan shared by the fp32 path (gnn.hip) and the bf16 path (gnn_bf16.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

struct ldpc_gnn_plan {
    int device = 0;
    int64_t E = 0;
    int Gv = 0, Gc = 0;
    int32_t *d_tab = nullptr;  // vgroup[E] cgroup[E] vg_ptr[Gv+1] vg_mem[E] cg_ptr[Gc+1] cg_mem[E]
    float *d_inv = nullptr;    // 1/|group|: inv_v[Gv] inv_c[Gc]
    const int32_t *vgroup, *cgroup, *vg_ptr, *vg_mem, *cg_ptr, *cg_mem;
    const float *inv_v, *inv_c;
    // weighted plan (ldpc_gnn_plan_create_csr): aggregation row m of each side is row m of a
    // general (E x E) adjacency in CSR form, vg_w / cg_w hold the member weights (inv = 1, every
    // message reads its own row).  Group plans leave these NULL.
    bool weighted = false;
    float *d_w = nullptr;
    const float *vg_w = nullptr, *cg_w = nullptr;
    // ... and the transposes (training backward: dc += A^T d(aggregated)), column j's nonzero rows
    // ascending with their weights: vt_ptr[E+1] vt_mem vt_w, ct_ptr[E+1] ct_mem ct_w
    int32_t *d_tt = nullptr;
    float *d_tw = nullptr;
    const int32_t *vt_ptr = nullptr, *vt_mem = nullptr, *ct_ptr = nullptr, *ct_mem = nullptr;
    const float *vt_w = nullptr, *ct_w = nullptr;
    // bf16 path: "group tiles" of 8 groups of one degree each (var groups first, then check
    // groups, each side sorted by degree), so one wave sums 8 groups with no divergence.
    //   gt_meta[t] = {degree, offset into gt_mem}, gt_grp[8 t + q] = group id (check groups
    //   offset by Gv; -1 = padding), gt_mem[off + 8 i + q] = i-th member message of group q.
    int n_gtiles = 0;
    int n_gtiles_v1 = 0;  // the leading tiles whose groups are var groups of degree 1
    int n_gtiles_v = 0;   // the var side's tiles (the check side's follow)
    int32_t *d_gt = nullptr;
    const int2 *gt_meta = nullptr;
    const int32_t *gt_grp = nullptr, *gt_mem = nullptr;
    // fp32 projection tiles (gnn.hip, gnn_group_proj_kernel): 32 groups of one side per tile,
    // each side sorted by degree.  pt_meta[t] = {side (0 var, 1 check), max degree, offset into
    // pt_mem, 0}; pt_grp[32 t + j] = group id within its side (-1 = padding), pt_deg[32 t + j]
    // its degree (0 for padding); pt_mem[off + 32 i + j] = i-th member message of lane j's group
    // (message 0 past its degree; max degree + 1 rows per tile).
    int n_ptiles = 0;
    int n_ptiles_v = 0;   // the leading tiles are the var side's
    int n_ptiles_v1 = 0;  // the leading var tiles whose groups all have degree 1
    int32_t *d_pt = nullptr;
    const int4 *pt_meta = nullptr;
    const int32_t *pt_grp = nullptr, *pt_deg = nullptr, *pt_mem = nullptr;
    // bf16 projected MLP (gnn_bf16.hip): message order of its 32-message tiles -- the messages of
    // degree-1 var groups first (ascending), then the rest (ascending), each part padded to whole
    // tiles with -1, so every tile is either all degree-1 or has none.  mt_perm[32 n_mtiles].
    int n_mtiles = 0, n_mtiles_v1 = 0;
    const int32_t *mt_perm = nullptr;
    // bf16 MLP message tiles (gnn_bf16.hip): tile k of a frame holds messages ct_m0[k] .. ct_m0[k+1]
    // - 1 (at most 32).  When every check group is a contiguous run of at most 32 messages (the
    // reference's check-major edge order, message_gnn_decoder.py:397-406), the tiles hold whole
    // check groups (ct_aligned) and the MLP forms the check means from its own tile; otherwise
    // they are the plain 32-message tiles.
    int n_ctiles = 0;
    bool ct_aligned = false;
    int32_t *d_ct = nullptr;
    const int32_t *ct_m0 = nullptr;  // [n_ctiles + 1]
    // fp32 row walk (gnn.hip gnn_mlp2s_kernel RW): check tile groups -- up to 32 consecutive check
    // groups of one degree d, each a contiguous message run -- rw_meta[2 c] = {first message, checks,
    // d, degree-1 tile mask (bit i: message i of every check belongs to a degree-1 var group)},
    // rw_meta[2 c + 1].x = the first check group (lane k holds group first + k).  n_rw = 0: no such walk
    // (the checks are not contiguous runs of consecutive groups, or the groups fill their tiles too
    // sparsely).  rw_d1: the masks are in use
    // (every degree-1 var group's message lies in a masked tile, so its projected row is never read).
    int n_rw = 0;
    bool rw_d1 = false;
    int32_t *d_rw = nullptr;
    const int4 *rw_meta = nullptr;
};

namespace ldpc {

// Deterministic output stage (message_gnn_decoder.py:277-307).  The last layer writes each
// message's projected LLR into msg_out (B, E); every variable then sums its messages in ascending
// message order, as the reference's loop does, from a per-call CSR of msg_var (gnn.hip).
// Workspace: gnn_csr_ints(E, N) int32 words.
inline int64_t gnn_csr_ints(int64_t E, int N) { return 2LL * N + 2 + E; }
int gnn_build_var_csr(const int32_t *d_msg_var, int64_t E, int N, int32_t *d_ints, hipStream_t s);
// probs[b][v] = sigmoid(sum_{m -> v} msg_out[b][m] + llr[b][v]) for frames with active[b] (null = all)
int gnn_output(const float *d_msg_out, const int32_t *d_ints, const float *d_llr, int64_t E, int N, int64_t B,
               const uint8_t *d_active, float *d_probs, hipStream_t s);
__device__ __forceinline__ const int32_t *csr_ptr(const int32_t *ints) { return ints; }
__device__ __forceinline__ const int32_t *csr_mem(const int32_t *ints, int N) { return ints + 2 * N + 2; }

// fp32 forward (precision 0).  d_saved (L, B, E, H) or null: when set, layer l writes its output
// features to d_saved[l] (the last layer included) for the backward pass (gnn_train.hip).
// d_proj (training, H = 64 group plans; gnn_proj_floats floats, null = none): every layer's projected
// group rows and group means, [l][Pv (B, Gv, H) | Pc (B, Gc, H) | gv (B, Gv, H) | gc (B, Gc, H)], kept
// for the backward instead of recomputed there.
int gnn_fp32_forward(const ldpc_gnn_plan *p, int hidden, int types, int layers, const float *d_weights,
                     const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N, int64_t B,
                     float *d_probs, float *d_saved, void *d_work, int64_t work_bytes, hipStream_t s,
                     float *d_proj = nullptr, bool fp32_products = false);
int64_t gnn_proj_floats(const ldpc_gnn_plan *p, int hidden, int64_t B, int layers);
// workspace of the training forward (gnn_fp32_forward with d_saved: never the wide path)
int64_t gnn_fp32_train_workspace(const ldpc_gnn_plan *p, int hidden, int N, int64_t B, int layers);

// Layer `layer`'s projected group rows W1_s,right g + b1_s (d_pv / d_pc, (B, G, 64)) and, when
// d_gv is set, the group means g themselves (d_gv / d_gc) of c = x + emb (x = d_x, or the LLR
// embedding when d_x is null): the fp32 forward's projection kernel, for the training backward.
int gnn_project_groups(const ldpc_gnn_plan *p, int types, const float *d_weights, int layer, const float *d_x,
                       const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N, int64_t B,
                       float *d_pv, float *d_pc, float *d_gv, float *d_gc, hipStream_t s);

// fp32 layer at hidden widths H = 32 k other than 64 (gnn_wide.hip): row GEMMs on the bf16 MFMA with
// three-term splits.  Pointers are offset to the frame range [0, B); y = the layer's output rows
// (x_out); msg_out set on the last layer (the output head is applied to y).
struct GnnWideLayer {
    const ldpc_gnn_plan *plan;
    int H, T, N;
    int64_t B, E;
    const float *x_in;  // (B, E, H), null at layer 0
    const float *llr;
    const int32_t *msg_type, *msg_var;
    const float *w_in, *b_in;
    const float *emb, *w1v, *b1v, *w2v, *b2v, *w1c, *b1c, *w2c, *b2c, *wo, *bo;
    float *Mv, *Mc, *Pv, *Pc, *hbuf, *y;
    int residual;
    float *msg_out;
    // f16: the row GEMMs on scaled two-term f16 splits (else bf16x6), with each row's largest |value|
    // (float bits) recorded by its producer: x_in's (null at layer 0), y's (written here), h's and
    // the group rows' (scratch)
    bool f16;
    const uint32_t *xmax_in;
    uint32_t *xmax_out, *hmax, *gmax_v, *gmax_c;
    // H = 96 / 128 with f16 splits: this layer's fused-MLP slice images and weight exponents
    // (gnn_wide_prep), or null for the row-GEMM sequence
    const char *wimg;
    const int *wexp;
    // this layer's mean type embedding per group ((Gv + Gc), H; gnn_wide_memb), or null
    const float *memb;
};
bool gnn_wide_supported(int H);
int gnn_wide_layer(const GnnWideLayer &L, hipStream_t s);
// bytes of every layer's fused-MLP slice images (0: this H runs the row GEMMs); whether the fused
// kernel's LDS image holds T message types
int64_t gnn_wide_fused_bytes(int H, int layers);
bool gnn_wide_fused_fits(int H, int T);
// every layer's mean type embedding per var / check group (the group-mean pass adds it once)
int gnn_wide_memb(const ldpc_gnn_plan *p, int H, int layers, const float *emb0, int64_t layer_stride,
                  const int32_t *msg_type, float *memb, hipStream_t s);
int gnn_wide_prep(int H, int layers, const float *blob, int64_t layer_floats, int T, char *wimg, int *wexp, hipStream_t s);

// The per-device side stream and the calling thread's fork/join events the forwards split their
// frames over (thread-safe: see gnn.hip).
int gnn_side_stream(hipStream_t *side, hipEvent_t *fork, hipEvent_t *join);

// bf16 forward (precision 1, H = 64); same arguments as ldpc_gnn_forward.
// The workspace is sized for the largest type count the LDS image admits (kBf16MaxTypes).
constexpr int kBf16MaxTypes = 200;
int64_t gnn_bf16_workspace(const ldpc_gnn_plan *p, int N, int64_t B, int layers);
int gnn_bf16_forward(const ldpc_gnn_plan *p, int types, int layers, const float *d_weights,
                     const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N,
                     int64_t B, int flags, float *d_probs, int32_t *d_iters, void *d_work, int64_t work_bytes,
                     hipStream_t s);

// XCD-aware block order (cdna_hip_programming.md T1, bijective form): blocks that share an
// XCD (equal blockIdx % 8 under round-robin dispatch) get one contiguous range of work, so a
// frame's features and group means are pulled into one XCD's L2 instead of all eight.
// Placement only changes speed, never results.
__device__ __forceinline__ int64_t xcd_block(int64_t bid, int64_t nblk) {
    const int64_t x = bid % 8, q = nblk / 8, r = nblk % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// Tile order for the persistent MLP kernels: the tiles are split into 8 contiguous ranges, one
// per XCD group (blockIdx % 8), and the waves of that group's blocks walk their range
// interleaved, so at any moment one XCD works on a few consecutive frames and their group-mean
// rows stay in its L2.  Returns this wave's first tile and stride; tiles stop at t_end.
struct TileWalk { int64_t first, stride, end; };
__device__ __forceinline__ TileWalk xcd_tiles(int64_t ntiles, int waves_per_block, int wave) {
    const int64_t nb = gridDim.x, x = blockIdx.x % 8, i = blockIdx.x / 8;
    const int64_t q = nb / 8, r = nb % 8;
    const int64_t nbx = q + (x < r ? 1 : 0);              // blocks in this XCD group
    const int64_t before = x * q + min<int64_t>(x, r);     // blocks in earlier groups
    const int64_t t0 = ntiles * before / nb, t1 = ntiles * (before + nbx) / nb;
    return {t0 + i * waves_per_block + wave, nbx * waves_per_block, t1};
}


// ---- fp32 products as three-term bf16 splits on v_mfma_f32_32x32x16_bf16 (gnn.hip gnn_mlp2s_kernel,
// gnn_train.hip train_mlp_bwd_split_kernel): see gnn_mlp2s_kernel's comment
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
__host__ __device__ constexpr int pi16(int p) {
    return 32 * (p >> 5) + 16 * ((p >> 4) & 1) + 8 * ((p >> 2) & 1) + 4 * ((p >> 3) & 1) + (p & 3);
}
__device__ __forceinline__ void split3(const float *v, bf16x8_t &a, bf16x8_t &b, bf16x8_t &c) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const __bf16 h0 = (__bf16)v[i];
        const float r1 = v[i] - (float)h0;
        const __bf16 h1 = (__bf16)r1;
        const float r2 = r1 - (float)h1;
        a[i] = h0;
        b[i] = h1;
        c[i] = (__bf16)r2;
    }
}
// one fp32 value's three split terms at d, d + stride, d + 2 stride (the weight images)
__device__ __forceinline__ void split_store(float w, __bf16 *d, int stride) {
    const __bf16 h0 = (__bf16)w;
    const float r1 = w - (float)h0;
    const __bf16 h1 = (__bf16)r1;
    d[0] = h0;
    d[stride] = h1;
    d[2 * stride] = (__bf16)(r1 - (float)h1);
}
__device__ __forceinline__ bf16x8_t lds8(const __bf16 *p) { return *reinterpret_cast<const bf16x8_t *>(p); }
// ---- fp32 products as scaled two-term f16 splits on v_mfma_f32_32x32x16_f16 (gnn.hip
// gnn_mlp2s_kernel, gnn_train.hip train_mlp_bwd_s6_kernel): an operand column scaled by a power of
// two (its largest magnitude to at most 2^15, inside f16's normal range) splits as v = v0 + v1,
// v0 = f16(v), v1 = f16(v - v0) (22 significant bits); a product is a1 b0 + a0 b1 + a0 b0
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
// v1 = f16(v - v0) as one v_fma_mixlo / mixhi_f16 per value: fma(-v0, 1, v) with v0 read as f16
// straight from the packed pair and rounded once to f16 -- the same value as converting v0 back,
// subtracting in f32 (exact: v0 is v rounded) and converting again (tools/ubench/split_mix.hip,
// 2^23 pairs bit for bit), in 12 instead of ~24 VALU per 8 values.  LDPC_SPLIT_MIX=0: that form.
#ifndef LDPC_SPLIT_MIX
#define LDPC_SPLIT_MIX 1
#endif
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2h(const float *v, f16x8_t &a, f16x8_t &b) {
#if LDPC_SPLIT_MIX
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const f16x2_t h = {(_Float16)v[2 * p], (_Float16)v[2 * p + 1]};  // v_cvt_pk_f16_f32
        hi[p] = __builtin_bit_cast(uint32_t, h);
        uint32_t r;
        asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hi[p]), "v"(v[2 * p]));
        asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(r) : "v"(hi[p]), "v"(v[2 * p + 1]));
        lo[p] = r;
    }
    a = __builtin_bit_cast(f16x8_t, hi);
    b = __builtin_bit_cast(f16x8_t, lo);
#else
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const _Float16 h0 = (_Float16)v[i];
        a[i] = h0;
        b[i] = (_Float16)(v[i] - (float)h0);
    }
#endif
}
__device__ __forceinline__ void split2h_store(float w, _Float16 *d, int stride) {
    const _Float16 h0 = (_Float16)w;
    d[0] = h0;
    d[stride] = (_Float16)(w - (float)h0);
}
// ReLU as torch.relu computes it (message_gnn_decoder.py:36-46): max(v, 0) for numbers, a NaN stays
// NaN.  One v_maximum3_f32 on gfx950 (IEEE 754-2019 maximum), the cost of the fmaxf / integer max it
// replaced, which both map a NaN to 0 (a NaN feature would then vanish from its frame mid-graph)
__device__ __forceinline__ float relu_nan(float v) { return __builtin_elementwise_maximum(v, 0.0f); }
// 2^e as a float (e clamped to the normal range)
__device__ __forceinline__ float pow2f(int e) { return __int_as_float((min(max(e, -126), 127) + 127) << 23); }
// the exponent that scales a column whose largest magnitude is m (>= 0) to at most 2^15 (0: m is
// zero, subnormal, inf or NaN)
__device__ __forceinline__ int col_exp(float m) {
    const int b = (__float_as_int(m) >> 23) & 0xff;
    return b == 0 || b == 255 ? 0 : 141 - b;  // 14 - (b - 127)
}
// ... for an activation column multiplied by weights scaled 2^wexp: clamped so that the product scale
// 2^(e + wexp) and its inverse stay normal floats, so csc * wsc, asc and iasc invert each other
// exactly.  The upper clamp only lowers the column's scale (its split stays in range);
// the lower one binds only where the fp32 products themselves overflow.  The outer clamp keeps the
// column's own scale 2^e a normal float too (pow2f exact) when the weights' exponent is far from 0.
__device__ __forceinline__ int col_exp_w(float m, int wexp) {
    return min(max(min(max(col_exp(m), -126 - wexp), 126 - wexp), -126), 127);
}
// acc += A B over one K = 16 step: A's two split images at img and img + img_stride
__device__ __forceinline__ f32x16_t mfma3h(const _Float16 *img, const f16x8_t &b0, const f16x8_t &b1, f32x16_t acc,
                                           int img_stride) {
    const f16x8_t a0 = *reinterpret_cast<const f16x8_t *>(img), a1 = *reinterpret_cast<const f16x8_t *>(img + img_stride);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc, 0, 0, 0);
}
// acc += A B over one K = 16 step, A from the three split images at img (+ img_stride, + 2 img_stride)
__device__ __forceinline__ f32x16_t mfma6(const __bf16 *img, const bf16x8_t &b0, const bf16x8_t &b1,
                                        const bf16x8_t &b2, f32x16_t acc, int img_stride) {
    const bf16x8_t a0 = lds8(img), a1 = lds8(img + img_stride), a2 = lds8(img + 2 * img_stride);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc, 0, 0, 0);
}


}  // namespace ldpc
