// gnn_wide.hip -- MessageGNNLayer (message_gnn_decoder.py:51-129) for hidden widths H = 32 k other
// than 64 (96 .. 256) on the MFMA, every fp32 product fp32-accurate:
//   F16 (default, round 6): scaled two-term f16 splits on v_mfma_f32_32x32x16_f16, as the H = 64
//       kernels (gnn.hpp split2h / mfma3h): each workgroup's weight slice under one power of two
//       (its largest |w| to at most 2^15), each input row under its own, from the row's largest
//       |value| that the row's producer recorded (GEMM2's epilogue for the next layer's x, GEMM1's
//       for h, the group-mean kernel for the group rows; layer 0 from its LLR), so both operands
//       hold 22 significant bits in f16's normal range: 3 MFMAs per K = 16 step.
//   !F16 (LDPC_GNN_FP32_PRODUCTS: weights whose rows span more than the splits' range): the three-term
//       bf16 split of gnn_mlp2s_kernel's earlier form (v = v0 + v1 + v2 in bf16, six cross products).
//
// The H = 64 path keeps a layer's four weight matrices in LDS and runs the whole MLP per 32-message
// tile.  At H = 128 the split images of those matrices are 384 KB, so a layer here is a sequence of
// row GEMMs, each over one slice of output units whose split weight images fit a CU's LDS:
//   gnn_wide_gm_kernel   group means of c = x + emb[type] (the normalized clique adjacencies of
//                        MGD:108/118 are segment means): Mv (B, Gv, H), Mc (B, Gc, H)
//   gnn_wgemm_kernel     P_s = W1_s,right g_s + b1_s per group          (mode PROJ, both sides)
//                        h_s = relu(W1_s,left c + P_s[group(m)])        (mode GEMM1, per side)
//                        y = W2_v h_v + W2_c h_c + b2_v + b2_c (+ x)    (mode GEMM2, K = 2 H)
//   gnn_wide_head_kernel msg_out = wo . y + bo on the last layer (MGD:142, :270)
// At H = 96 and 128 (round 6) GEMM1, GEMM2 and the head are one kernel, gnn_wide_mlp_kernel, that
// keeps h in registers and streams the weights slice by slice (below); the other widths run the
// row GEMMs, where h (B, E, 2 H) fp32 is the one extra round trip through HBM.  Each launch is persistent: a
// workgroup holds one output slice's split images in LDS and its waves walk 32-row tiles; the
// slices of one XCD walk the same tiles in step, so the input rows are read from HBM once per XCD
// and hit L2 for the other slices (placement changes speed only, never results).
#include <algorithm>
#include <type_traits>
#include <cstdint>
#include <cstdlib>

#include "common.hpp"
#include "gnn.hpp"

namespace ldpc {
namespace {

typedef float f32x16w __attribute__((ext_vector_type(16)));

enum WMode { kProj = 0, kGemm1 = 1, kGemm2 = 2 };

struct WArgs {
    int mode;
    int K;             // reduction length (H, or 2 H for GEMM2)
    int H;             // output row width
    int NS;            // output units per workgroup slice (32 * NT)
    int64_t R;         // rows
    // input rows: in + r * in_stride (K floats); GEMM1 at layer 0: x = llr w_in + b_in
    const float *in;
    int64_t in_stride;
    // weights: row u of the (H x ld) matrix W, columns col0 .. col0 + K (GEMM2: W2v | W2c)
    const float *w_a, *w_b;  // GEMM2: W2v, W2c; else w_a = W1_s (H x 2H), w_b unused
    int ld, col0;
    // GEMM1: c = x + emb[type]; rows are (frame, message) pairs of E messages
    const float *emb;      // (T, H)
    const int32_t *msg_type, *msg_var;
    const float *llr, *w_in, *b_in;
    int N, T;
    int64_t E;
    // init: PROJ bias vector b (H); GEMM1 P_s rows (B, G, H) indexed by grp[m]; GEMM2 b2v + b2c
    const float *init_a, *init_b;
    const int32_t *grp;
    int G;
    const float *resid;    // GEMM2: x (B E, H) or null
    float *out;
    int64_t out_stride;    // floats per output row
    // F16: per input row, the bits of its largest |value| (GEMM2: h; GEMM1: x, null at layer 0; PROJ:
    // the group row); per output row, atomicMax of the largest |output| (GEMM1: h; GEMM2: the next
    // layer's x; null: not recorded).  Non-negative floats order as their bits.
    const uint32_t *in_max;
    uint32_t *out_max;
};

constexpr int kWRowPad = 8;  // bf16 per image row past K: conflict-free ds_read_b128 (as gnn_bf16.hip's W1)
// split images of the slice's weights: 2 (f16) or 3 (bf16) terms, 2 bytes each
__host__ __device__ inline size_t wgemm_img_bytes(int NS, int K, bool f16) { return (size_t)(f16 ? 2 : 3) * NS * (K + kWRowPad) * 2; }
inline size_t wgemm_lds_bytes(const WArgs &a, bool f16) {
    size_t b = wgemm_img_bytes(a.NS, a.K, f16);
    if (a.mode == kGemm1) b += (size_t)(a.T + 2) * a.H * 4 + (size_t)(a.T + 2) * 4;  // emb rows, w_in, b_in; their maxima
    b += (size_t)a.NS * 4;                                  // the slice's init vector (PROJ / GEMM2)
    return (b + 15) / 16 * 16;
}

__device__ __forceinline__ void split3w(const float *v, bf16x8_t &a, bf16x8_t &b, bf16x8_t &c) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const __bf16 h0 = (__bf16)v[i];
        const float r1 = v[i] - (float)h0;
        const __bf16 h1 = (__bf16)r1;
        a[i] = h0;
        b[i] = h1;
        c[i] = (__bf16)(r1 - (float)h1);
    }
}


// NT accumulator tiles of 32 output units per wave; 512 threads (8 waves) per workgroup, one or two
// workgroups per CU by the LDS image
constexpr int kWThreads = 512, kWWaves = kWThreads / 64;
// AH: input k-steps in flight ahead of the one being multiplied.  The ring slot of chunk s is s % AH
// on every tile, so AH must divide the k-step count: 4 when it does (K = 64 k), else 2 (K = 32 k,
// the odd multiples of 32: H = 96, 160, 224 in the projection and GEMM1)
template <int NT, int AH, bool F16>
__global__ __launch_bounds__(kWThreads, 1) void gnn_wgemm_kernel(WArgs A, int nslices) {
    constexpr int kWAhead = AH;
    typedef typename std::conditional<F16, _Float16, __bf16>::type w_t;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ uint32_t wmax_bits;
    const int tid = threadIdx.x, lane = tid & 63, j = lane & 31, h = lane >> 5, wave = tid >> 6;
    constexpr int NS = 32 * NT;
    // placement: XCD x = blockIdx % 8 hosts every slice; the blocks of (x, slice) share x's tile range
    const int x = blockIdx.x % 8, ix = blockIdx.x / 8;
    const int per_x = gridDim.x / 8;
    const int slice = ix % nslices, rank = ix / nslices;
    const int nrank = per_x / nslices;
    if (rank >= nrank) return;
    const int n0 = slice * NS;
    const int K = A.K, rowb = K + kWRowPad;  // elements per image row
    w_t *img = reinterpret_cast<w_t *>(smem);
    const int imgstride = NS * rowb;
    auto wval = [&](int u, int k) {
        return A.mode == kGemm2 ? (k < A.H ? A.w_a[(int64_t)(n0 + u) * A.H + k] : A.w_b[(int64_t)(n0 + u) * A.H + k - A.H])
                                : A.w_a[(int64_t)(n0 + u) * A.ld + A.col0 + k];
    };
    int wexp = 0;
    if constexpr (F16) {  // the slice's weights under one power of two: its largest |w| to at most 2^15
        if (tid == 0) wmax_bits = 0u;
        __syncthreads();
        float m = 0.0f;
        for (int i = tid; i < NS * K; i += kWThreads) m = fmaxf(m, fabsf(wval(i / K, i % K)));
        atomicMax(&wmax_bits, __float_as_uint(m));
        __syncthreads();
        wexp = min(col_exp(__uint_as_float(wmax_bits)), 126);
        const float wsc = pow2f(wexp);
        for (int i = tid; i < NS * K; i += kWThreads) {
            const int u = i / K, k = i - u * K;
            split2h_store(wval(u, k) * wsc, img + u * rowb + k, imgstride);
        }
    } else {
        for (int i = tid; i < NS * K; i += kWThreads) {
            const int u = i / K, k = i - u * K;
            split_store(wval(u, k), img + u * rowb + k, imgstride);
        }
    }
    float *tabs = reinterpret_cast<float *>(smem + wgemm_img_bytes(NS, K, F16));
    float *initv = tabs;  // [NS]
    float *embs = tabs + NS;  // GEMM1: emb [T][H], w_in [H], b_in [H], then max |emb[t]| [T], max |w_in|, max |b_in|
    float *embmax = embs + (A.T + 2) * A.H;
    if (A.mode != kGemm1)
        for (int i = tid; i < NS; i += kWThreads)
            initv[i] = A.mode == kGemm2 ? A.init_a[n0 + i] + A.init_b[n0 + i] : A.init_a[n0 + i];
    if (A.mode == kGemm1) {
        for (int i = tid; i < A.T * A.H; i += kWThreads) embs[i] = A.emb[i];
        for (int i = tid; i < A.H; i += kWThreads) {
            embs[A.T * A.H + i] = A.w_in[i];
            embs[(A.T + 1) * A.H + i] = A.b_in[i];
        }
        if constexpr (F16) {
            for (int r = wave; r < A.T + 2; r += kWWaves) {  // one wave per row: its largest |value|
                const float *src = r < A.T ? A.emb + (int64_t)r * A.H : r == A.T ? A.w_in : A.b_in;
                float m = 0.0f;
                for (int u = lane; u < A.H; u += 64) m = fmaxf(m, fabsf(src[u]));
                for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
                if (lane == 0) embmax[r] = m;
            }
        }
    }
    __syncthreads();

    // this XCD's contiguous tile range, walked by the (x, slice) blocks' waves interleaved
    const int64_t ntiles = (A.R + 31) / 32;
    const int64_t t0 = ntiles * x / 8, t1 = ntiles * (x + 1) / 8;
    const int ksteps = K / 16;
    // Per tile: the row context (row, frame, message, input pointer, type embedding, LLR, the row's
    // split scale).  Past the end a context points at a valid row (its loads are discarded): no
    // branch around any load.
    struct Ctx {
        int64_t t, rr, fb, m;
        bool ok, live;
        const float *src, *eb;
        float lv, bnd;
    };
    auto ctx_of = [&](int64_t t) {
        Ctx c;
        c.t = t;
        c.live = t < t1;
        const int64_t r = t * 32 + j;
        c.ok = c.live && r < A.R;
        c.rr = c.ok ? r : A.R - 1;
        c.fb = 0;
        c.m = 0;
        if (A.mode == kGemm1) {
            c.fb = c.rr / A.E;
            c.m = c.rr - c.fb * A.E;
        }
        c.src = A.in ? A.in + c.rr * A.in_stride + 8 * h : nullptr;
        const int ty = A.mode == kGemm1 ? A.msg_type[c.m] : 0;
        c.eb = A.mode == kGemm1 ? embs + ty * A.H + 8 * h : nullptr;
        c.lv = (A.mode == kGemm1 && !A.in) ? A.llr[c.fb * A.N + A.msg_var[c.m]] : 0.0f;
        c.bnd = 0.0f;
        if constexpr (F16) {
            // a bound on the row's largest |input|: recorded (h, x, group rows), or for layer 0's
            // x = llr w_in + b_in, |llr| max |w_in| + max |b_in|; GEMM1 adds max |emb[type]|
            if (A.in) c.bnd = __uint_as_float(A.in_max[c.rr]);
            else c.bnd = fabsf(c.lv) * embmax[A.T] + embmax[A.T + 1];
            if (A.mode == kGemm1) c.bnd = c.bnd + embmax[ty];
        }
        return c;
    };
    // input chunk of k-step s: units 16 s + 8 h .. + 7 of the context's row (before the embedding)
    auto chunk = [&](const Ctx &c, int s, float *v) {
        if (c.src) {
            const float4 a = *reinterpret_cast<const float4 *>(c.src + 16 * s);
            const float4 b = *reinterpret_cast<const float4 *>(c.src + 16 * s + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        } else {  // layer 0: Linear(1, H) of the message's LLR
            const float *wi = embs + A.T * A.H + 16 * s + 8 * h, *bi = wi + A.H;
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = c.lv * wi[i] + bi[i];
        }
    };
    const int64_t stride = (int64_t)nrank * kWWaves;
    Ctx cur = ctx_of(t0 + (int64_t)rank * kWWaves + wave);
    if (!cur.live) return;
    // a ring of kWAhead input chunks, continuous over tiles: while chunk s of this tile is multiplied,
    // chunk s + kWAhead -- of this tile, or of the next one near the end -- is in flight
    float ring[kWAhead][8];
#pragma unroll
    for (int a = 0; a < kWAhead; ++a) chunk(cur, a, ring[a]);  // K >= 96: ksteps >= kWAhead, ksteps % kWAhead == 0
    const w_t *wl = img + j * rowb + 8 * h;
    while (cur.live) {
        const Ctx nxt = ctx_of(cur.t + stride);
        // the row's split scale (column j of B): csc = 2^cexp, the accumulators run at csc 2^wexp
        float csc = 1.0f, asc = 1.0f, iasc = 1.0f;
        if constexpr (F16) {
            const int cexp = col_exp_w(cur.bnd, wexp);
            csc = pow2f(cexp);
            asc = pow2f(cexp + wexp);
            iasc = pow2f(-cexp - wexp);
        }
        // accumulators start from the additive term (GEMM1: the projected group row; GEMM2: b2 + x;
        // projection: b1), loaded with the tile's first chunks instead of after its last MFMA
        f32x16w acc[NT];
        {
            const float *ip = A.mode == kGemm1 ? A.init_a + (cur.fb * A.G + A.grp[cur.m]) * A.H + n0 + 4 * h : nullptr;
            const float *xp = A.resid ? A.resid + cur.rr * A.H + n0 + 4 * h : nullptr;
#pragma unroll
            for (int tt = 0; tt < NT; ++tt)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int u = 32 * tt + 8 * q;
                    float4 iv = ip ? *reinterpret_cast<const float4 *>(ip + u) : *reinterpret_cast<const float4 *>(initv + u + 4 * h);
                    if (xp) {
                        const float4 xv = *reinterpret_cast<const float4 *>(xp + u);
                        iv = make_float4(xv.x + iv.x, xv.y + iv.y, xv.z + iv.z, xv.w + iv.w);
                    }
                    acc[tt][4 * q] = iv.x; acc[tt][4 * q + 1] = iv.y; acc[tt][4 * q + 2] = iv.z; acc[tt][4 * q + 3] = iv.w;
                }
            if constexpr (F16)
#pragma unroll
                for (int tt = 0; tt < NT; ++tt) acc[tt] *= asc;  // exact: a power of two
        }
        for (int s0 = 0; s0 < ksteps; s0 += kWAhead) {
#pragma unroll
            for (int a = 0; a < kWAhead; ++a) {
                const int s = s0 + a;
                if (s < ksteps) {
                    float v[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] = ring[a][i] + (cur.eb ? cur.eb[16 * s + i] : 0.0f);
                    if (s + kWAhead < ksteps)
                        chunk(cur, s + kWAhead, ring[a]);
                    else
                        chunk(nxt, s + kWAhead - ksteps, ring[a]);
                    if constexpr (F16) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) v[i] *= csc;
                        f16x8_t b0, b1;
                        split2h(v, b0, b1);
#pragma unroll
                        for (int q = 0; q < NT; ++q) acc[q] = mfma3h(wl + 32 * q * rowb + 16 * s, b0, b1, acc[q], imgstride);
                    } else {
                        bf16x8_t b0, b1, b2;
                        split3w(v, b0, b1, b2);
#pragma unroll
                        for (int q = 0; q < NT; ++q) acc[q] = mfma6(wl + 32 * q * rowb + 16 * s, b0, b1, b2, acc[q], imgstride);
                    }
                }
            }
        }
        if constexpr (F16)
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) acc[tt] *= iasc;
        // register 4 q + i of tile tt holds unit n0 + 32 tt + 8 q + 4 h + i of the row
        float om = 0.0f;  // the largest |output| of this lane's units (recorded for the row's consumer)
#pragma unroll
        for (int tt = 0; tt < NT; ++tt)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float4 o = make_float4(acc[tt][4 * q], acc[tt][4 * q + 1], acc[tt][4 * q + 2], acc[tt][4 * q + 3]);
                if (A.mode == kGemm1) o = make_float4(relu_nan(o.x), relu_nan(o.y), relu_nan(o.z), relu_nan(o.w));
                acc[tt][4 * q] = o.x; acc[tt][4 * q + 1] = o.y; acc[tt][4 * q + 2] = o.z; acc[tt][4 * q + 3] = o.w;
                om = fmaxf(om, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
            }
        if (cur.ok) {
            float *op = A.out + cur.rr * A.out_stride + n0 + 4 * h;
#pragma unroll
            for (int tt = 0; tt < NT; ++tt)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    *reinterpret_cast<float4 *>(op + 32 * tt + 8 * q) =
                        make_float4(acc[tt][4 * q], acc[tt][4 * q + 1], acc[tt][4 * q + 2], acc[tt][4 * q + 3]);
        }
        if (A.out_max) {  // both lane halves hold the row's units: one atomic per row and slice
            om = fmaxf(om, __shfl_xor(om, 32, 64));
            if (cur.ok && h == 0) atomicMax(A.out_max + cur.rr, __float_as_uint(om));
        }
        cur = nxt;
    }
}

// Group means of c = x + emb[type] (layer 0: x = llr w_in + b_in) over the plan's group tiles
// (gnn.hpp gt_*: 8 groups of one degree per tile, var side then check side): H / 4 lanes per group
// (one float4 each), 64 / (H / 4) groups per wave, members in ascending order, four in flight.
struct WGm {
    const float *x;        // (B, E, H) or null (layer 0)
    const float *llr, *w_in, *b_in, *emb;
    const int32_t *msg_type, *msg_var;
    const int2 *meta;
    const int32_t *grp, *mem;
    int n_tiles;
    const float *inv_v, *inv_c;
    float *Mv, *Mc;
    uint32_t *gmax_v, *gmax_c;  // F16: each row's largest |value| (bits), or null
    // this layer's mean type embedding per group ((Gv + Gc), H; gnn_wide_memb_kernel), or null: the
    // group mean is then mean(x) + memb[g] (the members' types are not read per frame)
    const float *memb;
    int Gv, Gc, H, N, gpw;  // gpw: groups per wave
    int64_t E, B;
};

// every layer's mean type embedding per var / check group: memb[l][g][u] = mean over g's members of
// emb_l[type][u] (ascending member order), g < Gv the var groups, then the check groups
__global__ void gnn_wide_memb_kernel(const float *__restrict__ emb0, int64_t layer_stride, int H,
                                     const int32_t *__restrict__ msg_type, const int32_t *__restrict__ vg_ptr,
                                     const int32_t *__restrict__ vg_mem, const float *__restrict__ inv_v,
                                     const int32_t *__restrict__ cg_ptr, const int32_t *__restrict__ cg_mem,
                                     const float *__restrict__ inv_c, int Gv, int Gc, int layers,
                                     float *__restrict__ memb) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, G = Gv + Gc;
    if (i >= (int64_t)layers * G * H) return;
    const int64_t l = i / (G * H);
    const int g = (int)(i / H - l * G), u = (int)(i % H);
    const float *emb = emb0 + l * layer_stride;
    const bool v = g < Gv;
    const int gg = v ? g : g - Gv;
    const int32_t *ptr = v ? vg_ptr : cg_ptr, *mem = v ? vg_mem : cg_mem;
    float s = 0.0f;
    for (int k = ptr[gg]; k < ptr[gg + 1]; ++k) s += emb[(int64_t)msg_type[mem[k]] * H + u];
    memb[i] = s * (v ? inv_v : inv_c)[gg];
}

// V float4 per lane (V = 2: half the lanes per group, twice the groups per wave -- most groups are
// of degree 1, so a wave's life is mostly its dispatch and its first load; V = 2 measured +4.3 % on
// gnn-z32-h128 against V = 1, profiles/r06/wgm_v/)
template <int V>
__global__ __launch_bounds__(256) void gnn_wide_gm_kernel(WGm A) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, lg = A.H / (4 * V);
    const int wpt = 8 / A.gpw;  // waves per tile
    const int64_t tile_w = w / wpt;
    if (tile_w >= A.B * A.n_tiles) return;
    const int64_t b = tile_w / A.n_tiles;
    const int t = (int)(tile_w - b * A.n_tiles);
    const int q = (int)(w - tile_w * wpt) * A.gpw + lane / lg, u = 4 * V * (lane % lg);
    if (lane / lg >= A.gpw) return;
    const int2 md = A.meta[t];
    const int g = A.grp[8 * t + q];
    if (g < 0) return;
    const int32_t *mem = A.mem + md.y + q;
    float4 s[V];
#pragma unroll
    for (int c = 0; c < V; ++c) s[c] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    auto feat = [&](int mm, int c) {
        if (A.x) return *reinterpret_cast<const float4 *>(A.x + (b * A.E + mm) * A.H + u + 4 * c);
        const float l = A.llr[b * A.N + A.msg_var[mm]];
        const float4 wi = *reinterpret_cast<const float4 *>(A.w_in + u + 4 * c), bi = *reinterpret_cast<const float4 *>(A.b_in + u + 4 * c);
        return make_float4(l * wi.x + bi.x, l * wi.y + bi.y, l * wi.z + bi.z, l * wi.w + bi.w);
    };
    auto add = [&](float4 v, int mm, int c) {
        if (A.memb) {  // (uniform) the type embeddings' mean is added once, below
            s[c].x += v.x; s[c].y += v.y; s[c].z += v.z; s[c].w += v.w;
        } else {
            const float4 e = *reinterpret_cast<const float4 *>(A.emb + (int64_t)A.msg_type[mm] * A.H + u + 4 * c);
            s[c].x += v.x + e.x; s[c].y += v.y + e.y; s[c].z += v.z + e.z; s[c].w += v.w + e.w;
        }
    };
    int i = 0;
    for (; i + 4 <= md.x; i += 4) {  // four members' rows in flight, summed in ascending order
        const int m0 = mem[8 * i], m1 = mem[8 * i + 8], m2 = mem[8 * i + 16], m3 = mem[8 * i + 24];
        float4 v0[V], v1[V], v2[V], v3[V];
#pragma unroll
        for (int c = 0; c < V; ++c) {
            v0[c] = feat(m0, c);
            v1[c] = feat(m1, c);
            v2[c] = feat(m2, c);
            v3[c] = feat(m3, c);
        }
#pragma unroll
        for (int c = 0; c < V; ++c) {
            add(v0[c], m0, c);
            add(v1[c], m1, c);
            add(v2[c], m2, c);
            add(v3[c], m3, c);
        }
    }
    for (; i < md.x; ++i) {
        const int mm = mem[8 * i];
        float4 v[V];
#pragma unroll
        for (int c = 0; c < V; ++c) v[c] = feat(mm, c);
#pragma unroll
        for (int c = 0; c < V; ++c) add(v[c], mm, c);
    }
    const bool isv = g < A.Gv;
    const int gg = isv ? g : g - A.Gv;
    const float inv = isv ? A.inv_v[gg] : A.inv_c[gg];
    float *dst = isv ? A.Mv + (b * A.Gv + gg) * A.H : A.Mc + (b * A.Gc + gg) * A.H;
    float m = 0.0f;
#pragma unroll
    for (int c = 0; c < V; ++c) {
        float4 mean = make_float4(s[c].x * inv, s[c].y * inv, s[c].z * inv, s[c].w * inv);
        if (A.memb) {
            const float4 e = *reinterpret_cast<const float4 *>(A.memb + (int64_t)g * A.H + u + 4 * c);
            mean = make_float4(mean.x + e.x, mean.y + e.y, mean.z + e.z, mean.w + e.w);
        }
        *reinterpret_cast<float4 *>(dst + u + 4 * c) = mean;
        m = fmaxf(m, fmaxf(fmaxf(fabsf(mean.x), fabsf(mean.y)), fmaxf(fabsf(mean.z), fabsf(mean.w))));
    }
    if (A.gmax_v) {  // the row's largest |value| over its lg lanes (a segmented max; no lane leaves it)
        const int seg0 = (lane / lg) * lg;
        for (int off = 1; off < lg; off <<= 1) {
            const float o = __shfl_down(m, off, 64);
            if (lane + off < seg0 + lg) m = fmaxf(m, o);
        }
        if (lane == seg0) (isv ? A.gmax_v + b * A.Gv + gg : A.gmax_c + b * A.Gc + gg)[0] = __float_as_uint(m);
    }
}

// msg_out[r] = wo . y[r] + bo (16 lanes per row)
__global__ __launch_bounds__(256) void gnn_wide_head_kernel(const float *__restrict__ y, int H, int64_t R,
                                                            const float *__restrict__ wo, const float *__restrict__ bo,
                                                            float *__restrict__ msg_out) {
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const int q = threadIdx.x & 15;
    if (r >= R) return;
    const float *yr = y + r * H;
    float part = 0.0f;
    for (int u = q; u < H; u += 16) part += yr[u] * wo[u];
    for (int off = 8; off > 0; off >>= 1) part += __shfl_xor(part, off, 16);
    if (q == 0) msg_out[r] = part + bo[0];
}

// ------------------------------------------------------------------------ fused MLP (H = 96 .. 192)
// The layer's whole MLP per 32-row tile, h never leaving registers: for each slice of 32 hidden units
// (side s, units 32 tt ..), h = relu(W1_s,left c + P_s[group]) on the tile (GEMM1, K = H), then its
// contribution W2_s[:, slice] relu(h) to every output unit of y (GEMM2 over the slice's 32 columns).
// The 2 H / 32 slices' split weight images (W1 rows of the slice, W2 columns of the slice; 38 KB at
// H = 128) stream from a per-forward global copy (gnn_wide_prep_kernel) through a two-slot LDS ring
// shared by the workgroup's waves, one barrier per slice; each wave owns one tile per pass.
// Scales: the tile's c per row from its exact largest |c|; relu(h) per row and slice from the slice's
// largest value, under a running exponent that only moves down (a larger slice maximum lowers it and
// rescales y's accumulators by the exact power of two), so every slice's split is at least as fine
// as one scale over the row's whole h would be.  This replaces GEMM1, GEMM2 and the head: h's
// (B, E, 2 H) round trip through HBM (4 E H of the layer's 12 E H words) disappears.
template <int H>
struct WFused {
    static constexpr int NT = H / 32;                  // 32-unit tiles per side (hidden or output)
    static constexpr int S = 2 * NT;                   // slices per layer (both sides)
    static constexpr int R1 = H + 8, R2 = 40;          // f16 per image row (W1: K = H; W2: K = 32) + pad
    static constexpr int I1 = 32 * R1, I2 = H * R2;    // elements per split image
    static constexpr int W2OFF = 2 * I1;               // W2's images after W1's two
    // waves per workgroup (one workgroup per CU): two per SIMD up to H = 128; past it the tile's y
    // and c split (H / 2 registers each) need one wave per SIMD's 512 registers
    static constexpr int NW = H <= 128 ? 8 : 4, NTH = 64 * NW;
    // bytes per slice, padded to whole 1-KB LDS-DMA rounds of the workgroup's waves
    static constexpr int BYTES = ((2 * I1 + 2 * I2) * 2 + 1024 * NW - 1) / (1024 * NW) * (1024 * NW);
    static constexpr int KS = H / 16;                  // GEMM1 k-steps
    static constexpr int ES = H + 4;                   // emb table row stride (floats)
};

// One 16-B LDS-DMA load per lane: the wave's 64 lanes' 16 B land at LDS byte address lds (wave
// uniform) + 16 lane.  Inline asm, because hipcc waits for a builtin LDS-DMA before every later
// ds_read it cannot prove disjoint (here: each weight read of the other ring slot), which drains the
// copy as soon as it is issued; the caller counts completion itself (s_waitcnt vmcnt, then a barrier).
// M0 is the compiler's: saved and restored inside the statement.
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds)
                 : "memory");
}

// one workgroup per layer: both power-of-two weight scales, then every slice image of the layer
template <int H>
__global__ __launch_bounds__(1024) void gnn_wide_prep_kernel(const float *blob, int64_t layer_floats, int T,
                                                              char *wimg, int *wexp) {
    using F = WFused<H>;
    __shared__ uint32_t m1b, m2b;
    const int tid = threadIdx.x, l = blockIdx.x;
    const float *w1v = blob + 2 * H + (int64_t)l * layer_floats + (int64_t)T * H;
    const float *w2v = w1v + 2 * H * H + H, *w1c = w2v + H * H + H, *w2c = w1c + 2 * H * H + H;
    if (tid == 0) { m1b = 0u; m2b = 0u; }
    __syncthreads();
    float m1 = 0.0f, m2 = 0.0f;
    for (int i = tid; i < H * H; i += 1024) {
        const int u = i / H, k = i - u * H;
        m1 = fmaxf(m1, fmaxf(fabsf(w1v[u * 2 * H + k]), fabsf(w1c[u * 2 * H + k])));
        m2 = fmaxf(m2, fmaxf(fabsf(w2v[i]), fabsf(w2c[i])));
    }
    atomicMax(&m1b, __float_as_uint(m1));
    atomicMax(&m2b, __float_as_uint(m2));
    __syncthreads();
    const int e1 = min(col_exp(__uint_as_float(m1b)), 126), e2 = min(col_exp(__uint_as_float(m2b)), 126);
    if (tid == 0) { wexp[2 * l] = e1; wexp[2 * l + 1] = e2; }
    const float s1 = pow2f(e1), s2 = pow2f(e2);
    _Float16 *base = reinterpret_cast<_Float16 *>(wimg + (int64_t)l * F::S * F::BYTES);
    for (int sl = 0; sl < F::S; ++sl) {
        const int side = sl / F::NT, tt = sl - side * F::NT;
        const float *W1 = side ? w1c : w1v, *W2 = side ? w2c : w2v;
        _Float16 *img = base + (int64_t)sl * (F::BYTES / 2);
        // W1 rows: hidden unit 32 tt + r, column p = x unit pi16(p) (GEMM1's B operand order)
        for (int i = tid; i < 32 * H; i += 1024) {
            const int r = i / H, p = i - r * H;
            split2h_store(W1[(32 * tt + r) * 2 * H + pi16(p)] * s1, img + r * F::R1 + p, F::I1);
        }
        // W2 columns of the slice: output unit o, column q = hidden unit 32 tt + pi16(q) (the order
        // in which a lane's h accumulator registers feed GEMM2's B operand)
        for (int i = tid; i < H * 32; i += 1024) {
            const int o = i >> 5, q = i & 31;
            split2h_store(W2[o * H + 32 * tt + pi16(q)] * s2, img + F::W2OFF + o * F::R2 + q, F::I2);
        }
    }
}

struct WMlp {
    const char *wimg;   // this layer's slice images (gnn_wide_prep_kernel)
    const int *wexp;    // this layer's {W1 scale, W2 scale} exponents
    const float *x_in;  // (R, H), null at layer 0
    const float *llr, *w_in, *b_in, *emb;
    const int32_t *msg_type, *msg_var, *vgroup, *cgroup;
    const float *Pv, *Pc;
    const float *b2v, *b2c, *wo, *bo;
    float *y, *msg_out;  // msg_out: the last layer's head (y then unused)
    int residual, N, T, Gv, Gc;
    int64_t E, R;
};

template <int H>
inline size_t wide_mlp_lds_bytes(int T) { return 2 * (size_t)WFused<H>::BYTES + ((size_t)T * WFused<H>::ES + 4 * H) * 4; }

// L0: layer 0 (x from the LLRs; no x rows to prefetch)
template <int H, bool L0>
__global__ __launch_bounds__(WFused<H>::NTH, 1) void gnn_wide_mlp_kernel(WMlp A) {
    using F = WFused<H>;
    constexpr int NT = F::NT, S = F::S, KS = F::KS, NW = F::NW, NTH = F::NTH;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, j = lane & 31, h = lane >> 5, wave = tid >> 6;
    float *tab = reinterpret_cast<float *>(smem + 2 * F::BYTES);
    float *embs = tab, *win = tab + A.T * F::ES, *bin = win + H, *b2 = bin + H, *wo = b2 + H;
    for (int i = tid; i < A.T * H; i += NTH) embs[(i / H) * F::ES + i % H] = A.emb[i];
    for (int i = tid; i < H; i += NTH) {
        win[i] = A.w_in[i];
        bin[i] = A.b_in[i];
        b2[i] = A.b2v[i] + A.b2c[i];
        wo[i] = A.msg_out ? A.wo[i] : 0.0f;
    }
    constexpr int NF4 = F::BYTES / 16, CP = NF4 / NTH;  // float4 per slice, per thread (exact)
    const float4 *gimg = reinterpret_cast<const float4 *>(A.wimg);
    auto slot = [&](int64_t k) { return reinterpret_cast<float4 *>(smem + (k & 1) * F::BYTES); };
    for (int i = tid; i < NF4; i += NTH) slot(0)[i] = gimg[i];
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)smem;
    const int wexp1 = A.wexp[0], wexp2 = A.wexp[1];
    const float bo = A.msg_out ? A.bo[0] : 0.0f;

    // passes: this XCD's tiles, NW per pass (one per wave) per workgroup
    const int64_t ntiles = (A.R + 31) / 32;
    const int x = blockIdx.x % 8, rank = blockIdx.x / 8, nrank = gridDim.x / 8;
    const int64_t t0 = ntiles * x / 8, t1 = ntiles * (x + 1) / 8;
    const int64_t npass = (t1 - t0 + (int64_t)NW * nrank - 1) / ((int64_t)NW * nrank);
    __syncthreads();
    // a pass's row: tile t = t0 + (ps nrank + rank) NW + wave, slot j (past the end: a valid row,
    // nothing written); the index loads for the next pass are issued a pass ahead
    struct Ctx {
        int64_t rr;
        bool ok;
        int ty;
        const float *pv, *pc;
        float lv;
    };
    auto ctx_of = [&](int64_t ps) {
        Ctx c;
        const int64_t t = t0 + (ps * nrank + rank) * NW + wave, r = t * 32 + j;
        c.ok = t < t1 && r < A.R;
        c.rr = c.ok ? r : A.R - 1;
        const int64_t b = c.rr / A.E, m = c.rr - b * A.E;
        c.ty = A.msg_type[m];
        c.pv = A.Pv + (b * A.Gv + A.vgroup[m]) * H + 4 * h;
        c.pc = A.Pc + (b * A.Gc + A.cgroup[m]) * H + 4 * h;
        c.lv = L0 ? A.llr[b * A.N + A.msg_var[m]] : 0.0f;
        return c;
    };
    // x in GEMM1's B operand order: x[s][e] = unit pi16(16 s + 8 h + e)
    float xv[KS][8];
    auto load_x = [&](const Ctx &c) {
        const float *xr = A.x_in + c.rr * H + 4 * h;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const float4 v = *reinterpret_cast<const float4 *>(xr + 32 * (s >> 1) + 16 * (s & 1) + 8 * q);
                xv[s][4 * q] = v.x; xv[s][4 * q + 1] = v.y; xv[s][4 * q + 2] = v.z; xv[s][4 * q + 3] = v.w;
            }
    };
    Ctx cur = ctx_of(0);
    if (!L0 && npass > 0) load_x(cur);
    for (int64_t ps = 0; ps < npass; ++ps) {
        const Ctx nxt = ctx_of(ps + 1 < npass ? ps + 1 : ps);
        if (L0) {  // layer 0: x = Linear(1, H) of the message's LLR
#pragma unroll
            for (int s = 0; s < KS; ++s)
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int u = pi16(16 * s + 8 * h + e);
                    xv[s][e] = cur.lv * win[u] + bin[u];
                }
        }
        // y starts from b2v + b2c (+ x): register 4 q + i of tile ot is unit 32 ot + 8 q + 4 h + i
        f32x16w y[NT];
#pragma unroll
        for (int ot = 0; ot < NT; ++ot)
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    y[ot][4 * q + i] = (A.residual ? xv[2 * ot + (q >> 1)][4 * (q & 1) + i] : 0.0f) + b2[32 * ot + 8 * q + 4 * h + i];
        // c = x + emb[type] under the row's scale, split once for every slice
        const float *eb = embs + cur.ty * F::ES;
        float cm = 0.0f;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                xv[s][e] += eb[pi16(16 * s + 8 * h + e)];
                cm = fmaxf(cm, fabsf(xv[s][e]));
            }
        cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
        const int cexp = col_exp_w(cm, wexp1);
        const float csc = pow2f(cexp), asc = pow2f(cexp + wexp1), iasc = pow2f(-cexp - wexp1);
        f16x8_t c0[KS], c1[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
#pragma unroll
            for (int e = 0; e < 8; ++e) xv[s][e] *= csc;
            split2h(xv[s], c0[s], c1[s]);
        }
        int erun = 1 << 20, ys = 0;  // relu(h)'s running exponent (none yet); y holds y_true 2^ys
        // the slice's projected group row (its 32 hidden units), one slice ahead
        auto prow = [&](int sl, f32x16w &v) {
            const int side = sl / NT, tt = sl - side * NT;
            const float *pr = (side ? cur.pc : cur.pv) + 32 * tt;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 f = *reinterpret_cast<const float4 *>(pr + 8 * q);
                v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
            }
        };
        f32x16w pnext;
        prow(0, pnext);
        // A slice in two halves: GEMM1 -> relu(h)'s split (r0, r1), then GEMM2 + the ring's barrier.
        // Between them on the pass's last slice, c's registers are free and the next pass's x rows
        // are loaded into them (after the ring copy: the barrier's wait then leaves them in flight)
        auto gemm1 = [&](int sl, f16x8_t (&r0)[2], f16x8_t (&r1)[2]) {
            const int64_t k = ps * S + sl;  // slice counter over the whole walk: ring slot k & 1
            const _Float16 *img = reinterpret_cast<const _Float16 *>(slot(k));
            // GEMM1 starts from the slice's projected group row; the next slice's row is loaded
            // before the ring's copy is issued (waiting for it then does not wait for the copy)
            f32x16w hacc = pnext;
            if (sl + 1 < S) prow(sl + 1, pnext);
            // the next slice's image into the other ring slot by LDS-DMA, 1 KB per wave instruction
            if (k + 1 < npass * S) {
                const float4 *src = gimg + (int64_t)((sl + 1) % S) * NF4 + lane;
                const uint32_t dst = lds_base + (uint32_t)((k + 1) & 1) * F::BYTES;
#pragma unroll
                for (int c = 0; c < CP; ++c) {
                    const int q = c * NW + wv;  // this wave's 1-KB rounds
                    glds16(src + 64 * q, __builtin_amdgcn_readfirstlane(dst + 1024 * q));
                }
            }
            hacc *= asc;
            const _Float16 *w1 = img + j * F::R1 + 8 * h;
#pragma unroll
            for (int s = 0; s < KS; ++s) hacc = mfma3h(w1 + 16 * s, c0[s], c1[s], hacc, F::I1);
            float hm = 0.0f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                hacc[i] = relu_nan(hacc[i] * iasc);
                hm = fmaxf(hm, hacc[i]);
            }
            hm = fmaxf(hm, __shfl_xor(hm, 32, 64));
            // the running exponent moves down only; a zero slice leaves it (its split is exact anyway)
            const int e = col_exp_w(hm, wexp2);
            const int en = hm > 0.0f ? min(erun, e) : erun;
            if (en != erun) {
                const int d = en + wexp2 - ys;
#pragma unroll
                for (int ot = 0; ot < NT; ++ot)
#pragma unroll
                    for (int i = 0; i < 16; ++i) y[ot][i] = ldexpf(y[ot][i], d);
                ys = en + wexp2;
                erun = en;
            }
            const float hsc = pow2f(erun < (1 << 20) ? erun : 0);
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                float hr[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) hr[i] = hacc[8 * a + i] * hsc;
                split2h(hr, r0[a], r1[a]);
            }
        };
        // GEMM2: the slice's 32 columns of W2_side into every output tile, then the ring's barrier
        // (vmcnt: the loads issued after the ring copy may stay in flight)
        auto gemm2 = [&](int sl, const f16x8_t (&r0)[2], const f16x8_t (&r1)[2], bool xpre) {
            const _Float16 *img = reinterpret_cast<const _Float16 *>(slot(ps * S + sl));
            const _Float16 *w2 = img + F::W2OFF + j * F::R2 + 8 * h;
#pragma unroll
            for (int ot = 0; ot < NT; ++ot)
#pragma unroll
                for (int a = 0; a < 2; ++a) y[ot] = mfma3h(w2 + 32 * ot * F::R2 + 16 * a, r0[a], r1[a], y[ot], F::I2);
            if (xpre)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * KS) : "memory");  // the 2 KS x loads are the youngest
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's share of the next image landed
            __syncthreads();
        };
#pragma unroll 1
        for (int sl = 0; sl < S - 1; ++sl) {
            f16x8_t r0[2], r1[2];
            gemm1(sl, r0, r1);
            gemm2(sl, r0, r1, false);
        }
        {
            f16x8_t r0[2], r1[2];
            gemm1(S - 1, r0, r1);
            if (!L0) {  // (the last pass loads its own rows again: a valid address, discarded)
                __builtin_amdgcn_sched_barrier(0);  // the x loads stay after the ring copy's
                load_x(nxt);
                __builtin_amdgcn_sched_barrier(0);
            }
            gemm2(S - 1, r0, r1, !L0);
        }
        // y back to scale; write it (and the head on the last layer)
        float part = 0.0f;
#pragma unroll
        for (int ot = 0; ot < NT; ++ot)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int u = 32 * ot + 8 * q + 4 * h;
                float4 v = make_float4(ldexpf(y[ot][4 * q], -ys), ldexpf(y[ot][4 * q + 1], -ys),
                                       ldexpf(y[ot][4 * q + 2], -ys), ldexpf(y[ot][4 * q + 3], -ys));
                if (A.msg_out) {
                    part += v.x * wo[u]; part += v.y * wo[u + 1]; part += v.z * wo[u + 2]; part += v.w * wo[u + 3];
                } else if (cur.ok) {
                    *reinterpret_cast<float4 *>(A.y + cur.rr * H + u) = v;
                }
            }
        if (A.msg_out) {
            part += __shfl_xor(part, 32, 64);
            if (cur.ok && h == 0) A.msg_out[cur.rr] = part + bo;
        }
        cur = nxt;
    }
}

int g_wcus = 0;

template <int NT, int AH, bool F16>
int go_wgemm(const WArgs &a, int nslices, dim3 grid, size_t lds, hipStream_t s) {
    LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(gnn_wgemm_kernel<NT, AH, F16>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((gnn_wgemm_kernel<NT, AH, F16>), grid, dim3(kWThreads), lds, s, a, nslices);
    return LDPC_OK;
}

template <bool F16>
int go_wgemm_nt(const WArgs &a, int nslices, dim3 grid, size_t lds, hipStream_t s, bool ah4) {
    if (a.NS == 128) return ah4 ? go_wgemm<4, 4, F16>(a, nslices, grid, lds, s) : go_wgemm<4, 2, F16>(a, nslices, grid, lds, s);
    if (a.NS == 64) return ah4 ? go_wgemm<2, 4, F16>(a, nslices, grid, lds, s) : go_wgemm<2, 2, F16>(a, nslices, grid, lds, s);
    return ah4 ? go_wgemm<1, 4, F16>(a, nslices, grid, lds, s) : go_wgemm<1, 2, F16>(a, nslices, grid, lds, s);
}

int launch_wgemm(WArgs a, bool f16, hipStream_t s) {
    if (!g_wcus) {
        int dev = 0;
        LDPC_HIP(hipGetDevice(&dev));
        LDPC_HIP(hipDeviceGetAttribute(&g_wcus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    if (a.R <= 0) return LDPC_OK;
    if (!f16) a.out_max = nullptr;
    // the widest output slice (4, 2 or 1 tiles of 32 units) whose split images fit the LDS
    const size_t extra = (a.mode == kGemm1 ? (size_t)(a.T + 2) * (a.H + 1) * 4 : 0) + 4 * 128 + 16;
    a.NS = 32;
    for (int nt : {4, 2}) {
        if (a.H % (32 * nt) == 0 && wgemm_img_bytes(32 * nt, a.K, f16) + extra <= 160 * 1024) {
            a.NS = 32 * nt;
            break;
        }
    }
    const size_t lds = wgemm_lds_bytes(a, f16);
    if (lds > 160 * 1024) return fail(LDPC_EUNSUPPORTED, "hidden_dim too wide for the MFMA row GEMM's LDS image");
    const int nslices = a.H / a.NS;
    const int per_cu = std::max(1, std::min(2, (int)((160 * 1024) / lds)));
    // blocks per XCD: a multiple of the slice count, about per_cu workgroups per CU
    const int per_x = std::max(nslices, (g_wcus / 8) * per_cu / nslices * nslices);
    if ((a.K / 16) % 2) return fail(LDPC_EUNSUPPORTED, "row GEMM reduction length must be a multiple of 32");
    const bool ah4 = (a.K / 16) % 4 == 0;
    const dim3 grid(8 * per_x);
    if (int rc = f16 ? go_wgemm_nt<true>(a, nslices, grid, lds, s, ah4) : go_wgemm_nt<false>(a, nslices, grid, lds, s, ah4))
        return rc;
    LDPC_CHECK_LAUNCH("gnn_wgemm_kernel");
    return LDPC_OK;
}

template <int H>
int launch_wide_mlp(const WMlp &a, hipStream_t s) {
    const size_t lds = wide_mlp_lds_bytes<H>(a.T);
    if (lds > 160 * 1024) return fail(LDPC_EUNSUPPORTED, "too many message types for the fused wide MLP's LDS image");
    const void *fn = a.x_in ? reinterpret_cast<const void *>(gnn_wide_mlp_kernel<H, false>)
                            : reinterpret_cast<const void *>(gnn_wide_mlp_kernel<H, true>);
    LDPC_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    // one workgroup per CU, a multiple of the eight XCDs
    const int64_t tiles = (a.R + 31) / 32;
    const int per_x = (int)std::max<int64_t>(1, std::min<int64_t>(g_wcus / 8, (tiles + 8 * WFused<H>::NW - 1) / (8 * WFused<H>::NW)));
    if (a.x_in)
        hipLaunchKernelGGL((gnn_wide_mlp_kernel<H, false>), dim3(8 * per_x), dim3(WFused<H>::NTH), lds, s, a);
    else
        hipLaunchKernelGGL((gnn_wide_mlp_kernel<H, true>), dim3(8 * per_x), dim3(WFused<H>::NTH), lds, s, a);
    LDPC_CHECK_LAUNCH("gnn_wide_mlp_kernel");
    return LDPC_OK;
}

// LDPC_GNN_WIDE_GM_V=1 / 2 / 4: float4 per lane in the group means (A/B); default LDPC_WIDE_GM_V
#ifndef LDPC_WIDE_GM_V
#define LDPC_WIDE_GM_V 2
#endif
int gm_v() {
    static const int v = [] {
        const char *e = std::getenv("LDPC_GNN_WIDE_GM_V");
        const int x = e ? std::atoi(e) : LDPC_WIDE_GM_V;
        return x == 1 || x == 4 ? x : 2;
    }();
    return v;
}

}  // namespace

bool gnn_wide_supported(int H) { return H != 64 && H % 32 == 0 && H >= 96 && H <= 256; }

// LDPC_GNN_WIDE_FUSED=0: the row-GEMM sequence at H = 96 / 128 too (A/B)
// LDPC_GNN_WIDE_FUSED_MAX=n: the fused MLP up to H = n (96, 128, 160 or 192; default 192)
int fused_max_h() {
    static const int v = [] {
        const char *e = std::getenv("LDPC_GNN_WIDE_FUSED_MAX");
        return e ? std::atoi(e) : 192;
    }();
    return v;
}

int64_t gnn_wide_fused_bytes(int H, int layers) {
    static const bool on = [] {
        const char *e = std::getenv("LDPC_GNN_WIDE_FUSED");
        return !e || std::atoi(e) != 0;
    }();
    if (!on || H > fused_max_h()) return 0;
    switch (H) {
        case 96: return (int64_t)layers * WFused<96>::S * WFused<96>::BYTES;
        case 128: return (int64_t)layers * WFused<128>::S * WFused<128>::BYTES;
        case 160: return (int64_t)layers * WFused<160>::S * WFused<160>::BYTES;
        case 192: return (int64_t)layers * WFused<192>::S * WFused<192>::BYTES;
        default: return 0;
    }
}

bool gnn_wide_fused_fits(int H, int T) {
    switch (H) {
        case 96: return wide_mlp_lds_bytes<96>(T) <= 160 * 1024;
        case 128: return wide_mlp_lds_bytes<128>(T) <= 160 * 1024;
        case 160: return wide_mlp_lds_bytes<160>(T) <= 160 * 1024;
        case 192: return wide_mlp_lds_bytes<192>(T) <= 160 * 1024;
        default: return false;
    }
}

template <int H>
void go_prep(int layers, const float *blob, int64_t layer_floats, int T, char *wimg, int *wexp, hipStream_t s) {
    hipLaunchKernelGGL(gnn_wide_prep_kernel<H>, dim3(layers), dim3(1024), 0, s, blob, layer_floats, T, wimg, wexp);
}

int gnn_wide_memb(const ldpc_gnn_plan *p, int H, int layers, const float *emb0, int64_t layer_stride,
                  const int32_t *msg_type, float *memb, hipStream_t s) {
    const int64_t n = (int64_t)layers * (p->Gv + p->Gc) * H;
    hipLaunchKernelGGL(gnn_wide_memb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, emb0, layer_stride, H,
                       msg_type, p->vg_ptr, p->vg_mem, p->inv_v, p->cg_ptr, p->cg_mem, p->inv_c, p->Gv, p->Gc, layers, memb);
    LDPC_CHECK_LAUNCH("gnn_wide_memb_kernel");
    return LDPC_OK;
}

int gnn_wide_prep(int H, int layers, const float *blob, int64_t layer_floats, int T, char *wimg, int *wexp, hipStream_t s) {
    switch (H) {
        case 96: go_prep<96>(layers, blob, layer_floats, T, wimg, wexp, s); break;
        case 128: go_prep<128>(layers, blob, layer_floats, T, wimg, wexp, s); break;
        case 160: go_prep<160>(layers, blob, layer_floats, T, wimg, wexp, s); break;
        case 192: go_prep<192>(layers, blob, layer_floats, T, wimg, wexp, s); break;
        default: return fail(LDPC_EINVAL, "fused wide MLP: H must be 96, 128, 160 or 192");
    }
    LDPC_CHECK_LAUNCH("gnn_wide_prep_kernel");
    return LDPC_OK;
}

int gnn_wide_layer(const GnnWideLayer &L, hipStream_t s) {
    const int H = L.H;
    const int64_t BE = L.B * L.E;
    // group means (every group: the H = 64 path's degree-1 shortcut is not taken here)
    {
        WGm g{};
        g.x = L.x_in;
        g.llr = L.llr; g.w_in = L.w_in; g.b_in = L.b_in; g.emb = L.emb;
        g.msg_type = L.msg_type; g.msg_var = L.msg_var;
        g.meta = L.plan->gt_meta; g.grp = L.plan->gt_grp; g.mem = L.plan->gt_mem; g.n_tiles = L.plan->n_gtiles;
        g.inv_v = L.plan->inv_v; g.inv_c = L.plan->inv_c;
        g.Mv = L.Mv; g.Mc = L.Mc;
        g.gmax_v = L.f16 ? L.gmax_v : nullptr;
        g.gmax_c = L.f16 ? L.gmax_c : nullptr;
        g.memb = L.memb;
        g.Gv = L.plan->Gv; g.Gc = L.plan->Gc; g.H = H; g.N = L.N;
        // groups per wave: a power of two dividing a tile's 8 that fits the wave's 64 lanes
        const int v2 = gm_v();
        const int lg = H / (4 * v2);
        g.gpw = 1;
        while (g.gpw * 2 <= 8 && g.gpw * 2 * lg <= 64) g.gpw *= 2;
        g.E = L.E; g.B = L.B;
        const int64_t waves = L.B * (int64_t)g.n_tiles * (8 / g.gpw);
        const dim3 grid((unsigned)((waves + 3) / 4));
        if (v2 == 4)
            hipLaunchKernelGGL(gnn_wide_gm_kernel<4>, grid, dim3(256), 0, s, g);
        else if (v2 == 2)
            hipLaunchKernelGGL(gnn_wide_gm_kernel<2>, grid, dim3(256), 0, s, g);
        else
            hipLaunchKernelGGL(gnn_wide_gm_kernel<1>, grid, dim3(256), 0, s, g);
        LDPC_CHECK_LAUNCH("gnn_wide_gm_kernel");
    }
    WArgs base{};
    base.H = H;
    base.emb = L.emb; base.msg_type = L.msg_type; base.msg_var = L.msg_var;
    base.llr = L.llr; base.w_in = L.w_in; base.b_in = L.b_in; base.N = L.N; base.T = L.T; base.E = L.E;
    // projections P_s = W1_s,right g + b1_s
    for (int side = 0; side < 2; ++side) {
        WArgs a = base;
        a.mode = kProj;
        a.K = H;
        a.R = L.B * (side ? L.plan->Gc : L.plan->Gv);
        a.in = side ? L.Mc : L.Mv;
        a.in_stride = H;
        a.w_a = side ? L.w1c : L.w1v;
        a.ld = 2 * H;
        a.col0 = H;
        a.init_a = side ? L.b1c : L.b1v;
        a.out = side ? L.Pc : L.Pv;
        a.out_stride = H;
        a.in_max = side ? L.gmax_c : L.gmax_v;
        if (int rc = launch_wgemm(a, L.f16, s)) return rc;
    }
    if (L.wimg) {  // H = 96 / 128: GEMM1 -> GEMM2 (-> head) fused per tile
        if (!g_wcus) {
            int dev = 0;
            LDPC_HIP(hipGetDevice(&dev));
            LDPC_HIP(hipDeviceGetAttribute(&g_wcus, hipDeviceAttributeMultiprocessorCount, dev));
        }
        WMlp a{};
        a.wimg = L.wimg; a.wexp = L.wexp;
        a.x_in = L.x_in; a.llr = L.llr; a.w_in = L.w_in; a.b_in = L.b_in; a.emb = L.emb;
        a.msg_type = L.msg_type; a.msg_var = L.msg_var; a.vgroup = L.plan->vgroup; a.cgroup = L.plan->cgroup;
        a.Pv = L.Pv; a.Pc = L.Pc;
        a.b2v = L.b2v; a.b2c = L.b2c; a.wo = L.wo; a.bo = L.bo;
        a.y = L.y; a.msg_out = L.msg_out;
        a.residual = L.residual; a.N = L.N; a.T = L.T; a.Gv = L.plan->Gv; a.Gc = L.plan->Gc;
        a.E = L.E; a.R = BE;
        switch (H) {
            case 96: return launch_wide_mlp<96>(a, s);
            case 128: return launch_wide_mlp<128>(a, s);
            case 160: return launch_wide_mlp<160>(a, s);
            default: return launch_wide_mlp<192>(a, s);
        }
    }
    // h_s = relu(W1_s,left c + P_s[group]) into h (B E, 2 H); both sides' row maxima into hmax
    if (L.f16) LDPC_HIP(hipMemsetAsync(L.hmax, 0, (size_t)BE * 4, s));
    for (int side = 0; side < 2; ++side) {
        WArgs a = base;
        a.mode = kGemm1;
        a.K = H;
        a.R = BE;
        a.in = L.x_in;
        a.in_stride = H;
        a.w_a = side ? L.w1c : L.w1v;
        a.ld = 2 * H;
        a.col0 = 0;
        a.init_a = side ? L.Pc : L.Pv;
        a.grp = side ? L.plan->cgroup : L.plan->vgroup;
        a.G = side ? L.plan->Gc : L.plan->Gv;
        a.out = L.hbuf + side * H;
        a.out_stride = 2 * H;
        a.in_max = L.xmax_in;
        a.out_max = L.hmax;
        if (int rc = launch_wgemm(a, L.f16, s)) return rc;
    }
    // y = W2_v h_v + W2_c h_c + (b2_v + b2_c) (+ x): the reference's MLP_v + MLP_c (+ residual)
    {
        WArgs a = base;
        a.mode = kGemm2;
        a.K = 2 * H;
        a.R = BE;
        a.in = L.hbuf;
        a.in_stride = 2 * H;
        a.w_a = L.w2v;
        a.w_b = L.w2c;
        a.init_a = L.b2v;
        a.init_b = L.b2c;
        a.resid = L.residual ? L.x_in : nullptr;
        a.out = L.y;
        a.out_stride = H;
        a.in_max = L.hmax;
        a.out_max = L.msg_out ? nullptr : L.xmax_out;  // the last layer's rows go to the head only
        if (L.f16 && a.out_max) LDPC_HIP(hipMemsetAsync(a.out_max, 0, (size_t)BE * 4, s));
        if (int rc = launch_wgemm(a, L.f16, s)) return rc;
    }
    if (L.msg_out) {
        hipLaunchKernelGGL(gnn_wide_head_kernel, dim3((unsigned)((BE * 16 + 255) / 256)), dim3(256), 0, s, L.y, H, BE,
                           L.wo, L.bo, L.msg_out);
        LDPC_CHECK_LAUNCH("gnn_wide_head_kernel");
    }
    return LDPC_OK;
}

}  // namespace ldpc
