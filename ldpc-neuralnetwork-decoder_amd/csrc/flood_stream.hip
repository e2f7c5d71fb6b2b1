// flood_stream.hip -- the streaming flooding decoders (every message in HBM, any graph) and the hybrid
// min-sum decoder on the same layout.  Split out of flood.hip (see flood.hip for the overview).
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "flood_host.hpp"

namespace ldpc {

// ---------------------------------------------------------------- streaming decoder (any graph)
// For graphs whose messages do not fit a CU's LDS (lifting sizes that do not divide 64 leave the
// QC detection at Z = 1; large Z; big non-QC codes): the same flooding iteration with every
// message in HBM, laid out edge-major and frame-fastest (msg[e][b]), so that the 64 lanes of a
// wave -- 64 consecutive frames of one row / column -- load and store 256 contiguous bytes.  One
// launch per phase; each thread owns one (check, frame) or (variable, frame).  The float32
// operation sequences are the LDS kernels' (= the reference's), so results are bit-identical
// (min-sum) / identical (BP) across the two paths.  Early stop keeps the reference's rules with
// device flags: a finished batch (LDPC_ES_BATCH) or frame (LDPC_ES_FRAME) skips the later launches.
struct StreamArgs {
    const int32_t *chk_ptr, *ev, *var_ptr, *var_edge;
    int M, N;
    int64_t E, B;
    float *msg;        // [E][B] v2c / c2v in place
    float *llrT;       // [N][B]
    uint8_t *bitsT;    // [N][B] hard decisions of the latest iteration
    uint8_t *done;     // [B] LDPC_ES_FRAME: frame frozen
    int32_t *iters;    // [B] LDPC_ES_FRAME: iterations of a frozen frame
    int32_t *ctl;      // [0] batch stopped  [1] batch iterations
    int32_t *invalid;  // [max_iter] LDPC_ES_BATCH: frames failing H x = 0 after each iteration
    float alpha;
    int es;
    // flooding decoders only (null for the hybrid min-sum): per edge, its variable when that has
    // degree 1.  Such an edge's v2c is the channel LLR forever, so the check phase leaves it in
    // place and takes the variable's decision itself (APP = llr + c2v = v2c + c2v, the same
    // float add); the degree-1 variables get no variable-phase launch.
    const int32_t *ext_var;
};

__device__ __forceinline__ bool stream_skip(const StreamArgs &S, int64_t b) {
    if (S.es == LDPC_ES_BATCH) return S.ctl[0] != 0;
    if (S.es == LDPC_ES_FRAME) return S.done[b] != 0;
    return false;
}

// (B, N) -> (N, B) through 64 x 64 LDS tiles
__global__ __launch_bounds__(256) void stream_transpose_llr_kernel(const float *__restrict__ llr, int64_t B, int N,
                                                                   float *__restrict__ llrT) {
    __shared__ float t[64][65];
    const int64_t b0 = (int64_t)blockIdx.x * 64;
    const int v0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4)
        if (b0 + r < B && v0 + tx < N) t[r][tx] = llr[(b0 + r) * N + v0 + tx];
    __syncthreads();
    for (int r = ty; r < 64; r += 4)
        if (v0 + r < N && b0 + tx < B) llrT[(int64_t)(v0 + r) * B + b0 + tx] = t[tx][r];
}


// one (check, frame): the row's DC messages in registers (DC is the row's degree, uniform over a
// wave of 64 consecutive frames of one row)
// FIRST: the first iteration of a flooding decode reads v2c = LLR straight from llrT (no init pass
// over the E x B messages) and seeds the degree-1 edges' messages with it
template <int ALGO, int DC, bool FIRST = false>
__device__ __forceinline__ void stream_row(const StreamArgs &S, float *m, int e0) {
    float v[DC];
#pragma unroll
    for (int e = 0; e < DC; ++e) {
        if constexpr (FIRST)
            v[e] = S.llrT[(int64_t)S.ev[e0 + e] * S.B + (m - S.msg)];
        else
            v[e] = m[(int64_t)(e0 + e) * S.B];
    }
    float out[DC];
    if constexpr (ALGO == LDPC_ALGO_MINSUM) {
        // the LDS kernels' fast path (two minima by v_min / v_med3, sign parity by xor) when the
        // row has no zero and no NaN message; else MinSumStats (exact torch.sign semantics)
        const float ninf = opaque_sf(-INFINITY);
        float m1 = fabsf(v[0]), m2 = opaque_sf(INFINITY);
        bool special = is_zero_sign(v[0]);
#pragma unroll
        for (int e = 1; e < DC; ++e) {
            two_min_step(m1, m2, v[e], ninf);
            special |= is_zero_sign(v[e]);
        }
        if (!special) {
            const uint32_t par = sign_parity_n<DC>(v) & 0x80000000u;
            const uint32_t s1 = __float_as_uint(S.alpha * m1) ^ par, s2 = __float_as_uint(S.alpha * m2) ^ par;
#pragma unroll
            for (int e = 0; e < DC; ++e)
                out[e] = __uint_as_float((__float_as_uint(v[e]) & 0x80000000u) ^ (fabsf(v[e]) == m1 ? s2 : s1));
        } else {
            MinSumStats st;
#pragma unroll
            for (int e = 0; e < DC; ++e) st.add(e, v[e]);
#pragma unroll
            for (int e = 0; e < DC; ++e) out[e] = st.c2v(e, v[e], S.alpha);
        }
    } else {
        // c2v_e = 2 atanh(prod_{f != e} tanh(v_f / 2)), product from 1.0 ascending (:72-81):
        // acc[e] = P_e * t_{e+1} * ... built column by column, as the LDS kernels do
        float acc[DC];
        float P = 1.0f;
#pragma unroll
        for (int j = 0; j < DC; ++j) {
            const float t = tanh_half(v[j]);
#pragma unroll
            for (int e = 0; e < j; ++e) acc[e] = acc[e] * t;
            acc[j] = P;
            P = P * t;
        }
#pragma unroll
        for (int e = 0; e < DC; ++e) out[e] = two_atanh(acc[e]);
    }
#pragma unroll
    for (int e = 0; e < DC; ++e) {
        const int xv = S.ext_var ? S.ext_var[e0 + e] : -1;  // wave-uniform (scalar load)
        if (xv < 0) {
            m[(int64_t)(e0 + e) * S.B] = out[e];
        } else {  // m - msg = the frame b: bitsT[xv][b]
            if constexpr (FIRST) m[(int64_t)(e0 + e) * S.B] = v[e];
            S.bitsT[(int64_t)xv * S.B + (m - S.msg)] = v[e] + out[e] < 0.0f;
        }
    }
}

#define LDPC_STREAM_DEG_CASES(X)                                                                       \
    X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) \
    X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32)

// one launch per check degree DC (graph.cpp groups the checks by degree): thread = (k-th check of
// the degree, frame), the frame fastest, so a wave is 64 frames of one check (coalesced rows)
template <int ALGO, int DC, bool FIRST>
__global__ __launch_bounds__(256) void stream_check_kernel(StreamArgs S, const int32_t *__restrict__ rows) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // grid: (frames, checks)
    if (b >= S.B || stream_skip(S, b)) return;
    stream_row<ALGO, DC, FIRST>(S, S.msg + b, S.chk_ptr[rows[blockIdx.y]]);
}

// one (variable, frame): v2c_e = llr + sum_{e' != e} c_e' in ascending check order as the prefix
// P_e followed by the tail adds (traditional_decoders.py:235-250); APP = P_DV -> decision
template <int DV>
__device__ __forceinline__ float stream_col(const StreamArgs &S, float *m, const int32_t *edges, float l, bool write) {
    float c[DV];
    int32_t ed[DV];  // edge ids (the 64-bit offsets are recomputed at the store: fewer live VGPRs)
#pragma unroll
    for (int p = 0; p < DV; ++p) {
        ed[p] = edges[p];
        c[p] = m[(int64_t)ed[p] * S.B];
    }
    f32x2 acc[(DV + 1) / 2];
    float P = l;
#pragma unroll
    for (int j = 0; j < DV; ++j) {
        const f32x2 cc = {c[j], c[j]};
#pragma unroll
        for (int p = 0; p < j / 2; ++p) acc[p] = acc[p] + cc;
        if (j % 2 == 1) {
            acc[j / 2].x = acc[j / 2].x + c[j];
            acc[j / 2].y = P;
        } else {
            acc[j / 2].x = P;
        }
        P = P + c[j];
    }
    if (write) {
#pragma unroll
        for (int p = 0; p < DV; ++p) m[(int64_t)ed[p] * S.B] = p % 2 == 0 ? acc[p / 2].x : acc[p / 2].y;
    }
    return P;
}

// one launch per variable degree DV (0 included: APP = llr)
template <int DV>
__global__ __launch_bounds__(256) void stream_var_kernel(StreamArgs S, const int32_t *__restrict__ cols, int write) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // grid: (frames, variables)
    if (b >= S.B || stream_skip(S, b)) return;
    const int j = cols[blockIdx.y];
    const int64_t jb = (int64_t)j * S.B + b;
    const float l = S.llrT[jb];
    float app = l;
    if constexpr (DV > 0) app = stream_col<DV>(S, S.msg + b, S.var_edge + S.var_ptr[j], l, write != 0);
    S.bitsT[jb] = app < 0.0f;  // NaN < 0 is false -> 0
}

// per-frame syndrome after an iteration: LDPC_ES_FRAME freezes valid frames, LDPC_ES_BATCH
// counts the invalid ones for stream_batch_step_kernel
__global__ __launch_bounds__(256) void stream_syndrome_kernel(StreamArgs S, int it) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int bad = 0;
    if (b < S.B && !stream_skip(S, b)) {
        for (int i = 0; i < S.M && !bad; ++i) {
            int p = 0;
            for (int e = S.chk_ptr[i]; e < S.chk_ptr[i + 1]; ++e) p ^= S.bitsT[(int64_t)S.ev[e] * S.B + b];
            bad = p;
        }
        if (S.es == LDPC_ES_FRAME && !bad) {
            S.done[b] = 1;
            S.iters[b] = it + 1;
        }
    } else {
        bad = 0;
    }
    if (S.es == LDPC_ES_BATCH) {
        const uint64_t m = __ballot(bad);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(&S.invalid[it], (int)__popcll(m));
    }
}

__global__ void stream_batch_step_kernel(StreamArgs S, int it) {
    if (S.ctl[0] == 0 && S.invalid[it] == 0) {  // every frame valid: the reference returns (:104-107)
        S.ctl[0] = 1;
        S.ctl[1] = it + 1;
    }
}

// (N, B) decisions -> (B, N) output bits, per-frame iteration counts and counter rows
__global__ __launch_bounds__(256) void stream_emit_kernel(StreamArgs S, int max_iter, int out_dtype, void *bits,
                                                          int32_t *iters_out, uint32_t *partials) {
    __shared__ uint8_t tile[64][65];
    __shared__ uint32_t errs[64];
    const int64_t b0 = (int64_t)blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    if (threadIdx.x < 64) errs[threadIdx.x] = 0;
    for (int v0 = 0; v0 < S.N; v0 += 64) {
        __syncthreads();
        for (int r = ty; r < 64; r += 4)
            tile[r][tx] = (v0 + r < S.N && b0 + tx < S.B) ? S.bitsT[(int64_t)(v0 + r) * S.B + b0 + tx] : 0;
        __syncthreads();
        for (int r = ty; r < 64; r += 4) {
            const int64_t b = b0 + r;
            if (b < S.B && v0 + tx < S.N) {
                const int bit = tile[tx][r];
                put_bit(bits, out_dtype, b * S.N + v0 + tx, bit);
                if (bit) atomicAdd(&errs[r], 1u);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const int64_t b = b0 + threadIdx.x;
        uint32_t be = 0, fe = 0, fr = 0, it = 0;
        if (b < S.B) {
            int n = max_iter;
            if (S.es == LDPC_ES_BATCH && S.ctl[0]) n = S.ctl[1];
            if (S.es == LDPC_ES_FRAME && S.done[b]) n = S.iters[b];
            if (iters_out) iters_out[b] = n;
            be = errs[threadIdx.x];
            fe = be > 0;
            fr = 1;
            it = (uint32_t)n;
        }
        uint32_t mx = it;
        for (int off = 32; off > 0; off >>= 1) {
            be += __shfl_xor(be, off, 64);
            fe += __shfl_xor(fe, off, 64);
            fr += __shfl_xor(fr, off, 64);
            it += __shfl_xor(it, off, 64);
            mx = max(mx, (uint32_t)__shfl_xor(mx, off, 64));
        }
        if (threadIdx.x == 0 && partials) {
            uint32_t *row = partials + (int64_t)blockIdx.x * kPartRow;
            row[0] = be;
            row[1] = fe;
            row[2] = fr;
            row[3] = it;
            row[4] = mx;
        }
    }
}

// ---------------------------------------------------------------- hybrid min-sum (CustomMinSum*)
// CustomMinSumMessageGNNDecoder (message_gnn_decoder.py:1137-1251) cannot run in the reference
// (MGD:1270 TypeError; its variable / check updates index per-node tensors as if
// they were per-message, MGD:636-657 / :999-1038).  This build defines the decoder by the updates those
// loops spell out, per edge m = (check c, variable v), one frame at a time, c2v = 0 at the start:
//   S_v     = sum of c2v over v's edges, ascending message order               (MGD:650 / :1231)
//   v2c_m   = (llr_v + S_v) - c2v_m                       "total minus own"     (MGD:650-654)
//   v2c_m   = 0.5 v2c_m + 0.5 c2v_m    from the second iteration on (damping)  (MGD:659-663)
//   c2v_m   = prod_{m' != m} sign(v2c_m') * min_{m' != m} |v2c_m'|  (unscaled; the learnable
//             alpha of MGD:974 is never used by the update, MGD:1009-1032)       (MGD:1006-1038)
//   probs_v = sigmoid(llr_v + S_v) after the last iteration                     (MGD:1222-1240)
// Same streaming layout as above (msg[e][b]); the check phase is stream_check_kernel<MINSUM> with
// alpha = 1 (exact: 1 * min = min).  Oracle: oracle/ldpc_oracle.c ldpc_oracle_custom_minsum.
template <int DV>
__device__ __forceinline__ void custom_col(const StreamArgs &S, float *m, const int32_t *edges, float l, bool damp) {
    float c[DV];
    int32_t ed[DV];  // edge ids (the 64-bit offsets are recomputed at the store: fewer live VGPRs)
#pragma unroll
    for (int p = 0; p < DV; ++p) {
        ed[p] = edges[p];
        c[p] = m[(int64_t)ed[p] * S.B];
    }
    float sum = c[0];
#pragma unroll
    for (int p = 1; p < DV; ++p) sum = sum + c[p];
    const float total = l + sum;
#pragma unroll
    for (int p = 0; p < DV; ++p) {
        float v = total - c[p];
        if (damp) v = 0.5f * v + 0.5f * c[p];
        m[(int64_t)ed[p] * S.B] = v;
    }
}

// one launch per variable degree >= 1 (a variable without edges sends nothing)
// FIRST (iteration 0, every c2v = +0): v2c = (llr + (+0 + ... + +0)) - (+0) = llr + 0.0f exactly
// (the + 0.0f turns a -0 LLR into +0 as the full sum does), so nothing is read and the messages
// need no zero-fill
template <int DV, bool FIRST>
__global__ __launch_bounds__(256) void custom_var_kernel(StreamArgs S, const int32_t *__restrict__ cols, int damp) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // grid: (frames, variables)
    if (b >= S.B) return;
    const int j = cols[blockIdx.y];
    const float l = S.llrT[(int64_t)j * S.B + b];
    if constexpr (FIRST) {
        const int32_t *edges = S.var_edge + S.var_ptr[j];
        const float v = l + 0.0f;
#pragma unroll
        for (int p = 0; p < DV; ++p) S.msg[(int64_t)edges[p] * S.B + b] = v;
    } else {
        custom_col<DV>(S, S.msg + b, S.var_edge + S.var_ptr[j], l, damp != 0);
    }
}

// probsT[v][b] = sigmoid(llr_v + S_v), S_v in ascending message order
__global__ __launch_bounds__(256) void custom_output_kernel(StreamArgs S, float *__restrict__ probsT) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)S.N * S.B) return;
    const int64_t j = t / S.B, b = t - j * S.B;
    const int p0 = S.var_ptr[j], p1 = S.var_ptr[j + 1];
    float out = S.llrT[t];
    if (p1 > p0) {
        float sum = S.msg[(int64_t)S.var_edge[p0] * S.B + b];
        for (int p = p0 + 1; p < p1; ++p) sum = sum + S.msg[(int64_t)S.var_edge[p] * S.B + b];
        out = out + sum;
    }
    probsT[t] = 1.0f / (1.0f + expf(-out));
}


namespace {
struct StreamWs {
    float *msg, *llrT;
    uint8_t *bitsT, *done;
    int32_t *iters, *ctl, *invalid;
    uint32_t *partials;
    int64_t bytes;
};

StreamWs stream_ws(const ldpc_graph *g, int64_t B, int max_iter, void *base) {
    StreamWs w{};
    char *p = static_cast<char *>(base);
    size_t off = 0;
    auto take = [&](size_t n) { char *q = p ? p + off : nullptr; off += align256(n); return q; };
    w.msg = reinterpret_cast<float *>(take((size_t)g->E * B * 4));
    w.llrT = reinterpret_cast<float *>(take((size_t)g->N * B * 4));
    w.bitsT = reinterpret_cast<uint8_t *>(take((size_t)g->N * B));
    w.done = reinterpret_cast<uint8_t *>(take((size_t)B));
    w.iters = reinterpret_cast<int32_t *>(take((size_t)B * 4));
    w.ctl = reinterpret_cast<int32_t *>(take(64));
    w.invalid = reinterpret_cast<int32_t *>(take((size_t)max_iter * 4));
    w.partials = reinterpret_cast<uint32_t *>(take((size_t)((B + 63) / 64) * kPartRow * 4));
    w.bytes = (int64_t)off;
    return w;
}

// one launch per node degree (graph.cpp groups the checks / variables by degree), on a 2-D grid
// (frames, nodes) so a thread finds its (node, frame) without a 64-bit division; grid.y is
// chunked to 65535 nodes
constexpr int kGridY = 65535;
template <class F>
void per_degree(const std::vector<int> &seg, const int32_t *order, int64_t B, F &&launch) {
    const unsigned gx = (unsigned)((B + 255) / 256);
    for (size_t q = 0; q + 2 < seg.size(); q += 3)
        for (int k0 = 0; k0 < seg[q + 2]; k0 += kGridY)
            launch(seg[q], dim3(gx, (unsigned)std::min(kGridY, seg[q + 2] - k0)), order + seg[q + 1] + k0);
}

template <int ALGO, bool FIRST = false>
void launch_stream_check(const ldpc_graph *g, const StreamArgs &S, int64_t B, hipStream_t s) {
    per_degree(g->row_seg, g->row_order, B, [&](int d, dim3 grid, const int32_t *rows) {
        switch (d) {  // degree 0: no messages; degrees above 32 are refused on the host
#define X(k) case k: hipLaunchKernelGGL((stream_check_kernel<ALGO, k, FIRST>), grid, dim3(256), 0, s, S, rows); break;
            LDPC_STREAM_DEG_CASES(X)
#undef X
            default: break;
        }
    });
}

void launch_stream_var(const ldpc_graph *g, const StreamArgs &S, int64_t B, int write, hipStream_t s) {
    per_degree(g->col_seg, g->col_order, B, [&](int d, dim3 grid, const int32_t *cols) {
        if (d == 1 && S.ext_var) return;  // degree-1 variables: handled by the check phase
        switch (d) {
#define X(k) case k: hipLaunchKernelGGL(stream_var_kernel<k>, grid, dim3(256), 0, s, S, cols, write); break;
            X(0) LDPC_STREAM_DEG_CASES(X)
#undef X
            default: break;
        }
    });
}

template <bool FIRST>
void launch_custom_var(const ldpc_graph *g, const StreamArgs &S, int64_t B, int damp, hipStream_t s) {
    per_degree(g->col_seg, g->col_order, B, [&](int d, dim3 grid, const int32_t *cols) {
        switch (d) {  // a variable without edges sends nothing
#define X(k) case k: hipLaunchKernelGGL((custom_var_kernel<k, FIRST>), grid, dim3(256), 0, s, S, cols, damp); break;
            LDPC_STREAM_DEG_CASES(X)
#undef X
            default: break;
        }
    });
}

template <int ALGO>
int run_stream(const ldpc_graph *g, const float *llr, int64_t B, int max_iter, float alpha, int es, int out_dtype,
               void *bits, int32_t *iters_out, uint64_t *counters, int32_t *batch_iters, void *work, hipStream_t s) {
    const StreamWs w = stream_ws(g, B, max_iter, work);
    StreamArgs S{g->chk_ptr, g->ev, g->var_ptr, g->var_edge, g->M, g->N, g->E, B, w.msg, w.llrT, w.bitsT, w.done,
                 w.iters, w.ctl, w.invalid, alpha, es, g->ext_var};
    LDPC_HIP(hipMemsetAsync(w.done, 0, (size_t)B, s));
    LDPC_HIP(hipMemsetAsync(w.ctl, 0, 64, s));
    LDPC_HIP(hipMemsetAsync(w.invalid, 0, (size_t)max_iter * 4, s));
    const dim3 tgrid((unsigned)((B + 63) / 64), (unsigned)((g->N + 63) / 64));
    hipLaunchKernelGGL(stream_transpose_llr_kernel, tgrid, dim3(256), 0, s, llr, B, g->N, w.llrT);
    auto blocks = [](int64_t n) { return dim3((unsigned)((n + 255) / 256)); };
    for (int it = 0; it < max_iter; ++it) {
        if (it == 0)  // v2c = LLR (traditional_decoders.py:199-202) read in place of an init pass
            launch_stream_check<ALGO, true>(g, S, B, s);
        else
            launch_stream_check<ALGO>(g, S, B, s);
        launch_stream_var(g, S, B, it < max_iter - 1 ? 1 : 0, s);
        if (es != LDPC_ES_OFF) {
            hipLaunchKernelGGL(stream_syndrome_kernel, blocks(B), dim3(256), 0, s, S, it);
            if (es == LDPC_ES_BATCH) hipLaunchKernelGGL(stream_batch_step_kernel, dim3(1), dim3(1), 0, s, S, it);
        }
        LDPC_CHECK_LAUNCH("stream iteration");
    }
    const bool want = counters || batch_iters;
    hipLaunchKernelGGL(stream_emit_kernel, dim3((unsigned)((B + 63) / 64)), dim3(256), 0, s, S, max_iter, out_dtype,
                       bits, iters_out, want ? w.partials : nullptr);
    LDPC_CHECK_LAUNCH("stream emit");
    if (!want) return LDPC_OK;
    // batch_iters: ES off was set before the launch; otherwise the largest per-frame count
    return reduce_counter_rows(w.partials, (B + 63) / 64, counters, es == LDPC_ES_OFF ? nullptr : batch_iters,
                               nullptr, s);
}

// CustomMinSum workspace: the streaming arrays (msg, llrT) + probsT [N][B]
int64_t custom_ws_bytes_(const ldpc_graph *g, int64_t B) {
    return (int64_t)(align256((size_t)g->E * B * 4) + 2 * align256((size_t)g->N * B * 4));
}

int run_custom_minsum_(const ldpc_graph *g, const float *llr, int64_t B, int iterations, float *probs, void *work,
                      hipStream_t s) {
    char *base = static_cast<char *>(work);
    StreamArgs S{};
    S.chk_ptr = g->chk_ptr; S.ev = g->ev; S.var_ptr = g->var_ptr; S.var_edge = g->var_edge;
    S.M = g->M; S.N = g->N; S.E = g->E; S.B = B;
    S.msg = reinterpret_cast<float *>(base);
    S.llrT = reinterpret_cast<float *>(base + align256((size_t)g->E * B * 4));
    float *probsT = reinterpret_cast<float *>(base + align256((size_t)g->E * B * 4) + align256((size_t)g->N * B * 4));
    S.alpha = 1.0f;
    S.es = LDPC_ES_OFF;
    // c2v = 0 at the start (MGD:1193): the first variable phase's FIRST form needs no zero-fill,
    // zero iterations read the zeros directly
    if (iterations == 0) LDPC_HIP(hipMemsetAsync(S.msg, 0, (size_t)g->E * B * 4, s));
    hipLaunchKernelGGL(stream_transpose_llr_kernel, dim3((unsigned)((B + 63) / 64), (unsigned)((g->N + 63) / 64)),
                       dim3(256), 0, s, llr, B, g->N, S.llrT);
    auto blocks = [](int64_t n) { return dim3((unsigned)((n + 255) / 256)); };
    for (int it = 0; it < iterations; ++it) {
        if (it == 0)
            launch_custom_var<true>(g, S, B, 0, s);
        else
            launch_custom_var<false>(g, S, B, 1, s);
        launch_stream_check<LDPC_ALGO_MINSUM>(g, S, B, s);
        LDPC_CHECK_LAUNCH("custom min-sum iteration");
    }
    hipLaunchKernelGGL(custom_output_kernel, blocks((int64_t)g->N * B), dim3(256), 0, s, S, probsT);
    // (N, B) -> (B, N): the transpose kernel with the roles of the two extents swapped
    hipLaunchKernelGGL(stream_transpose_llr_kernel, dim3((unsigned)((g->N + 63) / 64), (unsigned)((B + 63) / 64)),
                       dim3(256), 0, s, probsT, (int64_t)g->N, (int)B, probs);
    LDPC_CHECK_LAUNCH("custom min-sum output");
    return LDPC_OK;
}

}  // namespace

int64_t stream_ws_bytes(const ldpc_graph *g, int64_t B, int max_iter) { return stream_ws(g, B, max_iter, nullptr).bytes; }

int run_stream_decode(int algo, const ldpc_graph *g, const float *llr, int64_t B, int max_iter, float alpha, int es,
                      int out_dtype, void *bits, int32_t *iters_out, uint64_t *counters, int32_t *batch_iters,
                      void *work, hipStream_t s) {
    return algo == LDPC_ALGO_MINSUM
               ? run_stream<LDPC_ALGO_MINSUM>(g, llr, B, max_iter, alpha, es, out_dtype, bits, iters_out, counters,
                                              batch_iters, work, s)
               : run_stream<LDPC_ALGO_BP>(g, llr, B, max_iter, alpha, es, out_dtype, bits, iters_out, counters,
                                          batch_iters, work, s);
}

int64_t custom_ws_bytes(const ldpc_graph *g, int64_t B) { return custom_ws_bytes_(g, B); }

int run_custom_minsum(const ldpc_graph *g, const float *llr, int64_t B, int iterations, float *probs, void *work,
                      hipStream_t s) {
    return run_custom_minsum_(g, llr, B, iterations, probs, work, s);
}

}  // namespace ldpc
