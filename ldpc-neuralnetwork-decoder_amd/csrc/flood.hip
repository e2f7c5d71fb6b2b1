// flood.hip -- LDS-resident flooding min-sum / sum-product decoder for gfx950.
//
// Replaces (bit-for-bit for min-sum, see DESIGN.md "Parity"):
//   MinSumScaledDecoder.decode     traditional_decoders.py:177-260
//   BeliefPropagationDecoder.decode traditional_decoders.py:42-109
//   _check_valid_codeword           traditional_decoders.py:111-134 / 262-285
//
// One workgroup = 4 waves = one "lane vector" of FG = 64/Z frames; every message of those frames
// lives in LDS for the whole decode (layout: graph.hpp).  HBM sees the LLRs once (plus L2 re-reads
// of degree-1 columns) and the decisions once.  Per iteration:
//   check phase  each wave takes whole block-rows (LPT schedule); a lane owns check r*Z+k of
//                frame f, keeps the row's <= 24 messages in registers, writes c2v in place
//   var phase    each wave takes whole columns; a lane owns variable c*Z+t, reads its dv c2v
//                (rotated slot index), writes v2c in place as the reference's ordered sums
//   [ES]         decisions as 64-bit ballots per column in LDS, syndrome per block-row
//
// Exactness: the reference sums/multiplies in float32 in a fixed order.  The var update is
// v2c_i = (((llr + c_0) + c_1) ...) over i' != i in ascending check order; we compute it as the
// prefix P_i followed by the same tail adds, i.e. the identical operation sequence.  Min-sum's
// sign/min is order-free.  BP's exclusive product is prefix-then-tail as well; tanh/atanh are
// float32 approximations of a few ulp (tanh_half / two_atanh below; the reference uses torch-CPU
// SLEEF float versions; neither is correctly rounded, so BP parity is "within float32
// tolerance", not bitwise).
// Compile with -ffp-contract=off: no a*b+c may fuse on this path.
// Translation units: flood_dev.hpp (device code shared by all), flood_fixed_ms.hip / flood_fixed_bp.hip
// (compile-time schedules), flood_stream.hip (streaming decoders),
// and this file (table-driven kernel, early-stop passes, host dispatch, the C ABI).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "flood_host.hpp"

namespace ldpc {

// ---------------------------------------------------------------- batch-global early stop
__global__ void es_init_kernel(int32_t *ctl, uint64_t *staged, uint32_t *all_words) {
    const int t = threadIdx.x;
    if (t < 4) ctl[t] = 0;
    if (t < 4) staged[t] = 0;
    if (t < 64) all_words[t] = ~0u;
}

// fold the per-workgroup counter rows: counters[0..3] += column sums, *batch_iters = max(it) when
// set_iters (ES_FRAME: the largest per-frame count; the fallback: tstar + 1).  gate: run only
// when *gate != 0 (NULL: always).  One workgroup of 1024 threads.
__global__ __launch_bounds__(1024) void counters_reduce_kernel(const uint32_t *__restrict__ partials, int64_t nwg,
                                                               uint64_t *counters, int32_t *batch_iters,
                                                               const int32_t *gate) {
    if (gate && *gate == 0) return;
    uint64_t acc[4] = {0, 0, 0, 0};
    uint32_t mx = 0;
    for (int64_t r = threadIdx.x; r < nwg; r += blockDim.x) {
        const uint32_t *row = partials + r * kPartRow;
        for (int i = 0; i < 4; ++i) acc[i] += row[i];
        mx = max(mx, row[4]);
    }
    for (int off = 32; off > 0; off >>= 1) {
        for (int i = 0; i < 4; ++i) acc[i] += __shfl_xor(acc[i], off, 64);
        mx = max(mx, (uint32_t)__shfl_xor(mx, off, 64));
    }
    __shared__ uint64_t sh[16][5];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        for (int i = 0; i < 4; ++i) sh[w][i] = acc[i];
        sh[w][4] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t[5] = {0, 0, 0, 0, 0};
        for (int q = 0; q < (int)(blockDim.x >> 6); ++q) {
            for (int i = 0; i < 4; ++i) t[i] += sh[q][i];
            t[4] = max(t[4], sh[q][4]);
        }
        if (counters)
            for (int i = 0; i < 4; ++i) counters[i] += t[i];
        if (batch_iters) *batch_iters = (int32_t)t[4];
    }
}

__global__ void es_finalize_kernel(int32_t *ctl, int max_iter, const uint64_t *staged, uint64_t *counters,
                                   int32_t *batch_iters, int force_fallback) {
    const int T = ctl[0];
    const int fallback = force_fallback || (ctl[1] != 0 && T < max_iter);
    ctl[2] = fallback;
    if (!fallback) {
        if (counters)
            for (int i = 0; i < 4; ++i) counters[i] += staged[i];
        if (batch_iters) *batch_iters = T;
    } else if (batch_iters) {
        *batch_iters = 0;  // batch_emit_kernel takes the max
    }
}

__global__ void batch_and_kernel(const uint32_t *__restrict__ ws_valid, int64_t B, int nvw,
                                 uint32_t *__restrict__ all_words, const int32_t *__restrict__ ctl) {
    if (ctl[2] == 0) return;
    __shared__ uint32_t sh[32];
    if (threadIdx.x < 32) sh[threadIdx.x] = ~0u;
    __syncthreads();
    const int64_t frame = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (frame < B)
        for (int w = 0; w < nvw; ++w) atomicAnd(&sh[w], ws_valid[frame * nvw + w]);
    __syncthreads();
    if (threadIdx.x < nvw) atomicAnd(&all_words[threadIdx.x], sh[threadIdx.x]);
}

__global__ __launch_bounds__(512) void batch_emit_kernel(FloodTables T, const uint64_t *__restrict__ ws_words,
                                                         const uint32_t *__restrict__ all_words, int max_iter,
                                                         int nvw, int64_t B, int out_dtype, void *bits,
                                                         int32_t *iters_out, uint32_t *partials,
                                                         const int32_t *__restrict__ ctl) {
    if (ctl[2] == 0) return;
    __shared__ uint32_t red[2 * 512];
    int tstar = max_iter - 1;  // first iteration at which every frame was valid
    for (int w = 0; w < nvw; ++w) {
        const uint32_t aw = all_words[w];
        if (aw) {
            const int t = w * 32 + __builtin_ctz(aw);
            if (t < max_iter) { tstar = t; break; }
        }
    }
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Lane L = make_lane(T, nullptr, B);
    Ctx C;
    C.T = T;
    C.out_dtype = out_dtype;
    C.bits = bits;
    int errs = 0;
    emit_from_words(C, L, ws_words + ((int64_t)blockIdx.x * max_iter + tstar) * T.Nb, ~0ull, wave, errs);
    if (iters_out && L.valid && L.k == 0) iters_out[L.frame] = tstar + 1;
    const int nf = (int)min<int64_t>((int64_t)T.FG, B - (int64_t)blockIdx.x * T.FG);
    if (partials) reduce_counters(red, L, errs, tstar + 1, nf, T.Z, partials + (int64_t)blockIdx.x * kPartRow);
}

__global__ void fill_i32_kernel(int32_t *p, int32_t v) { *p = v; }


int reduce_counter_rows(const uint32_t *partials, int64_t nwg, uint64_t *counters, int32_t *batch_iters,
                        const int32_t *gate, hipStream_t s) {
    hipLaunchKernelGGL(counters_reduce_kernel, dim3(1), dim3(1024), 0, s, partials, nwg, counters, batch_iters, gate);
    LDPC_CHECK_LAUNCH("counters_reduce_kernel");
    return LDPC_OK;
}

// ---------------------------------------------------------------- host side
namespace {
constexpr size_t kLdsMax = 160 * 1024;

size_t flood_lds_bytes(const ldpc_graph *g, int es) {
    size_t b = (size_t)g->nslots * 64 * sizeof(float) + 8;  // slots + the NaN flag
    if (es != LDPC_ES_OFF) b += (size_t)(g->Nb + 1) * sizeof(uint64_t);
    return std::max<size_t>(b, 2 * 64 * (size_t)g->ft.W * sizeof(uint32_t));
}

// Workspace: [counter rows: nwg x kPartRow uint32] then, for LDPC_ES_BATCH, the EsWs arrays.
// base == nullptr only sizes it.
struct FloodWs {
    uint32_t *partials;
    EsWs es;
    uint32_t *all;
    int64_t bytes;
};

FloodWs flood_ws(const ldpc_graph *g, int64_t B, int max_iter, int early_stop, void *base) {
    FloodWs w{};
    const int64_t nwg = (B + g->FG - 1) / g->FG;
    char *p = static_cast<char *>(base);
    size_t off = 0;
    auto take = [&](size_t n) { char *q = p ? p + off : nullptr; off += align256(n); return q; };
    w.partials = reinterpret_cast<uint32_t *>(take((size_t)nwg * kPartRow * 4));
    if (early_stop == LDPC_ES_BATCH) {
        EsWs &e = w.es;
        e.nvw = (max_iter + 31) / 32;
        e.words = reinterpret_cast<uint64_t *>(take((size_t)nwg * max_iter * g->Nb * 8));
        e.valid = reinterpret_cast<uint32_t *>(take((size_t)B * e.nvw * 4));
        w.all = reinterpret_cast<uint32_t *>(take(64 * 4));
        e.cand = reinterpret_cast<uint64_t *>(take((size_t)nwg * g->Nb * 8));
        e.twg = reinterpret_cast<int32_t *>(take((size_t)nwg * 4));
        e.ctl = reinterpret_cast<int32_t *>(take(64));
        e.staged = reinterpret_cast<uint64_t *>(take(64));
    }
    w.bytes = (int64_t)off;
    return w;
}

bool use_stream(const ldpc_graph *g, int es) {
    if (!g->lds_ok || flood_lds_bytes(g, es) > kLdsMax) return true;
    const char *e = std::getenv("LDPC_FLOOD_STREAM");  // force the streaming kernels (tests, A/B)
    return e && std::atoi(e) != 0;
}

template <int ALGO, int ES>
int launch_flood(const ldpc_graph *g, const float *llr, int64_t B, int max_iter, float alpha, int out_dtype,
                 void *bits, const Outs &O, const EsWs &W, hipStream_t s) {
    const size_t lds = flood_lds_bytes(g, ES);
    const int64_t nwg = (B + g->FG - 1) / g->FG;
    if (g->fixed_id != 0) {  // compile-time schedules: their own translation units
        const dim3 grid((unsigned)nwg), block(64 * g->ft.W);
        return ALGO == LDPC_ALGO_MINSUM
                   ? launch_fixed_minsum(g->fixed_id, ES, grid, block, lds, s, g->ft, llr, B, max_iter, alpha,
                                         out_dtype, bits, O, W)
                   : launch_fixed_bp(g->fixed_id, ES, grid, block, lds, s, g->ft, llr, B, max_iter, alpha,
                                     out_dtype, bits, O, W);
    }
    auto kern = flood_kernel<ALGO, ES>;
    LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(64 * g->ft.W), lds, s, g->ft, llr, B, max_iter, alpha,
                       out_dtype, bits, O, W);
    LDPC_CHECK_LAUNCH("flood_kernel");
    return LDPC_OK;
}

int reduce_rows(const ldpc_graph *g, int64_t B, const uint32_t *partials, uint64_t *counters, int32_t *batch_iters,
                const int32_t *gate, hipStream_t s, int frames_per_wg = 0) {
    if (!counters && !batch_iters) return LDPC_OK;
    const int fg = frames_per_wg > 0 ? frames_per_wg : g->FG;
    const int64_t nwg = (B + fg - 1) / fg;
    return reduce_counter_rows(partials, nwg, counters, batch_iters, gate, s);
}

template <int ALGO>
int run_flood(const ldpc_graph *g, const float *llr, int64_t B, int max_iter, float alpha, int es, int out_dtype,
              void *bits, int32_t *iters_out, uint64_t *counters, int32_t *batch_iters, void *work, hipStream_t s) {
    const FloodWs ws = flood_ws(g, B, max_iter, es, work);
    const bool want = counters || batch_iters;
    const Outs O{iters_out, want ? ws.partials : nullptr};
    if (es == LDPC_ES_OFF) {
#ifdef LDPC_TIMELINE
        // timeline build: stamps of the first kTlWgs workgroups, dumped after the decode to
        // $LDPC_TIMELINE_OUT (header: kTlWgs, waves, stamps per wave, max_iter, then uint64 stamps)
        static uint64_t *tl = nullptr;
        const size_t tl_n = (size_t)kTlWgs * 4 * kTlPer;
        if (!tl) LDPC_HIP(hipMalloc(&tl, tl_n * 8));
        LDPC_HIP(hipMemsetAsync(tl, 0, tl_n * 8, s));
        Outs Ot = O;
        Ot.timeline = tl;
        int rc = launch_flood<ALGO, LDPC_ES_OFF>(g, llr, B, max_iter, alpha, out_dtype, bits, Ot, EsWs{}, s);
        if (const char *path = std::getenv("LDPC_TIMELINE_OUT")) {
            std::vector<uint64_t> h(tl_n);
            LDPC_HIP(hipStreamSynchronize(s));
            LDPC_HIP(hipMemcpy(h.data(), tl, tl_n * 8, hipMemcpyDeviceToHost));
            if (FILE *f = std::fopen(path, "wb")) {
                const int32_t hdr[4] = {kTlWgs, 4, kTlPer, max_iter};
                std::fwrite(hdr, 4, 4, f);
                std::fwrite(h.data(), 8, h.size(), f);
                std::fclose(f);
            }
        }
#else
        int rc = launch_flood<ALGO, LDPC_ES_OFF>(g, llr, B, max_iter, alpha, out_dtype, bits, O, EsWs{}, s);
#endif
        // ES off: every frame ran max_iter (batch_iters was set before the launch)
        return rc != LDPC_OK ? rc : reduce_rows(g, B, ws.partials, counters, nullptr, nullptr, s);
    }
    if (es == LDPC_ES_FRAME) {
        int rc = launch_flood<ALGO, LDPC_ES_FRAME>(g, llr, B, max_iter, alpha, out_dtype, bits, O, EsWs{}, s);
        return rc != LDPC_OK ? rc : reduce_rows(g, B, ws.partials, counters, batch_iters, nullptr, s);
    }
    const EsWs &W = ws.es;
    hipLaunchKernelGGL(es_init_kernel, dim3(1), dim3(64), 0, s, W.ctl, W.staged, ws.all);
    LDPC_CHECK_LAUNCH("es_init_kernel");
    LDPC_HIP(hipMemsetAsync(W.valid, 0, (size_t)B * W.nvw * 4, s));
    int rc = launch_flood<ALGO, ES_P1>(g, llr, B, max_iter, alpha, out_dtype, bits, Outs{}, W, s);
    if (rc != LDPC_OK) return rc;
    // P2 always writes its counter rows: they become `staged`, applied by es_finalize_kernel
    rc = launch_flood<ALGO, ES_P2>(g, llr, B, max_iter, alpha, out_dtype, bits, Outs{iters_out, ws.partials}, W, s);
    if (rc != LDPC_OK) return rc;
    rc = reduce_rows(g, B, ws.partials, W.staged, nullptr, nullptr, s);
    if (rc != LDPC_OK) return rc;
    // LDPC_FLOOD_ES_FALLBACK=1 forces the exhaustive pass (tests: both paths must agree)
    const char *ff = std::getenv("LDPC_FLOOD_ES_FALLBACK");
    hipLaunchKernelGGL(es_finalize_kernel, dim3(1), dim3(1), 0, s, W.ctl, max_iter, W.staged, counters,
                       batch_iters, (ff && std::atoi(ff) != 0) ? 1 : 0);
    LDPC_CHECK_LAUNCH("es_finalize_kernel");
    // fallback (runs only when es_finalize_kernel found a frame invalid at T)
    rc = launch_flood<ALGO, LDPC_ES_BATCH>(g, llr, B, max_iter, alpha, out_dtype, bits, Outs{}, W, s);
    if (rc != LDPC_OK) return rc;
    hipLaunchKernelGGL(batch_and_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, W.valid, B, W.nvw, ws.all,
                       W.ctl);
    LDPC_CHECK_LAUNCH("batch_and_kernel");
    const int64_t nwg = (B + g->FG - 1) / g->FG;
    hipLaunchKernelGGL(batch_emit_kernel, dim3((unsigned)nwg), dim3(64 * g->ft.W), 0, s, g->ft, W.words, ws.all,
                       max_iter, W.nvw, B, out_dtype, bits, iters_out, want ? ws.partials : nullptr, W.ctl);
    LDPC_CHECK_LAUNCH("batch_emit_kernel");
    return reduce_rows(g, B, ws.partials, counters, batch_iters, W.ctl + 2, s);
}
}  // namespace

}  // namespace ldpc

using namespace ldpc;

extern "C" int64_t ldpc_flood_workspace_size(const ldpc_graph *g, int64_t B, int max_iter, int early_stop) {
    if (!g || B < 0 || max_iter < 0) return fail(LDPC_EINVAL, "bad arguments");
    if (B == 0 || max_iter == 0) return 0;
    if (use_stream(g, early_stop)) return stream_ws_bytes(g, B, max_iter);
    return flood_ws(g, B, max_iter, early_stop, nullptr).bytes;
}

extern "C" int ldpc_flood_decode(const ldpc_graph *g, int algo, const float *d_llr, int64_t B,
                                 int max_iter, float alpha, int early_stop, int out_dtype,
                                 void *d_bits, int32_t *d_iters, int32_t *d_batch_iters,
                                 uint64_t *d_counters, void *d_work, int64_t work_bytes, void *stream) {
    if (!g) return fail(LDPC_EINVAL, "graph is NULL");
    if (algo != LDPC_ALGO_MINSUM && algo != LDPC_ALGO_BP) return fail(LDPC_EINVAL, "unknown algo");
    if (early_stop < 0 || early_stop > 2) return fail(LDPC_EINVAL, "unknown early_stop mode");
    if (out_dtype != LDPC_OUT_U8 && out_dtype != LDPC_OUT_F32) return fail(LDPC_EINVAL, "unknown out_dtype");
    if (B < 0) return fail(LDPC_EINVAL, "negative batch");
    if (max_iter < 1 || max_iter > 1024) return fail(LDPC_EINVAL, "max_iter must be in [1, 1024]");
    if (B == 0) return LDPC_OK;
    if (!d_llr || !d_bits) return fail(LDPC_EINVAL, "llr / bits is NULL");
    const bool streaming = use_stream(g, early_stop);
    if (streaming && (g->max_dv > kStreamMaxDeg || g->max_dc > kStreamMaxDeg))
        return fail(LDPC_EUNSUPPORTED, "streaming decoder: node degree above " + std::to_string(kStreamMaxDeg));
    // scratch is needed by the streaming decoder, the batch-global stop and any counter output
    if (streaming || early_stop == LDPC_ES_BATCH || d_counters || (d_batch_iters && early_stop == LDPC_ES_FRAME)) {
        const int64_t need = ldpc_flood_workspace_size(g, B, max_iter, early_stop);
        if (!d_work || work_bytes < need)
            return fail(LDPC_EINVAL, "workspace too small: need " + std::to_string(need) + " bytes");
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (d_batch_iters && early_stop == LDPC_ES_OFF) {
        hipLaunchKernelGGL(fill_i32_kernel, dim3(1), dim3(1), 0, s, d_batch_iters, max_iter);
        LDPC_CHECK_LAUNCH("fill");
    }
    if (streaming)
        return algo == LDPC_ALGO_MINSUM
                   ? run_stream_decode(LDPC_ALGO_MINSUM, g, d_llr, B, max_iter, alpha, early_stop, out_dtype, d_bits,
                                       d_iters, d_counters, d_batch_iters, d_work, s)
                   : run_stream_decode(LDPC_ALGO_BP, g, d_llr, B, max_iter, alpha, early_stop, out_dtype, d_bits,
                                       d_iters, d_counters, d_batch_iters, d_work, s);
    return algo == LDPC_ALGO_MINSUM
               ? run_flood<LDPC_ALGO_MINSUM>(g, d_llr, B, max_iter, alpha, early_stop, out_dtype, d_bits, d_iters,
                                             d_counters, d_batch_iters, d_work, s)
               : run_flood<LDPC_ALGO_BP>(g, d_llr, B, max_iter, alpha, early_stop, out_dtype, d_bits, d_iters,
                                         d_counters, d_batch_iters, d_work, s);
}

extern "C" int64_t ldpc_custom_minsum_workspace_size(const ldpc_graph *g, int64_t B) {
    if (!g || B < 0) return fail(LDPC_EINVAL, "bad arguments");
    return B == 0 ? 0 : custom_ws_bytes(g, B);
}

extern "C" int ldpc_custom_minsum_decode(const ldpc_graph *g, const float *d_llr, int64_t B, int iterations,
                                         float *d_probs, void *d_work, int64_t work_bytes, void *stream) {
    if (!g) return fail(LDPC_EINVAL, "graph is NULL");
    if (B < 0) return fail(LDPC_EINVAL, "negative batch");
    if (iterations < 0 || iterations > 1024) return fail(LDPC_EINVAL, "iterations must be in [0, 1024]");
    if (B == 0) return LDPC_OK;
    if (B > 65535LL * 64) return fail(LDPC_EUNSUPPORTED, "batch above 4194240 frames in one call (chunk it)");
    if (!d_llr || !d_probs) return fail(LDPC_EINVAL, "llr / probs is NULL");
    if (g->max_dv > kStreamMaxDeg || g->max_dc > kStreamMaxDeg)
        return fail(LDPC_EUNSUPPORTED, "node degree above " + std::to_string(kStreamMaxDeg));
    const int64_t need = custom_ws_bytes(g, B);
    if (!d_work || work_bytes < need) return fail(LDPC_EINVAL, "workspace too small: need " + std::to_string(need) + " bytes");
    return run_custom_minsum(g, d_llr, B, iterations, d_probs, d_work, static_cast<hipStream_t>(stream));
}
