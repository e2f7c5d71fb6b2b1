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
// evaluated in double and rounded (the reference uses torch-CPU SLEEF float versions, which are
// not correctly rounded, so BP parity is "within float32 tolerance", not bitwise).
// Compile with -ffp-contract=off: no a*b+c may fuse on this path.
#include <cmath>
#include <cstdint>

#include "common.hpp"
#include "graph.hpp"

namespace ldpc {

namespace {

// Graph tables are read-only for the kernel's lifetime and indexed by wave-uniform values:
// reading them through the constant address space lets the compiler use scalar (SMEM) loads
// instead of per-lane vector loads.
typedef const __attribute__((address_space(4))) int32_t const_i32;
__device__ __forceinline__ int32_t tab(const int32_t *p, int i) {
    return ((const_i32 *)p)[i];
}

__device__ __forceinline__ int rot_add(int k, int s, int Z) {
    const int t = k + s;
    return t >= Z ? t - Z : t;
}
__device__ __forceinline__ int rot_sub(int k, int s, int Z) {
    const int t = k - s;
    return t < 0 ? t + Z : t;
}

struct Lane {
    int lane, f, k, fz, Z;
    bool valid;    // the lane's frame exists (Z divides 64: every lane has a position)
    int64_t frame;
    const float *llr_row;
    // index of the message on a block with shift s, seen from variable t = k of frame f
    __device__ __forceinline__ int vidx(int s) const { return fz + rot_sub(k, s, Z); }
    // llr_row points at a real row for every lane (frame 0 for lanes without a frame), so the
    // load needs no branch; results of such lanes are never stored.
    __device__ __forceinline__ float llr(int col, int t) const { return llr_row[col * Z + t]; }
};

__device__ __forceinline__ void put_bit(void *bits, int out_dtype, int64_t idx, int bit) {
    if (out_dtype == LDPC_OUT_F32)
        static_cast<float *>(bits)[idx] = bit ? 1.0f : 0.0f;
    else
        static_cast<uint8_t *>(bits)[idx] = (uint8_t)bit;
}

__device__ __forceinline__ bool is_zero_sign(float x) { return !(x > 0.0f || x < 0.0f); }

// ---------------------------------------------------------------- check updates (registers)
// Min-sum statistics of one check row (traditional_decoders.py:207-232):
//   c2v_e = prod_{e'!=e} sign(v) * (alpha * min_{e'!=e} |v|)
// with torch.sign(0) = torch.sign(NaN) = 0 and NaN never winning the min (mag < min_mag fails).
struct MinSumStats {
    int nz = 0;         // number of zero/NaN signs in the row
    bool neg = false;   // parity of negative signs
    float m1 = INFINITY, m2 = INFINITY;
    int i1 = -1;        // first index attaining m1
    __device__ __forceinline__ void add(int e, float x) {
        const float a = fabsf(x);
        nz += is_zero_sign(x);
        neg ^= (x < 0.0f);
        const bool lt1 = a < m1, lt2 = a < m2;  // NaN: both false
        m2 = lt1 ? m1 : (lt2 ? a : m2);
        i1 = lt1 ? e : i1;
        m1 = lt1 ? a : m1;
    }
    __device__ __forceinline__ float c2v(int e, float x, float alpha) const {
        const float m = (e == i1) ? m2 : m1;
        const int zex = nz - (int)is_zero_sign(x);
        const float s = zex > 0 ? 0.0f : ((neg ^ (x < 0.0f)) ? -1.0f : 1.0f);
        return s * (alpha * m);
    }
};

__device__ __forceinline__ float tanh_half(float v) { return (float)tanh((double)(v / 2.0f)); }
__device__ __forceinline__ float two_atanh(float p) { return 2.0f * (float)atanh((double)p); }

struct Ctx {
    FloodTables T;
    float *lds;
    uint64_t *words;  // ES: Nb decision ballots + 1 invalid-lane word
    float alpha;
    int out_dtype;
    void *bits;
    bool direct_bits;  // mode 0, final iteration: write decisions straight to HBM
    bool ballots;      // ES: record decisions as ballots
};

// decision of variable (col, t = rot_add(k, s)) computed on the lane of check row k
__device__ __forceinline__ void ext_decision(const Ctx &C, const Lane &L, int col, int s, float app,
                                             int &errs) {
    const int bit = app < 0.0f;  // NaN < 0 is false -> 0 (traditional_decoders.py:252)
    if (C.direct_bits) {
        if (L.valid) {
            put_bit(C.bits, C.out_dtype, L.frame * C.T.N + (int64_t)col * L.Z + rot_add(L.k, s, L.Z), bit);
            errs += bit;
        }
    }
    if (C.ballots) {
        // move the bit of variable t to lane f*Z + t before the ballot
        const int src = L.fz + rot_sub(L.k, s, L.Z);
        const int bt = __shfl(bit, src, 64);
        const uint64_t w = __ballot(bt);
        if (L.lane == 0) C.words[col] = w;
    }
}

__device__ __forceinline__ void var_decision(const Ctx &C, const Lane &L, int col, float app, int &errs) {
    const int bit = app < 0.0f;
    if (C.direct_bits) {
        if (L.valid) {
            put_bit(C.bits, C.out_dtype, L.frame * C.T.N + (int64_t)col * L.Z + L.k, bit);
            errs += bit;
        }
    }
    if (C.ballots) {
        const uint64_t w = __ballot(bit);
        if (L.lane == 0) C.words[col] = w;
    }
}

template <int ALGO, int DC>
__device__ __forceinline__ void check_task(const Ctx &C, const Lane &L, int r, int &errs) {
    const int p0 = tab(C.T.row_ptr, r);
    float v[DC];
#pragma unroll
    for (int e = 0; e < DC; ++e) {
        const int sl = tab(C.T.row_slot, p0 + e);
        if (sl >= 0)
            v[e] = C.lds[sl * 64 + L.lane];
        else
            v[e] = L.llr(tab(C.T.row_col, p0 + e), rot_add(L.k, tab(C.T.row_shift, p0 + e), L.Z));
    }
    auto emit = [&](int e, float o) {
        const int sl = tab(C.T.row_slot, p0 + e);
        if (sl >= 0)
            C.lds[sl * 64 + L.lane] = o;
        else if (C.direct_bits || C.ballots)  // degree-1 variable: APP = llr.clone() + c2v
            ext_decision(C, L, tab(C.T.row_col, p0 + e), tab(C.T.row_shift, p0 + e), v[e] + o, errs);
    };
    if constexpr (ALGO == LDPC_ALGO_MINSUM) {
        MinSumStats st;
#pragma unroll
        for (int e = 0; e < DC; ++e) st.add(e, v[e]);
#pragma unroll
        for (int e = 0; e < DC; ++e) emit(e, st.c2v(e, v[e], C.alpha));
    } else {
        // sum-product (traditional_decoders.py:72-81): c2v_e = 2 atanh(prod_{e'!=e} tanh(v/2)),
        // product from 1.0 in ascending e'.  acc[e] = P_e * t_{e+1} * ... built column by column.
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
        for (int e = 0; e < DC; ++e) emit(e, two_atanh(acc[e]));
    }
}

// Any degree: messages re-read from LDS instead of registers (O(dc^2) reads; only used past
// kMaxUnroll).  In-place is safe in ascending e: slot e is overwritten after P_{e+1} used it.
template <int ALGO>
__device__ __forceinline__ void check_task_dyn(const Ctx &C, const Lane &L, int r, int &errs) {
    const int p0 = tab(C.T.row_ptr, r), p1 = tab(C.T.row_ptr, r + 1);
    auto rd = [&](int p) -> float {
        const int sl = tab(C.T.row_slot, p);
        return sl >= 0 ? C.lds[sl * 64 + L.lane] : L.llr(tab(C.T.row_col, p), rot_add(L.k, tab(C.T.row_shift, p), L.Z));
    };
    auto wr = [&](int p, float in, float out) {
        const int sl = tab(C.T.row_slot, p);
        if (sl >= 0)
            C.lds[sl * 64 + L.lane] = out;
        else if (C.direct_bits || C.ballots)
            ext_decision(C, L, tab(C.T.row_col, p), tab(C.T.row_shift, p), in + out, errs);
    };
    if constexpr (ALGO == LDPC_ALGO_MINSUM) {
        MinSumStats st;
        for (int p = p0; p < p1; ++p) st.add(p, rd(p));
        for (int p = p0; p < p1; ++p) {
            const float x = rd(p);
            wr(p, x, st.c2v(p, x, C.alpha));
        }
    } else {
        float P = 1.0f;
        for (int p = p0; p < p1; ++p) {
            const float x = rd(p);
            float rr = P;
            for (int q = p + 1; q < p1; ++q) rr = rr * tanh_half(rd(q));
            const float t = tanh_half(x);
            wr(p, x, two_atanh(rr));
            P = P * t;
        }
    }
}

// Variable update (traditional_decoders.py:235-250): v2c_e = llr + sum_{e'!=e} c_e' added in
// ascending check order, i.e. acc[e] = P_e (prefix) followed by c_{e+1}, c_{e+2}, ...;
// the APP is P_DV = llr + c_0 + ... + c_{DV-1}.
template <int DV>
__device__ __forceinline__ void var_task(const Ctx &C, const Lane &L, int task, bool write, int &errs) {
    const int col = tab(C.T.vc_col, task);
    const int p0 = tab(C.T.vc_ptr, task);
    float P = L.llr(col, L.k);
    if constexpr (DV > 0) {
        float acc[DV];
#pragma unroll
        for (int j = 0; j < DV; ++j) {
            const float c = C.lds[tab(C.T.vc_slot, p0 + j) * 64 + L.vidx(tab(C.T.vc_shift, p0 + j))];
#pragma unroll
            for (int e = 0; e < j; ++e) acc[e] = acc[e] + c;
            acc[j] = P;
            P = P + c;
        }
        if (write) {
#pragma unroll
            for (int e = 0; e < DV; ++e) C.lds[tab(C.T.vc_slot, p0 + e) * 64 + L.vidx(tab(C.T.vc_shift, p0 + e))] = acc[e];
        }
    }
    if (C.direct_bits || C.ballots) var_decision(C, L, col, P, errs);
}

__device__ __forceinline__ void var_task_dyn(const Ctx &C, const Lane &L, int task, bool write, int &errs) {
    const int col = tab(C.T.vc_col, task);
    const int p0 = tab(C.T.vc_ptr, task), p1 = tab(C.T.vc_ptr, task + 1);
    const float x = L.llr(col, L.k);
    float P = x;
    for (int p = p0; p < p1; ++p) {
        const int id = tab(C.T.vc_slot, p) * 64 + L.vidx(tab(C.T.vc_shift, p));
        const float cp = C.lds[id];
        float acc = P;
        for (int q = p + 1; q < p1; ++q) acc = acc + C.lds[tab(C.T.vc_slot, q) * 64 + L.vidx(tab(C.T.vc_shift, q))];
        P = P + cp;
        if (write) C.lds[id] = acc;
    }
    if (C.direct_bits || C.ballots) var_decision(C, L, col, P, errs);
}

// degrees with unrolled register code; larger ones take the *_dyn paths
#define LDPC_DC_CASES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12)
#define LDPC_DV_CASES(X) \
    X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) \
    X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24)

template <int ALGO>
__device__ __forceinline__ void check_dispatch(const Ctx &C, const Lane &L, int r, int &errs) {
    const int dc = tab(C.T.row_ptr, r + 1) - tab(C.T.row_ptr, r);
    switch (dc) {
        case 0: break;
#define X(n) case n: check_task<ALGO, n>(C, L, r, errs); break;
        LDPC_DC_CASES(X)
#undef X
        default: check_task_dyn<ALGO>(C, L, r, errs); break;
    }
}

__device__ __forceinline__ void var_dispatch(const Ctx &C, const Lane &L, int task, bool write, int &errs) {
    const int dv = tab(C.T.vc_ptr, task + 1) - tab(C.T.vc_ptr, task);
    switch (dv) {
        case 0: var_task<0>(C, L, task, write, errs); break;
#define X(n) case n: var_task<n>(C, L, task, write, errs); break;
        LDPC_DV_CASES(X)
#undef X
        default: var_task_dyn(C, L, task, write, errs); break;
    }
}

__device__ __forceinline__ int parity_row(const Ctx &C, const Lane &L, int r) {
    int p = 0;
    for (int q = tab(C.T.row_ptr, r); q < tab(C.T.row_ptr, r + 1); ++q)
        p ^= (int)((C.words[tab(C.T.row_col, q)] >> (L.fz + rot_add(L.k, tab(C.T.row_shift, q), L.Z))) & 1ull);
    return p;
}

__device__ __forceinline__ uint64_t frame_valid_mask(uint64_t invalid_lanes, int Z, int FG) {
    const uint64_t seg = Z >= 64 ? ~0ull : ((1ull << Z) - 1ull);
    uint64_t m = 0;
    for (int f = 0; f < FG; ++f)
        if (((invalid_lanes >> (f * Z)) & seg) == 0) m |= 1ull << f;
    return m;
}

// emit the decisions of frames in `mask` from the ballots (columns spread over the waves)
__device__ __forceinline__ void emit_from_words(const Ctx &C, const Lane &L, const uint64_t *words, uint64_t mask,
                                int wave, int &errs) {
    if (!(L.valid && ((mask >> L.f) & 1ull))) return;
    for (int i = tab(C.T.bw_ptr, wave); i < tab(C.T.bw_ptr, wave + 1); ++i) {
        const int col = tab(C.T.bw_task, i);
        const int bit = (int)((words[col] >> L.lane) & 1ull);
        put_bit(C.bits, C.out_dtype, L.frame * C.T.N + (int64_t)col * L.Z + L.k, bit);
        errs += bit;
    }
}

// per-workgroup reduction of the error counters: {bit errors, frame errors, frames, iter sum}
__device__ __forceinline__ void reduce_counters(float *lds, const Lane &L, int errs, int my_iters, int nf, int FG,
                                int Z, uint64_t *counters, int32_t *batch_iters) {
    uint32_t *u = reinterpret_cast<uint32_t *>(lds);
    const int nt = blockDim.x;
    __syncthreads();
    u[threadIdx.x] = (uint32_t)errs;
    u[nt + threadIdx.x] = (uint32_t)my_iters;
    __syncthreads();
    if (threadIdx.x < 64) {
        const int f = threadIdx.x;
        uint64_t be = 0, fe = 0, fr = 0, it = 0;
        int itmax = 0;
        if (f < nf) {
            for (int w = 0; w < nt / 64; ++w)
                for (int k = 0; k < Z; ++k) be += u[w * 64 + f * Z + k];
            fe = be > 0;
            fr = 1;
            it = u[nt + f * Z];
            itmax = (int)it;
        }
        for (int off = 32; off > 0; off >>= 1) {
            be += __shfl_xor(be, off, 64);
            fe += __shfl_xor(fe, off, 64);
            fr += __shfl_xor(fr, off, 64);
            it += __shfl_xor(it, off, 64);
            itmax = max(itmax, __shfl_xor(itmax, off, 64));
        }
        if (f == 0) {
            if (counters) {
                atomicAdd((unsigned long long *)&counters[0], (unsigned long long)be);
                atomicAdd((unsigned long long *)&counters[1], (unsigned long long)fe);
                atomicAdd((unsigned long long *)&counters[2], (unsigned long long)fr);
                atomicAdd((unsigned long long *)&counters[3], (unsigned long long)it);
            }
            if (batch_iters) atomicMax(batch_iters, itmax);
        }
    }
    (void)FG;
}

}  // namespace

template <int ALGO, int ES>
__global__ __launch_bounds__(512) void flood_kernel(FloodTables T, const float *__restrict__ llr,
                                                    int64_t B, int max_iter, float alpha,
                                                    int out_dtype, void *__restrict__ bits,
                                                    int32_t *__restrict__ iters_out,
                                                    uint64_t *__restrict__ counters,
                                                    int32_t *__restrict__ batch_iters,
                                                    uint64_t *__restrict__ ws_words,
                                                    uint32_t *__restrict__ ws_valid, int nvw) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    Lane L;
    L.lane = tid & 63;
    L.Z = T.Z;
    L.f = L.lane / T.Z;
    L.k = L.lane - L.f * T.Z;
    L.fz = L.f * T.Z;
    L.frame = (int64_t)blockIdx.x * T.FG + L.f;
    L.valid = L.frame < B;
    L.llr_row = llr + (L.valid ? L.frame : 0) * (int64_t)T.N;
    const int nf = (int)min<int64_t>((int64_t)T.FG, B - (int64_t)blockIdx.x * T.FG);
    const uint64_t exist = nf >= 64 ? ~0ull : ((1ull << nf) - 1ull);

    Ctx C;
    C.T = T;
    C.lds = lds;
    C.words = reinterpret_cast<uint64_t *>(lds + (size_t)T.nslots * 64);
    C.alpha = alpha;
    C.out_dtype = out_dtype;
    C.bits = bits;
    C.direct_bits = false;
    C.ballots = ES != LDPC_ES_OFF;

    // v2c <- llr on every slot (traditional_decoders.py:199-202)
    for (int i = tab(T.vw_ptr, wave); i < tab(T.vw_ptr, wave + 1); ++i) {
        const int task = tab(T.vw_task, i);
        const int col = tab(T.vc_col, task);
        const float x = L.llr(col, L.k);
        for (int p = tab(T.vc_ptr, task); p < tab(T.vc_ptr, task + 1); ++p)
            lds[tab(T.vc_slot, p) * 64 + L.vidx(tab(T.vc_shift, p))] = x;
    }
    __syncthreads();

    int errs = 0;
    int my_iters = max_iter;
    uint64_t done = 0;
    for (int it = 0; it < max_iter; ++it) {
        const bool last = it == max_iter - 1;
        C.direct_bits = (ES == LDPC_ES_OFF) && last;
        for (int i = tab(T.cw_ptr, wave); i < tab(T.cw_ptr, wave + 1); ++i) check_dispatch<ALGO>(C, L, tab(T.cw_task, i), errs);
        __syncthreads();
        if (ES != LDPC_ES_OFF && tid == 0) C.words[T.Nb] = 0;
        for (int i = tab(T.vw_ptr, wave); i < tab(T.vw_ptr, wave + 1); ++i) var_dispatch(C, L, tab(T.vw_task, i), !last, errs);
        __syncthreads();
        if constexpr (ES != LDPC_ES_OFF) {
            // syndrome H x = 0 per frame (traditional_decoders.py:111-134), from the ballots
            int inv = 0;
            for (int i = tab(T.cw_ptr, wave); i < tab(T.cw_ptr, wave + 1); ++i) inv |= parity_row(C, L, tab(T.cw_task, i));
            const uint64_t m = __ballot(inv);
            if (L.lane == 0 && m) atomicOr((unsigned long long *)&C.words[T.Nb], (unsigned long long)m);
            __syncthreads();
            const uint64_t vmask = frame_valid_mask(C.words[T.Nb], T.Z, T.FG) & exist;
            if constexpr (ES == LDPC_ES_BATCH) {
                if (L.valid && L.k == 0 && ((vmask >> L.f) & 1ull))
                    ws_valid[L.frame * nvw + (it >> 5)] |= 1u << (it & 31);
                uint64_t *dst = ws_words + ((int64_t)blockIdx.x * max_iter + it) * T.Nb;
                for (int c = tid; c < T.Nb; c += blockDim.x) dst[c] = C.words[c];
            } else {
                const uint64_t newly = vmask & ~done;
                if (newly) {
                    emit_from_words(C, L, C.words, newly, wave, errs);
                    if ((newly >> L.f) & 1ull) my_iters = it + 1;
                    if (iters_out && L.valid && L.k == 0 && ((newly >> L.f) & 1ull)) iters_out[L.frame] = it + 1;
                    done |= newly;
                }
            }
            __syncthreads();
            if (ES == LDPC_ES_FRAME && done == exist) break;
        }
    }
    if constexpr (ES == LDPC_ES_FRAME) {
        const uint64_t rest = exist & ~done;
        if (rest) {
            emit_from_words(C, L, C.words, rest, wave, errs);
            if (iters_out && L.valid && L.k == 0 && ((rest >> L.f) & 1ull)) iters_out[L.frame] = max_iter;
        }
    }
    if constexpr (ES == LDPC_ES_OFF) {
        if (iters_out && L.valid && L.k == 0) iters_out[L.frame] = max_iter;
    }
    if constexpr (ES != LDPC_ES_BATCH) {
        if (counters || batch_iters) reduce_counters(lds, L, errs, my_iters, nf, T.FG, T.Z, counters, batch_iters);
    }
}

// ---------------------------------------------------------------- batch-global early stop
__global__ void batch_and_kernel(const uint32_t *__restrict__ ws_valid, int64_t B, int nvw,
                                 uint32_t *__restrict__ all_words) {
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
                                                         int32_t *iters_out, int32_t *batch_iters,
                                                         uint64_t *counters) {
    __shared__ float red[2 * 512];
    int tstar = max_iter - 1;  // first iteration at which every frame was valid
    for (int w = 0; w < nvw; ++w) {
        const uint32_t aw = all_words[w];
        if (aw) {
            const int t = w * 32 + __builtin_ctz(aw);
            if (t < max_iter) { tstar = t; break; }
        }
    }
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    Lane L;
    L.lane = tid & 63;
    L.Z = T.Z;
    L.f = L.lane / T.Z;
    L.k = L.lane - L.f * T.Z;
    L.fz = L.f * T.Z;
    L.frame = (int64_t)blockIdx.x * T.FG + L.f;
    L.valid = L.frame < B;
    L.llr_row = nullptr;
    Ctx C;
    C.T = T;
    C.out_dtype = out_dtype;
    C.bits = bits;
    int errs = 0;
    emit_from_words(C, L, ws_words + ((int64_t)blockIdx.x * max_iter + tstar) * T.Nb, ~0ull, wave, errs);
    if (iters_out && L.valid && L.k == 0) iters_out[L.frame] = tstar + 1;
    const int nf = (int)min<int64_t>((int64_t)T.FG, B - (int64_t)blockIdx.x * T.FG);
    if (counters || batch_iters) reduce_counters(red, L, errs, tstar + 1, nf, T.FG, T.Z, counters, batch_iters);
}

__global__ void fill_i32_kernel(int32_t *p, int32_t v) { *p = v; }

// ---------------------------------------------------------------- host side
namespace {
constexpr size_t kLdsMax = 160 * 1024;

size_t flood_lds_bytes(const ldpc_graph *g, int es) {
    size_t b = (size_t)g->nslots * 64 * sizeof(float);
    if (es != LDPC_ES_OFF) b += (size_t)(g->Nb + 1) * sizeof(uint64_t);
    return std::max<size_t>(b, 2 * 64 * (size_t)g->ft.W * sizeof(uint32_t));
}

struct BatchWs {
    uint64_t *words;
    uint32_t *valid;
    uint32_t *all;
    int64_t bytes;
    int nvw;
};

BatchWs batch_ws(const ldpc_graph *g, int64_t B, int max_iter, void *base) {
    BatchWs w{};
    const int64_t nwg = (B + g->FG - 1) / g->FG;
    w.nvw = (max_iter + 31) / 32;
    char *p = static_cast<char *>(base);
    const int64_t words_b = nwg * max_iter * g->Nb * 8;
    const int64_t valid_b = ((B * w.nvw * 4) + 255) / 256 * 256;
    w.words = reinterpret_cast<uint64_t *>(p);
    w.valid = reinterpret_cast<uint32_t *>(p + words_b);
    w.all = reinterpret_cast<uint32_t *>(p + words_b + valid_b);
    w.bytes = words_b + valid_b + 256;
    return w;
}

template <int ALGO, int ES>
int launch_flood(const ldpc_graph *g, const float *llr, int64_t B, int max_iter, float alpha,
                 int out_dtype, void *bits, int32_t *iters, uint64_t *counters, int32_t *batch_iters,
                 uint64_t *ws_words, uint32_t *ws_valid, int nvw, hipStream_t s) {
    const size_t lds = flood_lds_bytes(g, ES);
    auto kern = flood_kernel<ALGO, ES>;
    LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int64_t nwg = (B + g->FG - 1) / g->FG;
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(64 * g->ft.W), lds, s, g->ft, llr, B, max_iter, alpha,
                       out_dtype, bits, iters, counters, batch_iters, ws_words, ws_valid, nvw);
    LDPC_CHECK_LAUNCH("flood_kernel");
    return LDPC_OK;
}
}  // namespace

}  // namespace ldpc

using namespace ldpc;

extern "C" int64_t ldpc_flood_workspace_size(const ldpc_graph *g, int64_t B, int max_iter, int early_stop) {
    if (!g || B < 0 || max_iter < 0) return fail(LDPC_EINVAL, "bad arguments");
    if (early_stop != LDPC_ES_BATCH || B == 0 || max_iter == 0) return 0;
    return batch_ws(g, B, max_iter, nullptr).bytes;
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
    if (flood_lds_bytes(g, early_stop) > kLdsMax)
        return fail(LDPC_EUNSUPPORTED, "graph too large for the LDS-resident decoder (" +
                                           std::to_string(g->nslots) + " slots)");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (d_batch_iters && early_stop != LDPC_ES_BATCH) {
        hipLaunchKernelGGL(fill_i32_kernel, dim3(1), dim3(1), 0, s, d_batch_iters,
                           early_stop == LDPC_ES_OFF ? max_iter : 0);
        LDPC_CHECK_LAUNCH("fill");
    }
    uint64_t *wsw = nullptr;
    uint32_t *wsv = nullptr;
    int nvw = 0;
    BatchWs bw{};
    if (early_stop == LDPC_ES_BATCH) {
        bw = batch_ws(g, B, max_iter, d_work);
        if (!d_work || work_bytes < bw.bytes)
            return fail(LDPC_EINVAL, "workspace too small: need " + std::to_string(bw.bytes) + " bytes");
        LDPC_HIP(hipMemsetAsync(bw.valid, 0, (size_t)B * bw.nvw * 4, s));
        LDPC_HIP(hipMemsetAsync(bw.all, 0xFF, 256, s));
        wsw = bw.words;
        wsv = bw.valid;
        nvw = bw.nvw;
    }
    int rc;
#define LAUNCH(A, E) rc = launch_flood<A, E>(g, d_llr, B, max_iter, alpha, out_dtype, d_bits, d_iters, \
                                             d_counters, d_batch_iters, wsw, wsv, nvw, s)
    if (algo == LDPC_ALGO_MINSUM) {
        if (early_stop == 0) LAUNCH(0, 0); else if (early_stop == 1) LAUNCH(0, 1); else LAUNCH(0, 2);
    } else {
        if (early_stop == 0) LAUNCH(1, 0); else if (early_stop == 1) LAUNCH(1, 1); else LAUNCH(1, 2);
    }
#undef LAUNCH
    if (rc != LDPC_OK) return rc;
    if (early_stop == LDPC_ES_BATCH) {
        hipLaunchKernelGGL(batch_and_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, bw.valid, B,
                           bw.nvw, bw.all);
        LDPC_CHECK_LAUNCH("batch_and_kernel");
        if (d_batch_iters) {
            hipLaunchKernelGGL(fill_i32_kernel, dim3(1), dim3(1), 0, s, d_batch_iters, 0);
            LDPC_CHECK_LAUNCH("fill");
        }
        const int64_t nwg = (B + g->FG - 1) / g->FG;
        hipLaunchKernelGGL(batch_emit_kernel, dim3((unsigned)nwg), dim3(64 * g->ft.W), 0, s, g->ft, bw.words, bw.all,
                           max_iter, bw.nvw, B, out_dtype, d_bits, d_iters, d_batch_iters, d_counters);
        LDPC_CHECK_LAUNCH("batch_emit_kernel");
    }
    return LDPC_OK;
}
