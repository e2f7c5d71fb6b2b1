// layers.hip -- the index-gather neural-BP layers of models/layers.py.
//
// The reference's CheckLayer / VariableLayer (layers.py:5-125) expand the (B, n) input to
// (n_out, B, n + 1), gather it through an (n_out, K) index tensor (-1 = padding -> a zero
// column) and reduce over K.  Here one thread owns one output (b, i) and walks its K indices:
// no expanded copies, every gathered value read once.  The index comes transposed, int32
// (K, n_out) -- prepared once per index tensor by the Python layer -- so that consecutive
// threads (consecutive i) read consecutive index words.  ResidualLayer (:128-168) and OutputLayer
// (:171-208) are elementwise / per-frame kernels.  Each forward has a backward that reproduces
// torch autograd through the reference's ops (gather -> scatter-add, min -> its argmin, the
// in-place masked writes -> zero gradient).
#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "common.hpp"

namespace ldpc {
namespace {

constexpr int kFB = 4;  // frames per thread in the forward gathers: one index read serves all four

__device__ __forceinline__ float torch_sign(float x) {  // torch.sign: NaN -> NaN, 0 -> 0
    return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : x * 0.0f);
}

// CheckLayer (layers.py:14-66): out[b][i] = prod_k sign(v_k + 1e-10) * min_k |v_k|' where
// v_k = in[b][idx[i][k]] (0 for idx -1) and |v|' replaces 0 by 1e10; torch.min propagates NaN and
// returns the first index of the minimum (kept for the backward).
__global__ void gather_minsum_kernel(const float *__restrict__ in, int64_t B, int n_in,
                                     const int32_t *__restrict__ idx, int n_out, int K, float *__restrict__ out,
                                     int32_t *__restrict__ argmin) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t ng = (B + kFB - 1) / kFB;
    if (t >= ng * n_out) return;
    const int64_t b0 = (t / n_out) * kFB;
    const int i = (int)(t % n_out);
    const int nb = (int)min<int64_t>(kFB, B - b0);
    float sp[kFB], m[kFB];
    int am[kFB];
#pragma unroll
    for (int f = 0; f < kFB; ++f) { sp[f] = 1.0f; m[f] = 0.0f; am[f] = 0; }
    for (int k = 0; k < K; ++k) {
        const int j = idx[(int64_t)k * n_out + i];  // one index read serves kFB frames
#pragma unroll
        for (int f = 0; f < kFB; ++f) {
            if (f >= nb) break;
            const float v = j < 0 ? 0.0f : in[(b0 + f) * n_in + j];
            sp[f] = sp[f] * torch_sign(v + 1e-10f);
            float a = fabsf(v);
            if (a == 0.0f) a = 1e10f;
            if (k == 0 || (!isnan(m[f]) && (a < m[f] || isnan(a)))) {
                m[f] = a;
                am[f] = k;
            }
        }
    }
#pragma unroll
    for (int f = 0; f < kFB; ++f) {
        if (f >= nb) break;
        const int64_t o = (b0 + f) * n_out + i;
        out[o] = sp[f] * m[f];
        if (argmin) argmin[o] = am[f];
    }
}

// LDS-staged form of the gathers (used for CheckLayer): a workgroup stages FPW whole input rows (frames) into LDS
// with coalesced 16-byte loads, then gathers from LDS.  The global kernels above gather 4-byte
// words at random columns of a row (a check's or variable's other edges are far apart in the
// var-major numbering), which is bound by address processing at ~0.8 TB/s; here the row is read
// once, contiguously.  Per output the arithmetic is the same sequence, so results are identical.
template <int FPW, bool MINSUM>
__global__ __launch_bounds__(512) void gather_lds_kernel(const float *__restrict__ in, const float *__restrict__ llr,
                                                         int64_t B, int n_in, const int32_t *__restrict__ idx, int n_out,
                                                         int K, float *__restrict__ out, int32_t *__restrict__ argmin) {
    extern __shared__ __attribute__((aligned(16))) float rows[];  // [FPW][n_in]
    const int64_t b0 = (int64_t)blockIdx.x * FPW;
    const int nb = (int)min<int64_t>(FPW, B - b0);
    const float *src = in + b0 * n_in;
    const int total = nb * n_in;
    if ((n_in & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        const float4 *s4 = reinterpret_cast<const float4 *>(src);
        float4 *r4 = reinterpret_cast<float4 *>(rows);
        for (int e = threadIdx.x; e < total / 4; e += blockDim.x) r4[e] = s4[e];
    } else {
        for (int e = threadIdx.x; e < total; e += blockDim.x) rows[e] = src[e];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n_out; i += blockDim.x) {
        float acc[FPW], m[FPW];
        int am[FPW];
#pragma unroll
        for (int f = 0; f < FPW; ++f) { acc[f] = MINSUM ? 1.0f : 0.0f; m[f] = 0.0f; am[f] = 0; }
        for (int k = 0; k < K; ++k) {
            const int j = idx[(int64_t)k * n_out + i];
            if (!MINSUM && j < 0) break;  // sum rows end at their first padding entry
#pragma unroll
            for (int f = 0; f < FPW; ++f) {
                if (f >= nb) break;
                const float v = j < 0 ? 0.0f : rows[f * n_in + j];
                if constexpr (MINSUM) {  // gather_minsum_kernel's update
                    acc[f] = acc[f] * torch_sign(v + 1e-10f);
                    float a = fabsf(v);
                    if (a == 0.0f) a = 1e10f;
                    if (k == 0 || (!isnan(m[f]) && (a < m[f] || isnan(a)))) {
                        m[f] = a;
                        am[f] = k;
                    }
                } else {  // gather_sum_kernel's update
                    acc[f] += v;
                }
            }
        }
#pragma unroll
        for (int f = 0; f < FPW; ++f) {
            if (f >= nb) break;
            const int64_t o = (b0 + f) * n_out + i;
            if constexpr (MINSUM) {
                out[o] = acc[f] * m[f];
                if (argmin) argmin[o] = am[f];
            } else {
                out[o] = llr ? llr[o] + acc[f] : acc[f];
            }
        }
    }
}

constexpr size_t kGatherLds = 64 * 1024;  // LDS per workgroup for the staged rows

// frames per workgroup for the staged gathers (0: a row does not fit, use the global kernel)
int gather_fpw(int n_in) {
    const size_t row = (size_t)n_in * 4;
    for (int f = 8; f >= 1; f /= 2)
        if ((size_t)f * row <= kGatherLds) return f;
    return 0;
}

template <bool MINSUM>
int launch_gather_lds(int fpw, const float *in, const float *llr, int64_t B, int n_in, const int32_t *idx, int n_out,
                      int K, float *out, int32_t *argmin, hipStream_t s) {
    const dim3 grid((unsigned)((B + fpw - 1) / fpw));
    const size_t lds = (size_t)fpw * n_in * 4;
    switch (fpw) {
        case 8: hipLaunchKernelGGL((gather_lds_kernel<8, MINSUM>), grid, dim3(512), lds, s, in, llr, B, n_in, idx, n_out, K, out, argmin); break;
        case 4: hipLaunchKernelGGL((gather_lds_kernel<4, MINSUM>), grid, dim3(512), lds, s, in, llr, B, n_in, idx, n_out, K, out, argmin); break;
        case 2: hipLaunchKernelGGL((gather_lds_kernel<2, MINSUM>), grid, dim3(512), lds, s, in, llr, B, n_in, idx, n_out, K, out, argmin); break;
        default: hipLaunchKernelGGL((gather_lds_kernel<1, MINSUM>), grid, dim3(512), lds, s, in, llr, B, n_in, idx, n_out, K, out, argmin); break;
    }
    LDPC_CHECK_LAUNCH("gather_lds_kernel");
    return LDPC_OK;
}

// CheckLayer when its index is a set of checks (every edge's row = the other edges of its check,
// as create_LLR_mapping builds it; detected once in Python): per (check, frame) one pass collects
// the sign-zero / NaN counts, the parity of negative signs and the two smallest |v|' (|0| -> 1e10),
// a second pass writes each edge's output, in place over its staged input, then the frame rows
// are copied out coalesced.  Every output equals gather_lds_kernel's: the sign product is exact
// (its value and the sign of a zero product follow from the counts and the parity), the min of
// the others is min1, or min2 for the edge holding min1, NaN if another edge is NaN, capped at
// 1e10 when the row has padding (K > degree - 1).  O(degree) per check instead of O(degree^2),
// and the (K, n) index is not re-read per workgroup.
// One check of a staged frame row r, members gmem[p0 .. p1): the two passes above, in place.  Shared
// by check_group_kernel (member indices from global memory, int32) and check_group_idx_kernel (LDS,
// uint16), so the two cannot drift apart.
template <typename Idx>
__device__ __forceinline__ void check_group_minsum(float *r, const Idx *gmem, int p0, int p1, int K) {
    int zeros = 0, nans = 0, neg = 0, pos = -1;
    float m1 = INFINITY, m2 = INFINITY;
    for (int p = p0; p < p1; ++p) {
        const float v = r[gmem[p]];
        const float sv = v + 1e-10f;
        zeros += sv == 0.0f;
        nans += sv != sv;
        neg ^= sv < 0.0f;
        float a = fabsf(v);
        if (a == 0.0f) a = 1e10f;
        if (a < m1) { m2 = m1; m1 = a; pos = p; }
        else if (a < m2) m2 = a;
    }
    const bool pad = K > p1 - p0 - 1;
    for (int p = p0; p < p1; ++p) {
        const int j = gmem[p];
        const float v = r[j];
        const float sv = v + 1e-10f;
        const int z = zeros - (sv == 0.0f), nn = nans - (sv != sv), ng = neg ^ (sv < 0.0f);
        float m = p == pos ? m2 : m1;
        if (pad) m = fminf(m, 1e10f);
        const float sp = z > 0 ? (ng ? -0.0f : 0.0f) : (ng ? -1.0f : 1.0f);
        r[j] = nn > 0 ? __builtin_nanf("") : sp * m;
    }
}

template <int FPW>
__global__ __launch_bounds__(512) void check_group_kernel(const float *__restrict__ in, int64_t B, int n,
                                                          const int32_t *__restrict__ gptr,
                                                          const int32_t *__restrict__ gmem, int G, int K,
                                                          float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float rows[];  // [FPW][n]
    const int64_t b0 = (int64_t)blockIdx.x * FPW;
    const int nb = (int)min<int64_t>(FPW, B - b0);
    const int total = nb * n;
    const bool vec = (n & 3) == 0 && (reinterpret_cast<uintptr_t>(in + b0 * n) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(out + b0 * n) & 15) == 0;
    if (vec) {
        const float4 *s4 = reinterpret_cast<const float4 *>(in + b0 * n);
        float4 *r4 = reinterpret_cast<float4 *>(rows);
        for (int e = threadIdx.x; e < total / 4; e += blockDim.x) r4[e] = s4[e];
    } else {
        for (int e = threadIdx.x; e < total; e += blockDim.x) rows[e] = in[b0 * n + e];
    }
    __syncthreads();
    for (int w = threadIdx.x; w < G * nb; w += blockDim.x) {
        const int g = w / nb, f = w - g * nb;
        float *r = rows + f * n;
        check_group_minsum(r, gmem, gptr[g], gptr[g + 1], K);
    }
    __syncthreads();
    if (vec) {
        const float4 *r4 = reinterpret_cast<const float4 *>(rows);
        float4 *o4 = reinterpret_cast<float4 *>(out + b0 * n);
        for (int e = threadIdx.x; e < total / 4; e += blockDim.x) o4[e] = r4[e];
    } else {
        for (int e = threadIdx.x; e < total; e += blockDim.x) out[b0 * n + e] = rows[e];
    }
}

// VariableLayer when its (compacted) index is a set of contiguous variable groups (every edge's row
// = the other edges of its variable, ascending, as create_LLR_mapping builds it; detected once in
// Python): out[b][i] = llr[b][i] + the sum of the other members in ascending order --
// gather_sum_kernel's sequence, so the same bits.  The frame row is staged in LDS; per (group,
// frame) one thread walks the members in order, keeping the running prefix P_q = m_s + ... + m_{q-1}
// (the fold every later member starts from) and adding each member's tail, and writes member q's
// sum over m_q in place (the prefix has already taken m_q, and later tails read only members past
// q).  Then the row goes out coalesced with the LLR added (llr + sum).  The gathered kernel re-read
// every group member from global memory per edge and frame (address-bound at 1.7 TB/s).  Measured
// and not kept: one thread per edge (its run bounds or check list through dependent global loads
// per frame: slower), and a persistent double-buffered walk over frames (the degree-23 runs' serial
// chains then sit on every frame's critical path: -24 %).
__global__ __launch_bounds__(512) void var_group_sum_kernel(const float *__restrict__ llr, const float *__restrict__ in,
                                                            int64_t B, int n, const int32_t *__restrict__ gptr, int G,
                                                            float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float rows[];  // [n]
    const int64_t b = blockIdx.x;
    const bool vec = (n & 3) == 0 && (reinterpret_cast<uintptr_t>(in + b * n) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(out + b * n) & 15) == 0 &&
                     (!llr || (reinterpret_cast<uintptr_t>(llr + b * n) & 15) == 0);
    if (vec) {
        const float4 *s4 = reinterpret_cast<const float4 *>(in + b * n);
        float4 *r4 = reinterpret_cast<float4 *>(rows);
        for (int e = threadIdx.x; e < n / 4; e += blockDim.x) r4[e] = s4[e];
    } else {
        for (int e = threadIdx.x; e < n; e += blockDim.x) rows[e] = in[b * n + e];
    }
    __syncthreads();
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
        const int s0 = gptr[g], s1 = gptr[g + 1];
        float P = 0.0f;
        for (int q = s0; q < s1; ++q) {
            const float mq = rows[q];
            float s = P;
            for (int t = q + 1; t < s1; ++t) s += rows[t];
            rows[q] = s;
            P += mq;
        }
    }
    __syncthreads();
    if (vec) {
        const float4 *r4 = reinterpret_cast<const float4 *>(rows);
        float4 *o4 = reinterpret_cast<float4 *>(out + b * n);
        const float4 *l4 = llr ? reinterpret_cast<const float4 *>(llr + b * n) : nullptr;
        for (int e = threadIdx.x; e < n / 4; e += blockDim.x) {
            const float4 s = r4[e];
            if (l4) {
                const float4 l = l4[e];
                o4[e] = make_float4(l.x + s.x, l.y + s.y, l.z + s.z, l.w + s.w);
            } else {
                o4[e] = s;
            }
        }
    } else {
        for (int e = threadIdx.x; e < n; e += blockDim.x) out[b * n + e] = llr ? llr[b * n + e] + rows[e] : rows[e];
    }
}

// check_group_kernel with the check lists in LDS (default): gptr / gmem staged once per workgroup as
// 16-bit words (n < 65536), then F = 4 frames in turn (row in, checks in place, row out).  The
// per-frame kernel's per-member index loads came from global memory, one dependent load per member
// and pass: 93 -> 83 us per BG2 Z = 32 call at B = 4096, +3.6 % on lay-z32 (F = 1 / 2: +3.4 %).
// Measured and not kept: the member indices in registers (-30 %), one thread per edge over its
// check's list (-120 %), a persistent double-buffered walk (-85 %).
template <int F>
__global__ __launch_bounds__(512) void check_group_idx_kernel(const float *__restrict__ in, int64_t B, int n,
                                                              const int32_t *__restrict__ gptr,
                                                              const int32_t *__restrict__ gmem, int G, int K,
                                                              float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float rows[];  // [n] row | [n] u16 gmem | [G + 1] u16 gptr
    uint16_t *gm = reinterpret_cast<uint16_t *>(rows + ((n + 3) & ~3)), *gp = gm + ((n + 7) & ~7);
    for (int e = threadIdx.x; e < n; e += blockDim.x) gm[e] = (uint16_t)gmem[e];
    for (int e = threadIdx.x; e <= G; e += blockDim.x) gp[e] = (uint16_t)gptr[e];
    const bool vec0 = (n & 3) == 0;
    for (int f = 0; f < F; ++f) {
        const int64_t b = (int64_t)blockIdx.x * F + f;
        if (b >= B) break;
        const bool vec = vec0 && (reinterpret_cast<uintptr_t>(in + b * n) & 15) == 0 &&
                         (reinterpret_cast<uintptr_t>(out + b * n) & 15) == 0;
        if (vec) {
            const float4 *s4 = reinterpret_cast<const float4 *>(in + b * n);
            float4 *r4 = reinterpret_cast<float4 *>(rows);
            for (int e = threadIdx.x; e < n / 4; e += blockDim.x) r4[e] = s4[e];
        } else {
            for (int e = threadIdx.x; e < n; e += blockDim.x) rows[e] = in[b * n + e];
        }
        __syncthreads();
        for (int g = threadIdx.x; g < G; g += blockDim.x) {
            check_group_minsum(rows, gm, gp[g], gp[g + 1], K);
        }
        __syncthreads();
        if (vec) {
            const float4 *r4 = reinterpret_cast<const float4 *>(rows);
            float4 *o4 = reinterpret_cast<float4 *>(out + b * n);
            for (int e = threadIdx.x; e < n / 4; e += blockDim.x) o4[e] = r4[e];
        } else {
            for (int e = threadIdx.x; e < n; e += blockDim.x) out[b * n + e] = rows[e];
        }
        __syncthreads();  // the row buffer is reused by the next frame
    }
}

// d in[b][idx[i][k*]] += g[b][i] * sign_product * sgn(v_k*)  (k* = argmin; sgn(0) = 0 covers the
// padded and zero entries, whose |v| was overwritten in place)
__global__ void gather_minsum_bwd_kernel(const float *__restrict__ g, const float *__restrict__ in, int64_t B,
                                         int n_in, const int32_t *__restrict__ idx, int n_out, int K,
                                         const int32_t *__restrict__ argmin, float *__restrict__ gin) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * n_out) return;
    const int64_t b = t / n_out;
    const int i = (int)(t - b * n_out);
    const float *x = in + b * n_in;
    float sp = 1.0f;
    for (int k = 0; k < K; ++k) {
        const int j = idx[(int64_t)k * n_out + i];
        sp = sp * torch_sign((j < 0 ? 0.0f : x[j]) + 1e-10f);
    }
    const int j = idx[(int64_t)argmin[t] * n_out + i];
    if (j < 0) return;
    const float v = x[j];
    const float s = v > 0.0f ? 1.0f : (v < 0.0f ? -1.0f : 0.0f);
    const float d = g[t] * sp * s;
    if (d != 0.0f) atomicAdd(&gin[b * n_in + j], d);
}

// VariableLayer (layers.py:78-125): out[b][i] = llr[b][i] + sum_k msgs[b][idx[i][k]] (0 for -1).
// Padding adds +0.0 to a sum that starts at +0.0 and so is never -0.0: an exact identity.  The
// Python layer therefore moves each row's padding to its end, and the loop stops at the first -1.
__global__ void gather_sum_kernel(const float *__restrict__ llr, const float *__restrict__ msgs, int64_t B, int n_in,
                                  const int32_t *__restrict__ idx, int n_out, int K, float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t ng = (B + kFB - 1) / kFB;
    if (t >= ng * n_out) return;
    const int64_t b0 = (t / n_out) * kFB;
    const int i = (int)(t % n_out);
    const int nb = (int)min<int64_t>(kFB, B - b0);
    float s[kFB];
#pragma unroll
    for (int f = 0; f < kFB; ++f) s[f] = 0.0f;
    for (int k = 0; k < K; ++k) {
        const int j = idx[(int64_t)k * n_out + i];
        if (j < 0) break;  // a row ends at its first padding entry (see ldpc_gather_sum)
#pragma unroll
        for (int f = 0; f < kFB; ++f) {
            if (f >= nb) break;
            s[f] += msgs[(b0 + f) * n_in + j];
        }
    }
#pragma unroll
    for (int f = 0; f < kFB; ++f) {
        if (f >= nb) break;
        const int64_t o = (b0 + f) * n_out + i;
        out[o] = llr ? llr[o] + s[f] : s[f];
    }
}

__global__ void gather_sum_bwd_kernel(const float *__restrict__ g, int64_t B, int n_in,
                                      const int32_t *__restrict__ idx, int n_out, int K, float *__restrict__ gmsgs) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * n_out) return;
    const int64_t b = t / n_out;
    const int i = (int)(t - b * n_out);
    const float d = g[t];
    for (int k = 0; k < K; ++k) {
        const int j = idx[(int64_t)k * n_out + i];
        if (j < 0) break;
        atomicAdd(&gmsgs[b * n_in + j], d);
    }
}

// ResidualLayer (layers.py:143-168): r = llr * w_ch + cm, then r = r + w_res[i] * prev_i, i < D
struct ResArgs {
    const float *llr, *w_ch, *cm, *w_res;
    const float *prev[8];
    int D, n;
    int64_t total;
};

__global__ void residual_kernel(ResArgs A, float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.total) return;
    float r = A.llr[t] * A.w_ch[t % A.n];
    r = r + A.cm[t];
    for (int i = 0; i < A.D; ++i) r = r + A.w_res[i] * A.prev[i][t];
    out[t] = r;
}

// the same per element, n % 4 == 0 and 16-byte aligned rows: one float4 per thread, frames on
// blockIdx.y (no 64-bit modulo per element; 114 -> 95 us per BG2 Z = 32 call at B = 4096)
template <int D>
__global__ void residual4_kernel(ResArgs A, float *__restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x, n4 = A.n >> 2;
    if (c >= n4) return;
    const int64_t t = (int64_t)blockIdx.y * n4 + c;
    const float4 l = reinterpret_cast<const float4 *>(A.llr)[t], w = reinterpret_cast<const float4 *>(A.w_ch)[c];
    const float4 m = reinterpret_cast<const float4 *>(A.cm)[t];
    float4 r = make_float4(l.x * w.x, l.y * w.y, l.z * w.z, l.w * w.w);
    r = make_float4(r.x + m.x, r.y + m.y, r.z + m.z, r.w + m.w);
#pragma unroll
    for (int i = 0; i < D; ++i) {
        const float wr = A.w_res[i];
        const float4 p = reinterpret_cast<const float4 *>(A.prev[i])[t];
        r = make_float4(r.x + wr * p.x, r.y + wr * p.y, r.z + wr * p.z, r.w + wr * p.w);
    }
    reinterpret_cast<float4 *>(out)[t] = r;
}

// grads: g_cm = g; g_prev_i = w_res[i] g; g_w_ch[n] = sum_b g llr; g_w_res[i] = sum g prev_i
struct ResBwd {
    ResArgs A;
    const float *g;
    float *g_prev[8];
    float *g_w_ch, *g_w_res, *g_llr;
    int64_t B;
};

__global__ void residual_bwd_kernel(ResBwd P) {
    const ResArgs &A = P.A;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float part[8] = {};
    if (t < A.total) {
        const float g = P.g[t];
        const int n = (int)(t % A.n);
        if (P.g_llr) P.g_llr[t] = g * A.w_ch[n];
        if (P.g_w_ch) atomicAdd(&P.g_w_ch[n], g * A.llr[t]);
        for (int i = 0; i < A.D; ++i) {
            if (P.g_prev[i]) P.g_prev[i][t] = A.w_res[i] * g;
            part[i] = g * A.prev[i][t];
        }
    }
    // w_res: wave reduction, one atomic per wave and residual term
    for (int i = 0; i < A.D; ++i) {
        float s = part[i];
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if ((threadIdx.x & 63) == 0 && P.g_w_res) atomicAdd(&P.g_w_res[i], s);
    }
}

// OutputLayer (layers.py:180-208): soft = sigmoid(final + llr); loss = max over n of
// BCE(soft, gt) (torch clamps log at -100), argmax kept for the backward
__global__ __launch_bounds__(256) void output_layer_kernel(const float *__restrict__ fin, const float *__restrict__ llr,
                                                           const float *__restrict__ gt, int n,
                                                           float *__restrict__ soft, float *__restrict__ maxloss,
                                                           int32_t *__restrict__ argmax) {
    __shared__ float sv[256];
    __shared__ int si[256];
    const int64_t b = blockIdx.x;
    float best = -INFINITY;
    int bi = 0;
    bool have = false;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int64_t t = b * n + i;
        const float p = 1.0f / (1.0f + expf(-(fin[t] + llr[t])));
        soft[t] = p;
        if (gt) {
            const float y = gt[t];
            // ATen binary_cross_entropy: (y - 1) max(log1p(-p), -100) - y max(log(p), -100)
            const float l = (y - 1.0f) * fmaxf(log1pf(-p), -100.0f) - y * fmaxf(logf(p), -100.0f);
            if (!have || l > best || (isnan(l) && !isnan(best))) {
                best = l;
                bi = i;
                have = true;
            }
        }
    }
    if (!gt) return;
    sv[threadIdx.x] = have ? best : -INFINITY;
    si[threadIdx.x] = have ? bi : 0x7fffffff;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (threadIdx.x < off) {
            const float a = sv[threadIdx.x], c = sv[threadIdx.x + off];
            const int ia = si[threadIdx.x], ic = si[threadIdx.x + off];
            // larger wins; NaN wins; ties -> smaller index (first occurrence)
            const bool take = (isnan(c) && !isnan(a)) || (!isnan(a) && c > a) || (c == a && ic < ia) ||
                              (isnan(c) && isnan(a) && ic < ia);
            if (take) {
                sv[threadIdx.x] = c;
                si[threadIdx.x] = ic;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        maxloss[b] = sv[0];
        argmax[b] = si[0];
    }
}

// g_final = g_llr = (g_soft + [i == argmax] g_loss[b] (p - y) / max((1 - p) p, 1e-12)) (1 - p) p
__global__ void output_layer_bwd_kernel(const float *__restrict__ soft, const float *__restrict__ gt,
                                        const float *__restrict__ g_soft, const float *__restrict__ g_loss,
                                        const int32_t *__restrict__ argmax, int64_t B, int n,
                                        float *__restrict__ g_z) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * n) return;
    const int64_t b = t / n;
    const int i = (int)(t - b * n);
    const float p = soft[t];
    float gp = g_soft ? g_soft[t] : 0.0f;  // BCE backward: g (p - y) / max((1 - p) p, 1e-12)
    if (g_loss && gt && argmax[b] == i) gp += g_loss[b] * (p - gt[t]) / fmaxf((1.0f - p) * p, 1e-12f);
    g_z[t] = gp * (1.0f - p) * p;  // sigmoid backward: g (1 - y) y
}

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace
}  // namespace ldpc

using namespace ldpc;

extern "C" int ldpc_gather_minsum(const float *d_in, int64_t B, int n_in, const int32_t *d_idx, int n_out, int K,
                                  float *d_out, int32_t *d_argmin, void *stream) {
    if (B < 0 || n_in <= 0 || n_out < 0 || K <= 0) return fail(LDPC_EINVAL, "bad gather dimensions");
    if (!B || !n_out) return LDPC_OK;
    if (!d_in || !d_idx || !d_out) return fail(LDPC_EINVAL, "NULL tensor");
    if (const int fpw = gather_fpw(n_in))
        return launch_gather_lds<true>(fpw, d_in, nullptr, B, n_in, d_idx, n_out, K, d_out, d_argmin,
                                       static_cast<hipStream_t>(stream));
    hipLaunchKernelGGL(gather_minsum_kernel, grid_for((B + kFB - 1) / kFB * n_out), dim3(256), 0,
                       static_cast<hipStream_t>(stream), d_in,
                       B, n_in, d_idx, n_out, K, d_out, d_argmin);
    LDPC_CHECK_LAUNCH("gather_minsum_kernel");
    return LDPC_OK;
}

extern "C" int ldpc_check_groups_minsum(const float *d_in, int64_t B, int n, const int32_t *d_gptr,
                                        const int32_t *d_gmem, int G, int K, float *d_out, void *stream) {
    if (B < 0 || n <= 0 || G < 0 || K <= 0) return fail(LDPC_EINVAL, "bad check-group dimensions");
    if (!B || !G) return LDPC_OK;
    if (!d_in || !d_gptr || !d_gmem || !d_out) return fail(LDPC_EINVAL, "NULL tensor");
    // one frame per workgroup by default: 4 workgroups per CU overlap staging with compute
    // (+1.8 % on lay-z32 over 2 frames; 4 frames, one workgroup per CU, -19 %)
    static const int idx_f = [] {  // LDPC_CHECK_IDX_F=0: the per-frame kernel (A/B); 1 / 2 / 4 frames per workgroup
        const char *e = std::getenv("LDPC_CHECK_IDX_F");
        return e ? std::atoi(e) : 4;
    }();
    if (idx_f > 0 && n < 65536 && G < 65536) {
        const size_t lds = ((size_t)((n + 3) & ~3)) * 4 + ((size_t)((n + 7) & ~7) + G + 1) * 2;
        if (lds <= 64 * 1024) {
            hipStream_t s = static_cast<hipStream_t>(stream);
            const int F = idx_f >= 4 ? 4 : idx_f >= 2 ? 2 : 1;
            const dim3 grid((unsigned)((B + F - 1) / F));
            if (F == 4) hipLaunchKernelGGL(check_group_idx_kernel<4>, grid, dim3(512), lds, s, d_in, B, n, d_gptr, d_gmem, G, K, d_out);
            else if (F == 2) hipLaunchKernelGGL(check_group_idx_kernel<2>, grid, dim3(512), lds, s, d_in, B, n, d_gptr, d_gmem, G, K, d_out);
            else hipLaunchKernelGGL(check_group_idx_kernel<1>, grid, dim3(512), lds, s, d_in, B, n, d_gptr, d_gmem, G, K, d_out);
            LDPC_CHECK_LAUNCH("check_group_idx_kernel");
            return LDPC_OK;
        }
    }
    // one frame per workgroup (2, 4 and 8 frames per workgroup measured slower, profiles/r04)
    if (!gather_fpw(n)) return fail(LDPC_EUNSUPPORTED, "check-group rows do not fit LDS");
    const size_t lds = (size_t)n * 4;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (lds > 64 * 1024)
        LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(check_group_kernel<1>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(check_group_kernel<1>, dim3((unsigned)B), dim3(512), lds, s, d_in, B, n, d_gptr, d_gmem, G, K, d_out);
    LDPC_CHECK_LAUNCH("check_group_kernel");
    return LDPC_OK;
}

extern "C" int ldpc_gather_minsum_backward(const float *d_grad_out, const float *d_in, int64_t B, int n_in,
                                           const int32_t *d_idx, int n_out, int K, const int32_t *d_argmin,
                                           float *d_grad_in, void *stream) {
    if (B < 0 || n_in <= 0 || n_out < 0 || K <= 0) return fail(LDPC_EINVAL, "bad gather dimensions");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (d_grad_in) LDPC_HIP(hipMemsetAsync(d_grad_in, 0, (size_t)B * n_in * 4, s));
    if (!B || !n_out) return LDPC_OK;
    if (!d_grad_out || !d_in || !d_idx || !d_argmin || !d_grad_in) return fail(LDPC_EINVAL, "NULL tensor");
    hipLaunchKernelGGL(gather_minsum_bwd_kernel, grid_for(B * n_out), dim3(256), 0, s, d_grad_out, d_in, B, n_in, d_idx,
                       n_out, K, d_argmin, d_grad_in);
    LDPC_CHECK_LAUNCH("gather_minsum_bwd_kernel");
    return LDPC_OK;
}

extern "C" int ldpc_gather_sum(const float *d_llr, const float *d_msgs, int64_t B, int n_in, const int32_t *d_idx,
                               int n_out, int K, float *d_out, void *stream) {
    if (B < 0 || n_in <= 0 || n_out < 0 || K <= 0) return fail(LDPC_EINVAL, "bad gather dimensions");
    if (!B || !n_out) return LDPC_OK;
    if (!d_msgs || !d_idx || !d_out) return fail(LDPC_EINVAL, "NULL tensor");
    // (an LDS-staged form of this sum, as the min-sum gather's, measured 12 % slower at BG2 Z=32: the
    // index, K = 22 with rows ending early, is then read once per 2 frames instead of 4)
    hipLaunchKernelGGL(gather_sum_kernel, grid_for((B + kFB - 1) / kFB * n_out), dim3(256), 0,
                       static_cast<hipStream_t>(stream), d_llr,
                       d_msgs, B, n_in, d_idx, n_out, K, d_out);
    LDPC_CHECK_LAUNCH("gather_sum_kernel");
    return LDPC_OK;
}

extern "C" int ldpc_var_groups_sum(const float *d_llr, const float *d_msgs, int64_t B, int n, const int32_t *d_gptr,
                                   int G, float *d_out, void *stream) {
    if (B < 0 || n <= 0 || G <= 0) return fail(LDPC_EINVAL, "bad variable-group dimensions");
    if (!B) return LDPC_OK;
    if (!d_msgs || !d_gptr || !d_out) return fail(LDPC_EINVAL, "NULL tensor");
    if (d_out == d_msgs || (d_llr && d_out == d_llr)) return fail(LDPC_EINVAL, "output aliases an input");
    const size_t lds = (size_t)n * 4;  // one frame per workgroup (staging overlaps across workgroups)
    if (lds > 64 * 1024) return fail(LDPC_EUNSUPPORTED, "variable-group rows do not fit LDS");
    hipLaunchKernelGGL(var_group_sum_kernel, dim3((unsigned)B), dim3(512), lds, static_cast<hipStream_t>(stream), d_llr,
                       d_msgs, B, n, d_gptr, G, d_out);
    LDPC_CHECK_LAUNCH("var_group_sum_kernel");
    return LDPC_OK;
}

extern "C" int ldpc_gather_sum_backward(const float *d_grad_out, int64_t B, int n_in, const int32_t *d_idx, int n_out,
                                        int K, float *d_grad_msgs, void *stream) {
    if (B < 0 || n_in <= 0 || n_out < 0 || K <= 0) return fail(LDPC_EINVAL, "bad gather dimensions");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (d_grad_msgs) LDPC_HIP(hipMemsetAsync(d_grad_msgs, 0, (size_t)B * n_in * 4, s));
    if (!B || !n_out) return LDPC_OK;
    if (!d_grad_out || !d_idx || !d_grad_msgs) return fail(LDPC_EINVAL, "NULL tensor");
    hipLaunchKernelGGL(gather_sum_bwd_kernel, grid_for(B * n_out), dim3(256), 0, s, d_grad_out, B, n_in, d_idx, n_out,
                       K, d_grad_msgs);
    LDPC_CHECK_LAUNCH("gather_sum_bwd_kernel");
    return LDPC_OK;
}

extern "C" int ldpc_residual(const float *d_llr, const float *d_w_ch, const float *d_cm, const float *d_w_res,
                             const float *const *h_prev, int depth, int64_t B, int n, float *d_out, void *stream) {
    if (B < 0 || n <= 0 || depth < 0 || depth > 8) return fail(LDPC_EINVAL, "bad residual arguments (depth <= 8)");
    if (!B) return LDPC_OK;
    ResArgs A{};
    A.llr = d_llr; A.w_ch = d_w_ch; A.cm = d_cm; A.w_res = d_w_res; A.D = depth; A.n = n; A.total = B * n;
    for (int i = 0; i < depth; ++i) A.prev[i] = h_prev[i];
    hipStream_t s = static_cast<hipStream_t>(stream);
    bool vec = (n & 3) == 0 && B <= 65535;
    for (const void *q : {(const void *)d_llr, (const void *)d_w_ch, (const void *)d_cm, (const void *)d_out})
        vec = vec && (reinterpret_cast<uintptr_t>(q) & 15) == 0;
    for (int i = 0; i < depth; ++i) vec = vec && (reinterpret_cast<uintptr_t>(h_prev[i]) & 15) == 0;
    if (vec && depth <= 4) {
        const dim3 grid((unsigned)((n / 4 + 255) / 256), (unsigned)B);
        switch (depth) {
            case 0: hipLaunchKernelGGL(residual4_kernel<0>, grid, dim3(256), 0, s, A, d_out); break;
            case 1: hipLaunchKernelGGL(residual4_kernel<1>, grid, dim3(256), 0, s, A, d_out); break;
            case 2: hipLaunchKernelGGL(residual4_kernel<2>, grid, dim3(256), 0, s, A, d_out); break;
            case 3: hipLaunchKernelGGL(residual4_kernel<3>, grid, dim3(256), 0, s, A, d_out); break;
            default: hipLaunchKernelGGL(residual4_kernel<4>, grid, dim3(256), 0, s, A, d_out); break;
        }
        LDPC_CHECK_LAUNCH("residual4_kernel");
        return LDPC_OK;
    }
    hipLaunchKernelGGL(residual_kernel, grid_for(A.total), dim3(256), 0, s, A, d_out);
    LDPC_CHECK_LAUNCH("residual_kernel");
    return LDPC_OK;
}

extern "C" int ldpc_residual_backward(const float *d_grad, const float *d_llr, const float *d_w_ch,
                                      const float *d_w_res, const float *const *h_prev, int depth, int64_t B, int n,
                                      float *d_grad_llr, float *d_grad_w_ch, float *d_grad_w_res,
                                      float *const *h_grad_prev, void *stream) {
    if (B < 0 || n <= 0 || depth < 0 || depth > 8) return fail(LDPC_EINVAL, "bad residual arguments (depth <= 8)");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (d_grad_w_ch) LDPC_HIP(hipMemsetAsync(d_grad_w_ch, 0, (size_t)n * 4, s));
    if (d_grad_w_res && depth) LDPC_HIP(hipMemsetAsync(d_grad_w_res, 0, (size_t)depth * 4, s));
    if (!B) return LDPC_OK;
    ResBwd P{};
    P.A.llr = d_llr; P.A.w_ch = d_w_ch; P.A.w_res = d_w_res; P.A.D = depth; P.A.n = n; P.A.total = B * n;
    for (int i = 0; i < depth; ++i) {
        P.A.prev[i] = h_prev[i];
        P.g_prev[i] = h_grad_prev ? h_grad_prev[i] : nullptr;
    }
    P.g = d_grad; P.g_w_ch = d_grad_w_ch; P.g_w_res = d_grad_w_res; P.g_llr = d_grad_llr; P.B = B;
    hipLaunchKernelGGL(residual_bwd_kernel, grid_for(P.A.total), dim3(256), 0, s, P);
    LDPC_CHECK_LAUNCH("residual_bwd_kernel");
    return LDPC_OK;
}

extern "C" int ldpc_output_layer(const float *d_final, const float *d_llr, const float *d_gt, int64_t B, int n,
                                 float *d_soft, float *d_max_loss, int32_t *d_argmax, void *stream) {
    if (B < 0 || n <= 0) return fail(LDPC_EINVAL, "bad output-layer dimensions");
    if (!B) return LDPC_OK;
    if (d_gt && (!d_max_loss || !d_argmax)) return fail(LDPC_EINVAL, "loss outputs are NULL");
    hipLaunchKernelGGL(output_layer_kernel, dim3((unsigned)B), dim3(256), 0, static_cast<hipStream_t>(stream), d_final,
                       d_llr, d_gt, n, d_soft, d_max_loss, d_argmax);
    LDPC_CHECK_LAUNCH("output_layer_kernel");
    return LDPC_OK;
}

extern "C" int ldpc_output_layer_backward(const float *d_soft, const float *d_gt, const float *d_grad_soft,
                                          const float *d_grad_loss, const int32_t *d_argmax, int64_t B, int n,
                                          float *d_grad_z, void *stream) {
    if (B < 0 || n <= 0) return fail(LDPC_EINVAL, "bad output-layer dimensions");
    if (!B) return LDPC_OK;
    hipLaunchKernelGGL(output_layer_bwd_kernel, grid_for(B * n), dim3(256), 0, static_cast<hipStream_t>(stream), d_soft,
                       d_gt, d_grad_soft, d_grad_loss, d_argmax, B, n, d_grad_z);
    LDPC_CHECK_LAUNCH("output_layer_bwd_kernel");
    return LDPC_OK;
}
