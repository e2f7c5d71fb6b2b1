// flood_dev.hpp -- device side of the flooding decoders, shared by the flood*.hip translation units.
// (Split out of flood.hip so that its kernel families compile in parallel; see flood.hip for the
// algorithm notes.)
//   LDS-resident flooding min-sum / sum-product decoder for gfx950.
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
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>

#include <utility>

#include "common.hpp"
#include "gen/fixed_codes.hpp"
#include "graph.hpp"

namespace ldpc {

// Shared by the flood translation units (flood*.hip): counter rows, internal early-stop modes
// (see flood_drive) and the workspace views the kernels take.
constexpr int kPartRow = 8;  // uint32 per workgroup row
constexpr int ES_P1 = 3, ES_P2 = 4;

struct EsWs {
    uint64_t *words;   // ES_BATCH: [nwg][max_iter][Nb] ballots
    uint32_t *valid;   // ES_BATCH: [B][nvw] validity bit per iteration
    int nvw;
    uint64_t *cand;    // ES_P1: [nwg][Nb] ballots at t_wg
    int32_t *twg;      // ES_P1: [nwg] t_wg
    int32_t *ctl;      // [0] T = max t_wg  [1] bad  [2] fallback needed
    uint64_t *staged;  // [4] counters of the P2 result (applied by es_finalize_kernel)
};

struct Outs {
    int32_t *iters_out;
    uint32_t *partials;  // [nwg][kPartRow] counter rows (NULL: no counters wanted)
    uint64_t *timeline;  // LDPC_TIMELINE builds only (tools/flood_timeline.py): NULL otherwise
};

// Timeline build (-DLDPC_TIMELINE, tools/build_timeline.sh): lane 0 of every wave of the first
// kTlWgs workgroups stores s_memtime at each phase boundary of the iteration loop -- after the
// init barrier, then per iteration: check phase done, barrier 1 passed, variable phase done,
// barrier 2 passed -- so the waves each barrier waits on can be read off.
constexpr int kTlWgs = 2048, kTlMaxIter = 16, kTlPer = 2 + 4 * kTlMaxIter;

namespace {

// Graph programs are read-only for the kernel's lifetime and indexed by wave-uniform values:
// reading them through the constant address space makes every word a scalar (SMEM) load.
typedef const __attribute__((address_space(4))) int32_t const_i32;
__device__ __forceinline__ int32_t tab(const int32_t *p, int i) { return ((const_i32 *)p)[i]; }

// compile-time loop: f(ic<0>{}), ..., f(ic<N-1>{})
template <int I>
using ic = std::integral_constant<int, I>;
template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F &&f, std::integer_sequence<int, I...>) {
    (f(ic<I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F &&f) {
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}

struct Lane {
    int lane;      // 0..63 = f * Z + k
    int f, k;      // frame within the lane vector, row (or column position) within a block
    int lane4;     // 4 * lane: byte offset of this lane's entry in a slot
    int fz4;       // 4 * f * Z
    int k4;        // 4 * k
    int zmask4;    // 4 * Z - 1 (Z is a power of two)
    int z4;        // 4 * Z
    bool valid;    // the lane's frame exists
    int64_t frame;
    const char *llr_row;  // this lane's frame row (frame 0 for lanes without a frame)
    // byte offset inside a slot of the message on a block with byte shift s4, seen from the
    // variable at position k: row (k - s) mod Z of frame f
    __device__ __forceinline__ int vrot(int s4) const { return fz4 + ((k4 - s4) & zmask4); }
    // byte offset of variable (col, (k + s) mod Z) in an LLR row
    __device__ __forceinline__ int col_off(int col, int s4) const { return col * z4 + ((k4 + s4) & zmask4); }
    __device__ __forceinline__ int Z() const { return z4 >> 2; }
    __device__ __forceinline__ float llr_at(int byte_off) const {
        return *reinterpret_cast<const float *>(llr_row + byte_off);
    }
};

__device__ __forceinline__ float lds_rd(const char *lds, int off) { return *reinterpret_cast<const float *>(lds + off); }

// ds_write_addtid_b32: LDS[M0 + OFF + 4 * lane] = v.  No address VGPR, and half the LDS cycles of a
// ds_write_b32 (MI355X_MICROARCH.md, LDS table: 2 vs 4 per wave-instruction).  M0 must hold the
// LDS base (addtid_begin) and the compiler must not see these stores: callers drain them with
// addtid_end() (s_waitcnt lgkmcnt(0)) before any barrier or LDS read of the same bytes.
__device__ __forceinline__ void addtid_begin(const char *lds) {
    const uint32_t base = (uint32_t)(uintptr_t)lds;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(base) : "memory");
}
template <int OFF>
__device__ __forceinline__ void lds_wr_tid(float v) {
    static_assert(OFF >= 0 && OFF < 65536, "addtid offset is 16 bits");
    asm volatile("ds_write_addtid_b32 %0 offset:%1" : : "v"(v), "i"(OFF) : "memory");
}
__device__ __forceinline__ void addtid_end() { asm volatile("s_waitcnt lgkmcnt(0)" : : : "memory"); }
__device__ __forceinline__ void lds_wr(char *lds, int off, float v) { *reinterpret_cast<float *>(lds + off) = v; }

__device__ __forceinline__ void put_bit(void *bits, int out_dtype, int64_t idx, int bit) {
    if (out_dtype == LDPC_OUT_F32)
        static_cast<float *>(bits)[idx] = bit ? 1.0f : 0.0f;
    else
        static_cast<uint8_t *>(bits)[idx] = (uint8_t)bit;
}

__device__ __forceinline__ bool is_zero_sign(float x) { return !(x > 0.0f || x < 0.0f); }
typedef float f32x2 __attribute__((ext_vector_type(2)));

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

// Fast path of the same update for a row with no zero and no NaN message (every row, in practice;
// a wave takes it when none of its 64 rows has one).  Then torch.sign is +-1, so
//   * the sign parity is the XOR of the sign bits, and the output sign is parity ^ signbit(x);
//   * the two smallest magnitudes are a min/max network (v_min/v_max are exact, NaN-free here);
//   * the excluded minimum is m2 exactly when |x| == m1: a tie at m1 puts m1 in m2 as well, so
//     no first-index bookkeeping is needed.
// Every output is bit-identical to MinSumStats::c2v: +-(alpha * m) with the same alpha * m.
// xor of the messages' bit patterns (its sign bit = the row's sign parity): v_bitop3_b32 with the
// three-input xor table (0x96) takes two messages per instruction (the compiler keeps a chain of
// two-input xors here)
template <int DC, int CAP>
__device__ __forceinline__ uint32_t sign_parity_n(const float (&v)[CAP]) {
    static_assert(DC <= CAP, "row longer than its buffer");
    uint32_t p = __float_as_uint(v[0]);
#pragma unroll
    for (int e = 1; e + 1 < DC; e += 2)
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(p) : "v"(p), "v"(v[e]), "v"(v[e + 1]));
    if constexpr (DC % 2 == 0) p ^= __float_as_uint(v[DC - 1]);
    return p;
}

// m2 = median(m1, |x|, m2) then m1 = min(m1, |x|): the two smallest magnitudes of a row with no
// NaN (v_min / v_med3 with |x| as a source modifier; fminf would add a NaN-quieting v_max)
// -inf in a VGPR the compiler cannot see through: med3(m, |x|, -inf) = min(m, |x|) for non-NaN
// operands, and an opaque third operand keeps the compiler from turning it back into a
// canonicalising fminf
// (an SGPR: one scalar operand per v_med3 is within the constant-bus limit)
__device__ __forceinline__ float opaque_sf(float v) {
    asm volatile("" : "+s"(v));
    return v;
}
// a uniform constant held in a VGPR: a VALU op with an SGPR source issues at half rate
__device__ __forceinline__ uint32_t opaque_vu(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ float opaque_vf(float v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ void two_min_step(float &m1, float &m2, float x, float ninf) {
    // builtins, not inline asm: a VALU reading a VGPR written by inline asm gets a conservative
    // s_nop from the hazard recognizer (one per edge in the check phase)
    m2 = __builtin_amdgcn_fmed3f(m1, fabsf(x), m2);
    m1 = __builtin_amdgcn_fmed3f(m1, fabsf(x), ninf);
}

// The two smallest magnitudes of a row with no NaN, three messages per step: the smallest and the
// middle of a triple are one v_minimum3 and one v_med3 (|x| as source modifiers), and a sorted
// pair (m1 <= m2) absorbs a sorted pair (t1 <= t2) as m1' = min(m1, t1),
// m2' = min(max(m1, t1), m2, t2) -- 5 ops per further triple, 2 per leftover message, against 2 per
// message for the running med3 / min chain (BG2: 217 instead of 310 of these half-rate ops per
// base-graph iteration).  Every op returns one of its inputs: the pair (m1, m2) is bit-identical.
// minimum / maximum (IEEE, NaN-propagating) need no canonicalising v_max, unlike fminf.
__device__ __forceinline__ float vmin(float a, float b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ float vmax(float a, float b) { return __builtin_elementwise_maximum(a, b); }
template <int DC, int CAP>
__device__ __forceinline__ void two_smallest(const float (&v)[CAP], float &m1, float &m2, float ninf) {
    static_assert(DC <= CAP, "row longer than its buffer");
    if constexpr (DC == 1) {
        m1 = fabsf(v[0]);
    } else if constexpr (DC == 2) {
        m1 = vmin(fabsf(v[0]), fabsf(v[1]));
        m2 = vmax(fabsf(v[0]), fabsf(v[1]));
    } else {
        m1 = vmin(vmin(fabsf(v[0]), fabsf(v[1])), fabsf(v[2]));
        m2 = __builtin_amdgcn_fmed3f(fabsf(v[0]), fabsf(v[1]), fabsf(v[2]));
        constexpr int NT = (DC - 3) / 3;  // further whole triples
        sfor<NT>([&](auto q) {
            constexpr int B0 = 3 + 3 * decltype(q)::value;
            const float a = fabsf(v[B0]), b = fabsf(v[B0 + 1]), c = fabsf(v[B0 + 2]);
            const float t1 = vmin(vmin(a, b), c), t2 = __builtin_amdgcn_fmed3f(a, b, c);
            m2 = vmin(vmin(vmax(m1, t1), m2), t2);
            m1 = vmin(m1, t1);
        });
        sfor<DC - 3 - 3 * NT>([&](auto q) { two_min_step(m1, m2, v[3 + 3 * NT + decltype(q)::value], ninf); });
    }
}

// lane mask of |x| == m (v_cmp_eq_f32 into an SGPR pair) and a select by it; volatile so that the
// issue order written by the caller is kept
__device__ __forceinline__ uint64_t cmp_eq_abs(float x, float m) {
    uint64_t k;
    asm volatile("v_cmp_eq_f32_e64 %0, |%1|, %2" : "=s"(k) : "v"(x), "v"(m));
    return k;
}
__device__ __forceinline__ uint32_t cndmask(uint32_t if0, uint32_t if1, uint64_t k) {
    uint32_t r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(k));
    return r;
}

struct MinSumFast {
    float m1 = INFINITY, m2 = INFINITY;
    uint32_t par = 0;
    bool special = false;  // a zero or NaN message: the row needs MinSumStats
    __device__ __forceinline__ void add(float x) {
        const float a = fabsf(x);
        special |= is_zero_sign(x);
        // m2 = min(m2, max(m1, a)) = median(m1, a, m2) since m1 <= m2: one v_med3_f32 with |x|
        // as a source modifier.  m1 = min(m1, |x|) as one v_min_f32 in asm: fminf (and a med3
        // with -inf, which the compiler turns back into it) adds a NaN-quieting v_max per edge,
        // and this path never sees a NaN (special -> MinSumStats).
        m2 = __builtin_amdgcn_fmed3f(m1, a, m2);
        asm("v_min_f32 %0, %1, |%2|" : "=v"(m1) : "v"(m1), "v"(x));
    }
    // s1 / s2 = |alpha m1| / |alpha m2| with the row's sign parity in the sign bit (sel_words);
    // the message's own sign bit is xored back out: out = (x & SIGN) ^ sel (one v_bitop3)
    __device__ __forceinline__ float c2v(float x, uint32_t s1, uint32_t s2) const {
        const uint32_t sel = fabsf(x) == m1 ? s2 : s1;
        return __uint_as_float((__float_as_uint(x) & 0x80000000u) ^ sel);
    }
    __device__ __forceinline__ void sel_words(float alpha, uint32_t &s1, uint32_t &s2) const {
        const uint32_t ps = par & 0x80000000u;
        s1 = __float_as_uint(fabsf(alpha * m1)) | ps;
        s2 = __float_as_uint(fabsf(alpha * m2)) | ps;
    }
};

// float32 tanh / atanh, branch-free, a few ulp (the reference calls torch-CPU's float32 SLEEF
// versions, 1 ulp; neither is correctly rounded).  Small arguments: the odd minimax polynomials of
// the Cephes float library (tanh |y| < 0.625, atanh |p| < 0.5; 1.1 and 1.4 ulp in float
// arithmetic); larger ones: the exp / log forms on the hardware v_exp_f32 / v_log_f32 / v_rcp_f32.
// Measured against double: <= 1.5e-7 relative with exact exp2/log2/rcp.  Saturation as in the
// reference: tanh rounds to +-1 for |y| >~ 9, and 2 atanh(+-1) = +-inf.  ~16 + ~18 VALU per edge
// against ~130 for the ROCm libm calls (and 4x that for double).
__device__ __forceinline__ float tanh_half(float v) {
    const float y = v * 0.5f;  // exact, = v / 2
    const float a = fabsf(y), z = y * y;
    float p = fmaf(-5.70498872745e-3f, z, 2.06390887954e-2f);
    p = fmaf(p, z, -5.37397155531e-2f);
    p = fmaf(p, z, 1.33314422036e-1f);
    p = fmaf(p, z, -3.33332819422e-1f);
    const float small = fmaf(p * z, y, y);
    const float e = __builtin_amdgcn_exp2f(a * 2.88539008177792681f);  // exp(2a)
    const float big = fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
    return a < 0.625f ? small : copysignf(big, y);
}
__device__ __forceinline__ float two_atanh(float x) {
    const float z = x * x;
    float p = fmaf(1.81740078349e-1f, z, 8.24370301058e-2f);
    p = fmaf(p, z, 1.46691431730e-1f);
    p = fmaf(p, z, 1.99782164500e-1f);
    p = fmaf(p, z, 3.33337300303e-1f);
    const float small = 2.0f * fmaf(p * z, x, x);
    // log((1 + x) / (1 - x)); 1 - x is exact for x >= 0.5, (1 + x) * rcp(0) = +inf at x = 1
    const float r = (1.0f + x) * __builtin_amdgcn_rcpf(1.0f - x);
    const float big = __builtin_amdgcn_logf(r) * 0.693147180559945309f;
    return fabsf(x) < 0.5f ? small : big;
}

struct Ctx {
    FloodTables T;
    char *lds;
    uint64_t *words;  // ES: Nb decision ballots + 1 invalid-lane word (in LDS)
    uint32_t *flag;   // LDS: sticky "a v2c may be NaN" flag of the fixed kernel's fast check path
    float alpha;
    int out_dtype;
    void *bits;
    bool direct_bits;  // mode 0, final iteration: write decisions straight to HBM
    bool ballots;      // ES: record decisions as ballots
};

// rotate each z-bit segment of w left by s (0 <= s < z; z a power of two dividing 64), given
// rep1 = the word with a 1 at the bottom of every segment (scalar ops: w and rep1 are uniform)
__device__ __forceinline__ uint64_t seg_rotl(uint64_t w, int s, int z, uint64_t rep1) {
    if (s == 0) return w;
    if (z >= 64) return (w << s) | (w >> (64 - s));
    const uint64_t low = ((1ull << (z - s)) - 1ull) * rep1;  // the low z - s bits of every segment
    return ((w & low) << s) | ((w & ~low) >> (z - s));
}

// decision of variable (col, (k + s) mod Z) computed on the lane of check row k
__device__ __forceinline__ void ext_decision(const Ctx &C, const Lane &L, int col, int s4, float app,
                                             int &errs) {
    const int bit = app < 0.0f;  // NaN < 0 is false -> 0 (traditional_decoders.py:252)
    if (C.direct_bits && L.valid) {
        // the empty asm keeps the (final-iteration only) 64-bit output address from being
        // hoisted out of the iteration loop, where it would hold registers for nothing
        int64_t fr = L.frame;
        int k4 = L.k4;
        asm volatile("" : "+v"(fr), "+v"(k4));
        put_bit(C.bits, C.out_dtype, fr * C.T.N + (col * L.z4 + ((k4 + s4) & L.zmask4)) / 4, bit);
        errs += bit;
    }
    if (C.ballots) {
        // lane f*Z + k holds variable (k + s) mod Z: rotate every Z-bit segment of the ballot left
        // by s (uniform, scalar) so that bit f*Z + t is variable t, as in var_decision
        const uint64_t w = seg_rotl(__ballot(bit), s4 >> 2, C.T.Z, C.T.rep1);
        if (L.lane == 0) C.words[col] = w;
    }
}

__device__ __forceinline__ void var_decision(const Ctx &C, const Lane &L, int col, float app, int &errs) {
    const int bit = app < 0.0f;
    if (C.direct_bits && L.valid) {
        int64_t fr = L.frame;
        int k = L.k;
        asm volatile("" : "+v"(fr), "+v"(k));
        put_bit(C.bits, C.out_dtype, fr * C.T.N + (int64_t)col * L.Z() + k, bit);
        errs += bit;
    }
    if (C.ballots) {
        const uint64_t w = __ballot(bit);
        if (L.lane == 0) C.words[col] = w;
    }
}

// ---------------------------------------------------------------- check node update
// prog points at the row's first edge word (uniform); DC compile-time.
template <int ALGO, int DC>
__device__ __forceinline__ void check_task(const Ctx &C, const Lane &L, const int32_t *prog, int &errs) {
    float v[DC];
    int32_t w[DC];
#pragma unroll
    for (int e = 0; e < DC; ++e) {
        w[e] = tab(prog, e);
        const int lo = w[e] & kLowMask, s4 = (w[e] >> kShiftBit) & 0xFF;
        v[e] = w[e] < 0 ? L.llr_at(L.col_off(lo, s4)) : lds_rd(C.lds, lo + L.lane4);
    }
    auto emit = [&](int e, float o) {
        const int lo = w[e] & kLowMask;
        if (w[e] >= 0)
            lds_wr(C.lds, lo + L.lane4, o);
        else if (C.direct_bits || C.ballots)  // degree-1 variable: APP = llr.clone() + c2v
            ext_decision(C, L, lo, (w[e] >> kShiftBit) & 0xFF, v[e] + o, errs);
    };
    if constexpr (ALGO == LDPC_ALGO_MINSUM) {
        MinSumFast fs;
#pragma unroll
        for (int e = 0; e < DC; ++e) fs.add(v[e]);
        fs.par = sign_parity_n<DC>(v);
        if (!__any(fs.special)) {  // wave-uniform
            uint32_t s1, s2;
            fs.sel_words(C.alpha, s1, s2);
#pragma unroll
            for (int e = 0; e < DC; ++e) emit(e, fs.c2v(v[e], s1, s2));
        } else {
            MinSumStats st;
#pragma unroll
            for (int e = 0; e < DC; ++e) st.add(e, v[e]);
#pragma unroll
            for (int e = 0; e < DC; ++e) emit(e, st.c2v(e, v[e], C.alpha));
        }
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

// Any degree: messages re-read instead of kept in registers (O(dc^2) reads; used past the
// unrolled range).  In-place is safe in ascending e: slot e is overwritten after P_{e+1} used it.
template <int ALGO>
__device__ __forceinline__ void check_task_dyn(const Ctx &C, const Lane &L, const int32_t *prog, int dc,
                                               int &errs) {
    auto rd = [&](int e) -> float {
        const int32_t w = tab(prog, e);
        const int lo = w & kLowMask;
        return w < 0 ? L.llr_at(L.col_off(lo, (w >> kShiftBit) & 0xFF)) : lds_rd(C.lds, lo + L.lane4);
    };
    auto wr = [&](int e, float in, float out) {
        const int32_t w = tab(prog, e);
        const int lo = w & kLowMask;
        if (w >= 0)
            lds_wr(C.lds, lo + L.lane4, out);
        else if (C.direct_bits || C.ballots)
            ext_decision(C, L, lo, (w >> kShiftBit) & 0xFF, in + out, errs);
    };
    if constexpr (ALGO == LDPC_ALGO_MINSUM) {
        MinSumStats st;
        for (int e = 0; e < dc; ++e) st.add(e, rd(e));
        for (int e = 0; e < dc; ++e) {
            const float x = rd(e);
            wr(e, x, st.c2v(e, x, C.alpha));
        }
    } else {
        float P = 1.0f;
        for (int e = 0; e < dc; ++e) {
            const float x = rd(e);
            float rr = P;
            for (int q = e + 1; q < dc; ++q) rr = rr * tanh_half(rd(q));
            const float t = tanh_half(x);
            wr(e, x, two_atanh(rr));
            P = P * t;
        }
    }
}

// ---------------------------------------------------------------- variable node update
// Variable update (traditional_decoders.py:235-250): v2c_e = llr + sum_{e'!=e} c_e' added in
// ascending check order, i.e. acc[e] = P_e (prefix) followed by c_{e+1}, c_{e+2}, ...;
// the APP is P_DV = llr + c_0 + ... + c_{DV-1}.
template <int DV>
__device__ __forceinline__ void var_task(const Ctx &C, const Lane &L, const int32_t *prog, int col, bool write,
                                         int &errs) {
    float P = L.llr_at(col * L.z4 + L.k4);
    if constexpr (DV > 0) {
        float acc[DV];
        int off[DV];
#pragma unroll
        for (int j = 0; j < DV; ++j) {
            const int32_t w = tab(prog, j);
            off[j] = (w & kLowMask) + L.vrot((w >> kShiftBit) & 0xFF);
            const float c = lds_rd(C.lds, off[j]);
#pragma unroll
            for (int e = 0; e < j; ++e) acc[e] = acc[e] + c;
            acc[j] = P;
            P = P + c;
        }
        if (write) {
#pragma unroll
            for (int e = 0; e < DV; ++e) lds_wr(C.lds, off[e], acc[e]);
        }
    }
    if (C.direct_bits || C.ballots) var_decision(C, L, col, P, errs);
}

__device__ __forceinline__ void var_task_dyn(const Ctx &C, const Lane &L, const int32_t *prog, int dv, int col,
                                             bool write, int &errs) {
    auto off = [&](int e) {
        const int32_t w = tab(prog, e);
        return (w & kLowMask) + L.vrot((w >> kShiftBit) & 0xFF);
    };
    float P = L.llr_at(col * L.z4 + L.k4);
    for (int e = 0; e < dv; ++e) {
        const int o = off(e);
        const float cp = lds_rd(C.lds, o);
        float acc = P;
        for (int q = e + 1; q < dv; ++q) acc = acc + lds_rd(C.lds, off(q));
        P = P + cp;
        if (write) lds_wr(C.lds, o, acc);
    }
    if (C.direct_bits || C.ballots) var_decision(C, L, col, P, errs);
}

// degrees with unrolled register code; larger ones take the *_dyn paths
#define LDPC_DC_CASES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12)
#define LDPC_DV_CASES(X) \
    X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) \
    X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24)

// run this wave's check program
template <int ALGO>
__device__ __forceinline__ void check_phase(const Ctx &C, const Lane &L, int wave, int &errs) {
    const int p1 = tab(C.T.prog_ptr, wave + 1);
    for (int pc = tab(C.T.prog_ptr, wave); pc < p1;) {
        const int dc = tab(C.T.chk_prog, pc);
        const int32_t *prog = C.T.chk_prog + pc + 1;
        switch (dc) {
            case 0: break;
#define X(n) case n: check_task<ALGO, n>(C, L, prog, errs); break;
            LDPC_DC_CASES(X)
#undef X
            default: check_task_dyn<ALGO>(C, L, prog, dc, errs); break;
        }
        pc += 1 + dc;
    }
}

__device__ __forceinline__ void var_phase(const Ctx &C, const Lane &L, int wave, bool write, int &errs) {
    const int W1 = C.T.W + 1;
    const int p1 = tab(C.T.prog_ptr, W1 + wave + 1);
    for (int pc = tab(C.T.prog_ptr, W1 + wave); pc < p1;) {
        const int h = tab(C.T.var_prog, pc);
        const int dv = h & 0xFF, col = h >> 8;
        const int32_t *prog = C.T.var_prog + pc + 1;
        switch (dv) {
            case 0: var_task<0>(C, L, prog, col, write, errs); break;
#define X(n) case n: var_task<n>(C, L, prog, col, write, errs); break;
            LDPC_DV_CASES(X)
#undef X
            default: var_task_dyn(C, L, prog, dv, col, write, errs); break;
        }
        pc += 1 + dv;
    }
}

// v2c <- llr on every slot (traditional_decoders.py:199-202)
__device__ __forceinline__ void init_phase(const Ctx &C, const Lane &L, int wave) {
    const int W1 = C.T.W + 1;
    const int p1 = tab(C.T.prog_ptr, W1 + wave + 1);
    for (int pc = tab(C.T.prog_ptr, W1 + wave); pc < p1;) {
        const int h = tab(C.T.var_prog, pc);
        const int dv = h & 0xFF, col = h >> 8;
        const float x = L.llr_at(col * L.z4 + L.k4);
        for (int e = 0; e < dv; ++e) {
            const int32_t w = tab(C.T.var_prog, pc + 1 + e);
            lds_wr(C.lds, (w & kLowMask) + L.vrot((w >> kShiftBit) & 0xFF), x);
        }
        pc += 1 + dv;
    }
}

// syndrome of this wave's rows from the ballots: 1 if any of its checks fails for this lane
__device__ __forceinline__ int parity_phase(const Ctx &C, const Lane &L, int wave) {
    const int W1 = C.T.W + 1;
    const int p1 = tab(C.T.prog_ptr, 2 * W1 + wave + 1);
    int inv = 0;
    for (int pc = tab(C.T.prog_ptr, 2 * W1 + wave); pc < p1;) {
        const int dc = tab(C.T.par_prog, pc);
        int p = 0;
        for (int e = 0; e < dc; ++e) {
            const int32_t w = tab(C.T.par_prog, pc + 1 + e);
            const int col = w & kLowMask, s = w >> kShiftBit;
            p ^= (int)((C.words[col] >> (L.f * L.Z() + ((L.k + s) & (L.Z() - 1)))) & 1ull);
        }
        inv |= p;
        pc += 1 + dc;
    }
    return inv;
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
    const int W1 = C.T.W + 1;
    for (int i = tab(C.T.prog_ptr, 3 * W1 + wave); i < tab(C.T.prog_ptr, 3 * W1 + wave + 1); ++i) {
        const int col = tab(C.T.bw_task, i);
        const int bit = (int)((words[col] >> L.lane) & 1ull);
        put_bit(C.bits, C.out_dtype, L.frame * C.T.N + (int64_t)col * L.Z() + L.k, bit);
        errs += bit;
    }
}

// per-workgroup totals of the error counters, written to this workgroup's row of the partials
// array (no global atomics: 32 768 workgroups adding into the same 4 words serialise at L2):
//   row = {bit errors, frame errors, frames, iteration sum, max iterations}
// counters_reduce_kernel folds the rows into the caller's counters afterwards.
__device__ __forceinline__ void reduce_counters(void *lds, const Lane &L, int errs, int my_iters, int nf,
                                                int Z, uint32_t *row) {
    uint32_t *u = reinterpret_cast<uint32_t *>(lds);
    const int nt = blockDim.x;
    __syncthreads();
    u[threadIdx.x] = (uint32_t)errs;
    u[nt + threadIdx.x] = (uint32_t)my_iters;
    __syncthreads();
    if (threadIdx.x < 64) {
        const int f = threadIdx.x;
        uint32_t be = 0, fe = 0, fr = 0, it = 0, itmax = 0;
        if (f < nf) {
            for (int w = 0; w < nt / 64; ++w)
                for (int k = 0; k < Z; ++k) be += u[w * 64 + f * Z + k];
            fe = be > 0;
            fr = 1;
            it = u[nt + f * Z];
            itmax = it;
        }
        for (int off = 32; off > 0; off >>= 1) {
            be += __shfl_xor(be, off, 64);
            fe += __shfl_xor(fe, off, 64);
            fr += __shfl_xor(fr, off, 64);
            it += __shfl_xor(it, off, 64);
            itmax = max(itmax, (uint32_t)__shfl_xor(itmax, off, 64));
        }
        if (f == 0) {
            row[0] = be;
            row[1] = fe;
            row[2] = fr;
            row[3] = it;
            row[4] = itmax;
        }
    }
}

__device__ __forceinline__ Lane make_lane(const FloodTables &T, const float *llr, int64_t B) {
    Lane L;
    L.lane = threadIdx.x & 63;
    const int lz = __builtin_ctz((unsigned)T.Z);  // Z is a power of two
    L.f = L.lane >> lz;
    L.k = L.lane & (T.Z - 1);
    L.lane4 = 4 * L.lane;
    L.fz4 = 4 * (L.f << lz);
    L.k4 = 4 * L.k;
    L.z4 = 4 * T.Z;
    L.zmask4 = 4 * T.Z - 1;
    L.frame = (int64_t)blockIdx.x * T.FG + L.f;
    L.valid = L.frame < B;
    L.llr_row = reinterpret_cast<const char *>(llr ? llr + (L.valid ? L.frame : 0) * (int64_t)T.N : nullptr);
    return L;
}

// ---------------------------------------------------------------- early stop: internal modes
// Public early_stop values are LDPC_ES_OFF / LDPC_ES_BATCH / LDPC_ES_FRAME.  The reference's
// batch-global rule (stop at the first iteration at which EVERY frame satisfies H x = 0 and return
// that iteration's decisions, traditional_decoders.py:104-107) runs as up to three passes, so that
// a batch that converges after t iterations costs about t iterations, not max_iter:
//   ES_P1     each workgroup iterates until all of ITS frames are valid at the same iteration
//             t_wg (or max_iter), keeps that iteration's decision ballots; T = max over t_wg.
//             No iteration before T can be valid for the whole batch.
//   ES_P2     workgroups with t_wg == T emit their kept ballots; the others decode T iterations
//             again and emit; a frame that is not valid at T (with T < max_iter) raises `bad`.
//   ES_BATCH  (runs only when bad) the exhaustive search: decode max_iter iterations keeping every
//             iteration's ballots and validity bits; batch_and / batch_emit take the first
//             iteration at which every frame is valid.
// es_finalize_kernel between P2 and the fallback decides, on the device, which result stands.

#ifdef LDPC_EXP_NOBARRIER  // timing experiment only: results are wrong without the phase barriers
#define LDPC_ITER_SYNC() ((void)0)
#else
#define LDPC_ITER_SYNC() __syncthreads()
#endif



// The iteration loop shared by both kernels.  Body supplies the four per-wave phases:
//   init(C, L)             v2c <- llr on every slot
//   check(C, L, errs)      c2v of this wave's check rows, in place
//   var(C, L, write, errs) v2c (write) and APP of this wave's columns; decisions when asked
//   parity(C, L) -> int    1 if any of this wave's checks fails for this lane (needs ballots)
// Every branch below depends on workgroup-uniform values only, so all waves meet the same
// barriers even when Body is specialised per wave.
template <int ES, class Body>
__device__ __forceinline__ void flood_drive(Body &body, Ctx &C, const Lane &L, int64_t B, int max_iter,
                                            const Outs &O, const EsWs &W) {
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int FG = C.T.FG, Nb = C.T.Nb, Z = C.T.Z;
    const int nf = (int)min<int64_t>((int64_t)FG, B - (int64_t)blockIdx.x * FG);
    const uint64_t exist = nf >= 64 ? ~0ull : ((1ull << nf) - 1ull);
    int errs = 0;
    if constexpr (ES == LDPC_ES_BATCH) {
        if (__builtin_amdgcn_readfirstlane(W.ctl[2]) == 0) return;  // the fast passes stood
    }
    if constexpr (ES == ES_P2) {
        const int T = __builtin_amdgcn_readfirstlane(W.ctl[0]);
        if (__builtin_amdgcn_readfirstlane(W.twg[blockIdx.x]) == T) {
            emit_from_words(C, L, W.cand + (int64_t)blockIdx.x * Nb, exist, wave, errs);
            if (O.iters_out && L.valid && L.k == 0) O.iters_out[L.frame] = T;
            reduce_counters(C.lds, L, errs, T, nf, Z, O.partials + (int64_t)blockIdx.x * kPartRow);
            return;
        }
        max_iter = T;
    }
    if (tid == 0) *C.flag = 0;
    __syncthreads();
    body.init(C, L);
    __syncthreads();
#ifdef LDPC_TIMELINE
    uint64_t *tl = (O.timeline && blockIdx.x < (unsigned)kTlWgs && L.lane == 0)
                       ? O.timeline + ((int64_t)blockIdx.x * 4 + wave) * kTlPer : nullptr;
    // one asm statement with its own lgkmcnt(0) and scheduling fences around it: the builtin form
    // leaves the wait's place to the compiler, which then drains LDS reads all over the loop
    auto mark = [&](int k) {
        uint64_t t;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (tl && k < kTlPer) tl[k] = t;
    };
#else
    auto mark = [](int) {};
#endif
    mark(0);

    int my_iters = max_iter;
    uint64_t done = 0;
    constexpr bool kEvery = ES == LDPC_ES_BATCH || ES == LDPC_ES_FRAME || ES == ES_P1;  // ballots every iteration
    for (int it = 0; it < max_iter; ++it) {
        const bool last = it == max_iter - 1;
        C.direct_bits = (ES == LDPC_ES_OFF || ES == ES_P2) && last;
        C.ballots = ES == LDPC_ES_BATCH || ES == LDPC_ES_FRAME || ES == ES_P1 || (ES == ES_P2 && last);
        // decisions are taken only in the iterations that need them (DEC = true), so the other
        // iterations carry no decision code at all
        if (kEvery || last)
            body.template check<true>(C, L, errs);
        else
            body.template check<false>(C, L, errs);
        mark(1 + 4 * it);
        LDPC_ITER_SYNC();
        mark(2 + 4 * it);
        if (C.ballots && tid == 0) C.words[Nb] = 0;
        if (last)
            body.template var<true, false>(C, L, errs);
        else if (kEvery)
            body.template var<true, true>(C, L, errs);
        else
            body.template var<false, true>(C, L, errs);
        mark(3 + 4 * it);
        LDPC_ITER_SYNC();
        mark(4 + 4 * it);
        if (C.ballots) {
            // syndrome H x = 0 per frame (traditional_decoders.py:111-134), from the ballots
            const uint64_t m = __ballot(body.parity(C, L));
            if (L.lane == 0 && m) atomicOr((unsigned long long *)&C.words[Nb], (unsigned long long)m);
            __syncthreads();
            const uint64_t vmask = frame_valid_mask(C.words[Nb], Z, FG) & exist;
            bool stop = false;
            if constexpr (ES == LDPC_ES_BATCH) {
                if (L.valid && L.k == 0 && ((vmask >> L.f) & 1ull))
                    W.valid[L.frame * W.nvw + (it >> 5)] |= 1u << (it & 31);
                uint64_t *dst = W.words + ((int64_t)blockIdx.x * max_iter + it) * Nb;
                for (int c = tid; c < Nb; c += blockDim.x) dst[c] = C.words[c];
            } else if constexpr (ES == LDPC_ES_FRAME) {
                const uint64_t newly = vmask & ~done;
                if (newly) {
                    emit_from_words(C, L, C.words, newly, wave, errs);
                    if ((newly >> L.f) & 1ull) my_iters = it + 1;
                    if (O.iters_out && L.valid && L.k == 0 && ((newly >> L.f) & 1ull)) O.iters_out[L.frame] = it + 1;
                    done |= newly;
                }
                stop = done == exist;
            } else if constexpr (ES == ES_P1) {
                stop = vmask == exist || last;
                if (stop) {
                    uint64_t *dst = W.cand + (int64_t)blockIdx.x * Nb;
                    for (int c = tid; c < Nb; c += blockDim.x) dst[c] = C.words[c];
                    if (tid == 0) {
                        W.twg[blockIdx.x] = it + 1;
                        atomicMax(&W.ctl[0], it + 1);
                    }
                }
            } else if constexpr (ES == ES_P2) {
                if (vmask != exist && tid == 0) atomicOr(&W.ctl[1], 1);
            }
            __syncthreads();
            if (stop) break;
        }
    }
    if constexpr (ES == LDPC_ES_FRAME) {
        const uint64_t rest = exist & ~done;
        if (rest) {
            emit_from_words(C, L, C.words, rest, wave, errs);
            if (O.iters_out && L.valid && L.k == 0 && ((rest >> L.f) & 1ull)) O.iters_out[L.frame] = max_iter;
        }
    }
    if constexpr (ES == LDPC_ES_OFF || ES == ES_P2) {
        if (O.iters_out && L.valid && L.k == 0) O.iters_out[L.frame] = max_iter;
    }
    if constexpr (ES == LDPC_ES_OFF || ES == LDPC_ES_FRAME) {
        if (O.partials) reduce_counters(C.lds, L, errs, my_iters, nf, Z, O.partials + (int64_t)blockIdx.x * kPartRow);
    }
    if constexpr (ES == ES_P2) reduce_counters(C.lds, L, errs, max_iter, nf, Z, O.partials + (int64_t)blockIdx.x * kPartRow);
}

template <int ALGO>
struct GenericBody {
    int wave;
    __device__ __forceinline__ void init(Ctx &C, const Lane &L) { init_phase(C, L, wave); }
    template <bool DEC>
    __device__ __forceinline__ void check(const Ctx &C, const Lane &L, int &errs) { check_phase<ALGO>(C, L, wave, errs); }
    template <bool DEC, bool WRITE>
    __device__ __forceinline__ void var(const Ctx &C, const Lane &L, int &errs) {
        var_phase(C, L, wave, WRITE, errs);
    }
    __device__ __forceinline__ int parity(const Ctx &C, const Lane &L) { return parity_phase(C, L, wave); }
};

__device__ __forceinline__ void init_ctx(Ctx &C, const FloodTables &T, char *lds, float alpha, int out_dtype,
                                         void *bits) {
    C.T = T;
    C.lds = lds;
    C.flag = reinterpret_cast<uint32_t *>(lds + (size_t)T.nslots * 256);
    C.words = reinterpret_cast<uint64_t *>(lds + (size_t)T.nslots * 256 + 8);
    C.alpha = alpha;
    C.out_dtype = out_dtype;
    C.bits = bits;
    C.direct_bits = false;
    C.ballots = false;
}

}  // namespace

template <int ALGO, int ES>
__global__ __launch_bounds__(512) void flood_kernel(FloodTables T, const float *__restrict__ llr, int64_t B,
                                                    int max_iter, float alpha, int out_dtype,
                                                    void *__restrict__ bits, Outs O, EsWs W) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const Lane L = make_lane(T, llr, B);
    Ctx C;
    init_ctx(C, T, lds, alpha, out_dtype, bits);
    GenericBody<ALGO> body{__builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6)};
    flood_drive<ES>(body, C, L, B, max_iter, O, W);
}

// ---------------------------------------------------------------- compile-time schedules
// flood_fixed_kernel: the same algorithm for a graph whose schedule is known at compile time
// (gen/fixed_codes.hpp: the reference's two codes), specialised per wave.  Every slot offset,
// shift, degree and task list is a constant, and the loop-invariant per-lane data lives in
// registers for the whole decode:
//   ext[]   the channel LLRs of the wave's degree-1 edges (their v2c forever)
//   cllr[]  the channel LLRs of the wave's columns
//   rot[]   the rotated byte base f*Z + (k - s) mod Z of every shift s the wave's columns use
// so the iteration touches no global memory and computes no addresses: a check-row message is
// ds_read at lane4 + slot*256, a column message at rot[s] + slot*256 (immediate offsets).  Both
// phases are software-pipelined: the next row's / column's LDS reads are issued before the
// current one is computed (slots are disjoint between rows and between columns, so the reads
// never depend on the writes in flight).  Bit-identical to flood_kernel.
namespace {


// Variable-phase schedule (gen/fixed_codes.hpp): VT pairs two columns per task on v_pk_add_f32
// (default), VS runs every column alone (LDPC_VAR_PAIRS=0, A/B builds)
#ifndef LDPC_VAR_PAIRS
#define LDPC_VAR_PAIRS 1
#endif
#if LDPC_VAR_PAIRS
#define LDPC_VT(x) G::VT_##x
#else
#define LDPC_VT(x) G::VS_##x
#endif

// per-wave compile-time plan
template <class G, int WV>
struct FxPlan {
    static constexpr int R0 = G::CHK_PTR[WV], NR = G::CHK_PTR[WV + 1] - R0;
    // the wave's columns (LLRs in registers, init, shifts) and its variable tasks
    static constexpr int C0 = LDPC_VT(COL_PTR)[WV], NC = LDPC_VT(COL_PTR)[WV + 1] - C0;
    static constexpr int T0 = LDPC_VT(PTR)[WV], NT = LDPC_VT(PTR)[WV + 1] - T0;
    static constexpr int col_index(int col) {
        for (int i = 0; i < NC; ++i)
            if (LDPC_VT(COLS)[C0 + i] == col) return i;
        return -1;
    }
    struct Tab {
        int nsh = 0, next = 0, maxdc = 1, maxdv = 1;
        int shv[64] = {};        // distinct shifts of the wave's columns
        int shidx[64] = {};      // shift -> index into shv (or -1)
        int ext_before[64] = {}; // ext edges in the wave's rows before row i
    };
    static constexpr Tab make() {
        Tab t{};
        for (int i = 0; i < 64; ++i) t.shidx[i] = -1;
        for (int i = 0; i < NR; ++i) {
            const int R = G::CHK_ROWS[R0 + i];
            t.ext_before[i] = t.next;
            const int dc = G::ROW_PTR[R + 1] - G::ROW_PTR[R];
            if (dc > t.maxdc) t.maxdc = dc;
            for (int e = G::ROW_PTR[R]; e < G::ROW_PTR[R + 1]; ++e)
                if (G::ROW_SLOT[e] < 0) ++t.next;
        }
        for (int i = 0; i < NC; ++i) {
            const int c = LDPC_VT(COLS)[C0 + i];
            const int dv = G::COL_PTR[c + 1] - G::COL_PTR[c];
            if (dv > t.maxdv) t.maxdv = dv;
            for (int j = G::COL_PTR[c]; j < G::COL_PTR[c + 1]; ++j) {
                const int s = G::COL_SHIFT[j];
                if (t.shidx[s] < 0) {
                    t.shidx[s] = t.nsh;
                    t.shv[t.nsh++] = s;
                }
            }
        }
        return t;
    }
    static constexpr Tab T = make();
    // index into ext[] of edge e of the wave's row i (an edge without a slot)
    static constexpr int ext_index(int i, int e) {
        const int R = G::CHK_ROWS[R0 + i];
        int x = T.ext_before[i];
        for (int q = 0; q < e; ++q)
            if (G::ROW_SLOT[G::ROW_PTR[R] + q] < 0) ++x;
        return x;
    }
};

#ifndef LDPC_VAR_PIPE
#define LDPC_VAR_PIPE 24
#endif
// the next column's reads are issued before the current column's adds when the two columns hold
// at most this many messages together (register budget: 4 workgroups per CU = 128 VGPRs)
constexpr int kVarPipe = LDPC_VAR_PIPE;

template <class G, int ALGO, int WV>
struct FixedBody {
    using P = FxPlan<G, WV>;
    static constexpr int ZM4 = 4 * G::Z - 1;
    static constexpr int NEXT = P::T.next > 0 ? P::T.next : 1;
    static constexpr int NCOL = P::NC > 0 ? P::NC : 1;
    static constexpr int NSH = P::T.nsh > 0 ? P::T.nsh : 1;
    static constexpr int MAXDC = P::T.maxdc, MAXDV = P::T.maxdv;
    float ext[NEXT];
    float cllr[NCOL];
    int rot[NSH];

    __device__ __forceinline__ void init(Ctx &C, const Lane &L) {
        bool nan = false;
        sfor<P::NR>([&](auto i) {
            constexpr int I = decltype(i)::value, R = G::CHK_ROWS[P::R0 + I];
            constexpr int P0 = G::ROW_PTR[R], DC = G::ROW_PTR[R + 1] - P0;
            sfor<DC>([&](auto e) {
                constexpr int E = decltype(e)::value;
                if constexpr (G::ROW_SLOT[P0 + E] < 0) {
                    constexpr int X = P::ext_index(I, E), COL = G::ROW_COL[P0 + E], S4 = 4 * G::ROW_SHIFT[P0 + E];
                    ext[X] = L.llr_at(COL * 4 * G::Z + ((L.k4 + S4) & ZM4));
                    nan |= is_zero_sign(ext[X]);  // zero or NaN: the sticky flag (see check())
                }
            });
        });
        sfor<P::T.nsh>([&](auto j) {
            constexpr int J = decltype(j)::value;
            rot[J] = L.fz4 + ((L.k4 + (4 * G::Z - 4 * P::T.shv[J])) & ZM4);
        });
        sfor<P::NC>([&](auto i) {
            constexpr int I = decltype(i)::value, COL = LDPC_VT(COLS)[P::C0 + I];
            constexpr int P0 = G::COL_PTR[COL], DV = G::COL_PTR[COL + 1] - P0;
            cllr[I] = L.llr_at(COL * 4 * G::Z + L.k4);
            nan |= is_zero_sign(cllr[I]);
            sfor<DV>([&](auto jj) {
                constexpr int J = decltype(jj)::value, SL = G::COL_SLOT[P0 + J];
                constexpr int SI = P::T.shidx[G::COL_SHIFT[P0 + J]];
                lds_wr(C.lds + SL * 256, rot[SI], cllr[I]);
            });
        });
        if (__any(nan) && L.lane == 0) *C.flag = 1;
    }

    // ---- check phase
    template <int I>
    __device__ __forceinline__ void load_row(const Ctx &C, const Lane &L, float (&v)[MAXDC]) const {
        constexpr int R = G::CHK_ROWS[P::R0 + I], P0 = G::ROW_PTR[R], DC = G::ROW_PTR[R + 1] - P0;
        sfor<DC>([&](auto e) {
            constexpr int E = decltype(e)::value, SL = G::ROW_SLOT[P0 + E];
            if constexpr (SL >= 0)
                v[E] = lds_rd(C.lds + SL * 256, L.lane4);
            else
                v[E] = ext[P::ext_index(I, E)];
        });
    }

    template <int I, bool DEC, bool SLOW = false>
    __device__ __forceinline__ void row(const Ctx &C, const Lane &L, const float (&v)[MAXDC], int &errs, float ninf, float pinf, uint32_t sgn, float alv) const {
        constexpr int R = G::CHK_ROWS[P::R0 + I], P0 = G::ROW_PTR[R], DC = G::ROW_PTR[R + 1] - P0;
        // an output is needed for a slot edge always, for a degree-1 edge only to take its decision
        auto needed = [](int e) constexpr { return DEC || G::ROW_SLOT[P0 + e] >= 0; };
        auto emit = [&](auto e, float o) {
            constexpr int E = decltype(e)::value, SL = G::ROW_SLOT[P0 + E];
            if constexpr (SL >= 0) {
                lds_wr_tid<SL * 256>(o);  // ds_write_addtid_b32: the slot entry of a row is slot[lane]
            } else if constexpr (DEC) {
                if (C.direct_bits || C.ballots)  // degree-1 variable: APP = llr + c2v
                    ext_decision(C, L, G::ROW_COL[P0 + E], 4 * G::ROW_SHIFT[P0 + E], v[E] + o, errs);
            }
        };
        if constexpr (ALGO == LDPC_ALGO_MINSUM) {
            // the two smallest magnitudes (v_med3 / v_min with |x| source modifiers)
            // m2 starts as an opaque +inf: a constant one lets the compiler rewrite the first
            // v_med3 as a canonicalising fmaxf
            float m1 = fabsf(v[0]), m2 = pinf;
            two_smallest<DC>(v, m1, m2, ninf);
            // Fast path: no zero message in the row (then m1 > 0) and no possible NaN in the
            // workgroup (the sticky flag, see var()): torch.sign is +-1 on every message, so
            //   c2v_e = (par ^ sign(x_e)) * (alpha * (|x_e| == m1 ? m2 : m1))
            // bit for bit (a tie at m1 puts m1 in m2 too).  Otherwise MinSumStats (exact
            // torch.sign(0) = 0 and NaN semantics).
            // the workgroup's sticky flag (init / var) covers zero and NaN inputs: one branch per
            // phase (check) instead of one per row, and the hot loop holds the fast code only
            if (!SLOW) {
                // the sign mask and alpha as VGPR operands: an SGPR (or SGPR-held constant) source
                // halves a VALU op's issue rate (tools/ubench), so the per-edge v_bitop3 below and
                // the per-row products run at the full rate
                const uint32_t par = sign_parity_n<DC>(v) & sgn;
                const uint32_t s1 = __float_as_uint(alv * m1) ^ par, s2 = __float_as_uint(alv * m2) ^ par;
                // |x_e| == m1 ? s2 : s1, with each compare issued three instructions ahead of its
                // select (a VALU-written lane mask read by a VALU needs 2 wait states on gfx950;
                // left to the compiler, every edge paid an s_nop 1)
                uint64_t mk[DC];
                uint32_t sel[DC];
                sfor<DC + 3>([&](auto q) {
                    constexpr int Q = decltype(q)::value;
                    if constexpr (Q < DC && needed(Q)) mk[Q] = cmp_eq_abs(v[Q], m1);
                    if constexpr (Q >= 3 && needed(Q - 3)) sel[Q - 3] = cndmask(s1, s2, mk[Q - 3]);
                });
                sfor<DC>([&](auto e) {
                    constexpr int E = decltype(e)::value;
                    if constexpr (needed(E))
                        emit(e, __uint_as_float(__builtin_amdgcn_bitop3_b32(sel[E], __float_as_uint(v[E]), sgn, 0x78)));
                });
            } else {
                MinSumStats st;
                sfor<DC>([&](auto e) { st.add(decltype(e)::value, v[decltype(e)::value]); });
                sfor<DC>([&](auto e) { emit(e, st.c2v(decltype(e)::value, v[decltype(e)::value], C.alpha)); });
            }
        } else {
            // sum-product (traditional_decoders.py:72-81): exclusive product from 1.0 ascending
            float acc[DC];
            float Pp = 1.0f;
            sfor<DC>([&](auto jj) {
                constexpr int J = decltype(jj)::value;
                const float t = tanh_half(v[J]);
                sfor<J>([&](auto e) { acc[decltype(e)::value] = acc[decltype(e)::value] * t; });
                acc[J] = Pp;
                Pp = Pp * t;
            });
            sfor<DC>([&](auto e) { emit(e, two_atanh(acc[decltype(e)::value])); });
        }
    }

    template <bool DEC>
    __device__ __forceinline__ void check(const Ctx &C, const Lane &L, int &errs) const {
        if constexpr (ALGO == LDPC_ALGO_MINSUM) {
            if (__builtin_amdgcn_readfirstlane(*C.flag) != 0)
                rows<DEC, true>(C, L, errs);
            else
                rows<DEC, false>(C, L, errs);
            return;
        }
        rows<DEC, false>(C, L, errs);
    }

    template <bool DEC, bool SLOW>
    __device__ __forceinline__ void rows(const Ctx &C, const Lane &L, int &errs) const {
        float va[MAXDC], vb[MAXDC];
        addtid_begin(C.lds);
        const float ninf = opaque_sf(-INFINITY), pinf = opaque_sf(INFINITY);
        const uint32_t sgn = opaque_vu(0x80000000u);
        const float alv = opaque_vf(C.alpha);
        load_row<0>(C, L, va);
        sfor<P::NR>([&](auto i) {
            constexpr int I = decltype(i)::value;
            if constexpr (I % 2 == 0) {
                if constexpr (I + 1 < P::NR) load_row<I + 1>(C, L, vb);
                row<I, DEC, SLOW>(C, L, va, errs, ninf, pinf, sgn, alv);
            } else {
                if constexpr (I + 1 < P::NR) load_row<I + 1>(C, L, va);
                row<I, DEC, SLOW>(C, L, vb, errs, ninf, pinf, sgn, alv);
            }
        });
        addtid_end();
    }

    // ---- variable phase: tasks (column A, column B or none, outputs [LO, HI) of both), see
    // tools/gen_fixed_codes.py var_schedule.  Per output e of a column of degree D:
    //   v2c_e = P_e + c_{e+1} + ... + c_{D-1},  P_0 = llr, P_{J+1} = P_J + c_J
    // in this order (traditional_decoders.py:235-250: the sum over i' != i from llr in ascending
    // check order); the APP is P_D.  A pair runs both columns' chains in the two halves of
    // v_pk_add_f32 (two independent IEEE fp32 adds: each half is the scalar sequence, bit for bit)
    // while both have messages (J < DB); column A's remaining steps are scalar v_add_f32.
    template <int TK>
    struct Task {
        static constexpr int X = P::T0 + TK;
        static constexpr int CA = LDPC_VT(A)[X], CB = LDPC_VT(B)[X], LO = LDPC_VT(LO)[X], HI = LDPC_VT(HI)[X];
        static constexpr int PA = G::COL_PTR[CA], DA = G::COL_PTR[CA + 1] - PA;
        static constexpr int PB = CB >= 0 ? G::COL_PTR[CB] : 0, DB = CB >= 0 ? G::COL_PTR[CB + 1] - PB : 0;
        static_assert(DB <= DA && (DB == 0 || LO < DB), "pair tasks: A is the longer column, B has outputs");
        static constexpr int IA = P::col_index(CA), IB = CB >= 0 ? P::col_index(CB) : 0;
        static constexpr int NPREFA = HI == DA ? DA : (HI > 0 ? HI - 1 : 0);
        static constexpr bool BLAST = DB > 0 && LO <= DB - 1 && DB - 1 < HI;  // B's APP here
        static constexpr int NPREF = NPREFA > (BLAST ? DB : 0) ? NPREFA : (BLAST ? DB : 0);
        static constexpr int NMSG = DA + DB;
    };
    struct TaskIn {
        f32x2 cp[MAXDV];  // J < DB: {c_A[J], c_B[J]}
        float cs[MAXDV];  // DB <= J < DA: c_A[J]
    };

    template <int TK>
    __device__ __forceinline__ void load_task(const Ctx &C, TaskIn &in) const {
        using K = Task<TK>;
        sfor<K::DA>([&](auto jj) {
            constexpr int J = decltype(jj)::value;
            constexpr int SA = G::COL_SLOT[K::PA + J], RA = P::T.shidx[G::COL_SHIFT[K::PA + J]];
            if constexpr (J < K::DB) {
                constexpr int SB = G::COL_SLOT[K::PB + J], RB = P::T.shidx[G::COL_SHIFT[K::PB + J]];
                in.cp[J].x = lds_rd(C.lds + SA * 256, rot[RA]);
                in.cp[J].y = lds_rd(C.lds + SB * 256, rot[RB]);
            } else {
                in.cs[J] = lds_rd(C.lds + SA * 256, rot[RA]);
            }
        });
    }

    template <int TK, bool DEC, bool WRITE>
    __device__ __forceinline__ void task(const Ctx &C, const Lane &L, const TaskIn &in, int &errs, bool &bad,
                                         float &mz) const {
        using K = Task<TK>;
        constexpr int DA = K::DA, DB = K::DB, LO = K::LO, HI = K::HI;
        f32x2 P2;
        float PA = cllr[K::IA];
        if constexpr (DB > 0) {
            P2.x = cllr[K::IA];
            P2.y = cllr[K::IB];
        }
        f32x2 acc2[DB > 0 ? DB : 1];
        float accA[DA];
        sfor<DA>([&](auto jj) {
            constexpr int J = decltype(jj)::value;
            constexpr int EN = (J < HI ? J : HI) - LO;  // outputs [LO, min(J, HI)) take c_J
            if constexpr (J < DB) {
                if constexpr (EN > 0)
                    sfor<EN>([&](auto q) {
                        constexpr int E = LO + decltype(q)::value;
                        acc2[E] = acc2[E] + in.cp[J];
                    });
                if constexpr (LO <= J && J < HI) acc2[J] = P2;
                if constexpr (J < K::NPREF) P2 = P2 + in.cp[J];
                if constexpr (J == DB - 1) PA = P2.x;
            } else {
                if constexpr (EN > 0)
                    sfor<EN>([&](auto q) {
                        constexpr int E = LO + decltype(q)::value;
                        if constexpr (E < DB)
                            acc2[E].x = acc2[E].x + in.cs[J];
                        else
                            accA[E] = accA[E] + in.cs[J];
                    });
                if constexpr (LO <= J && J < HI) accA[J] = PA;
                if constexpr (J < K::NPREF) PA = PA + in.cs[J];
            }
        });
        if constexpr (WRITE) {
            sfor<HI - LO>([&](auto q) {
                constexpr int E = LO + decltype(q)::value;
                constexpr int SA = G::COL_SLOT[K::PA + E], RA = P::T.shidx[G::COL_SHIFT[K::PA + E]];
                if constexpr (E < DB) {
                    constexpr int SB = G::COL_SLOT[K::PB + E], RB = P::T.shidx[G::COL_SHIFT[K::PB + E]];
                    lds_wr(C.lds + SA * 256, rot[RA], acc2[E].x);
                    lds_wr(C.lds + SB * 256, rot[RB], acc2[E].y);
                    // smallest |v2c| written: a zero sets the flag (v_minimum3: no canonicalising
                    // v_max; a NaN here implies a non-finite APP, caught by `bad`)
                    if constexpr (ALGO == LDPC_ALGO_MINSUM) mz = vmin(vmin(mz, fabsf(acc2[E].x)), fabsf(acc2[E].y));
                } else {
                    lds_wr(C.lds + SA * 256, rot[RA], accA[E]);
                    if constexpr (ALGO == LDPC_ALGO_MINSUM) {
                        // two A-only outputs per v_minimum3
                        if constexpr ((E - (DB > LO ? DB : LO)) % 2 == 1)
                            mz = vmin(vmin(mz, fabsf(accA[E - 1])), fabsf(accA[E]));
                        else if constexpr (E == HI - 1)
                            mz = vmin(mz, fabsf(accA[E]));
                    }
                }
            });
        }
        // a NaN v2c implies a NaN or infinite APP of its column (every summand of a v2c is a
        // summand of the APP; +-inf is absorbing), so this flag bounds the fast check path
        if constexpr (HI == DA) {
            if constexpr (ALGO == LDPC_ALGO_MINSUM) bad |= !(fabsf(PA) < INFINITY);
            if constexpr (DEC) {
                if (C.direct_bits || C.ballots) var_decision(C, L, K::CA, PA, errs);
            }
        }
        if constexpr (K::BLAST) {
            if constexpr (ALGO == LDPC_ALGO_MINSUM) bad |= !(fabsf(P2.y) < INFINITY);
            if constexpr (DEC) {
                if (C.direct_bits || C.ballots) var_decision(C, L, K::CB, P2.y, errs);
            }
        }
    }

    template <bool DEC, bool WRITE>
    __device__ __forceinline__ void var(const Ctx &C, const Lane &L, int &errs) const {
        bool bad = false;
        float mz = INFINITY;
        if constexpr (P::NT > 0) {
            // software pipelining: the next task's reads are issued before the current task's adds
            // when the two hold at most kVarPipe messages together (slots are disjoint between
            // tasks, so the reads never depend on the writes in flight)
            TaskIn ta, tb;
            load_task<0>(C, ta);
            sfor<P::NT>([&](auto i) {
                constexpr int I = decltype(i)::value;
                constexpr bool more = I + 1 < P::NT;
                constexpr bool ahead = more && Task<I>::NMSG + Task<(more ? I + 1 : I)>::NMSG <= kVarPipe;
                if constexpr (I % 2 == 0) {
                    if constexpr (ahead) load_task<I + 1>(C, tb);
                    task<I, DEC, WRITE>(C, L, ta, errs, bad, mz);
                    if constexpr (more && !ahead) load_task<(more ? I + 1 : I)>(C, tb);
                } else {
                    if constexpr (ahead) load_task<I + 1>(C, ta);
                    task<I, DEC, WRITE>(C, L, tb, errs, bad, mz);
                    if constexpr (more && !ahead) load_task<(more ? I + 1 : I)>(C, ta);
                }
            });
        }
        if constexpr (ALGO == LDPC_ALGO_MINSUM) {
            bad |= mz == 0.0f;
            if (__any(bad) && L.lane == 0) *C.flag = 1;
        }
        (void)mz;
    }

    __device__ __forceinline__ int parity(const Ctx &C, const Lane &L) const {
        int inv = 0;
        // opaque copies: the per-edge bit positions are recomputed here (early-stop iterations
        // only) instead of being hoisted out of the loop into ~50 live registers
        int f = L.f, k = L.k;
        asm volatile("" : "+v"(f), "+v"(k));
        sfor<P::NR>([&](auto i) {
            constexpr int R = G::CHK_ROWS[P::R0 + decltype(i)::value];
            constexpr int P0 = G::ROW_PTR[R], DC = G::ROW_PTR[R + 1] - P0;
            int p = 0;  // parity of check r*Z + k of frame f: xor of its variables' decisions
            sfor<DC>([&](auto e) {
                constexpr int E = decltype(e)::value;
                constexpr int COL = G::ROW_COL[P0 + E], S = G::ROW_SHIFT[P0 + E];
                p ^= (int)(C.words[COL] >> (f * G::Z + ((k + S) & (G::Z - 1))));
            });
            inv |= p;
        });
        return inv & 1;
    }
};

template <class G, class F>
__device__ __forceinline__ void fx_by_wave(int wave, F &&f) {
    static_assert(G::W == 4, "fixed schedules are generated for 4 waves");
    switch (wave) {
        case 0: f(ic<0>{}); break;
        case 1: f(ic<1>{}); break;
        case 2: f(ic<2>{}); break;
        default: f(ic<3>{}); break;
    }
}

}  // namespace

// 4 workgroups per CU without early stop (LDS: 159 slots x 256 B + 8 B each); the early-stop
// modes also keep Nb + 1 ballot words in LDS, which leaves room for 3, so they may use 168 VGPRs
template <class G, int ALGO, int ES>
__global__ __launch_bounds__(256, ES == LDPC_ES_OFF ? 4 : 3) void flood_fixed_kernel(FloodTables T, const float *__restrict__ llr,
                                                          int64_t B, int max_iter, float alpha, int out_dtype,
                                                          void *__restrict__ bits, Outs O, EsWs W) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const Lane L = make_lane(T, llr, B);
    Ctx C;
    init_ctx(C, T, lds, alpha, out_dtype, bits);
    fx_by_wave<G>(__builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), [&](auto wv) {
        FixedBody<G, ALGO, decltype(wv)::value> body;
        flood_drive<ES>(body, C, L, B, max_iter, O, W);
    });
}

}  // namespace ldpc
