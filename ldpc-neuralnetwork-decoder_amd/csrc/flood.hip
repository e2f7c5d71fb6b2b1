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
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>

#include <utility>

#include "common.hpp"
#include "gen/fixed_codes.hpp"
#include "graph.hpp"

namespace ldpc {

namespace {

// Graph programs are read-only for the kernel's lifetime and indexed by wave-uniform values:
// reading them through the constant address space makes every word a scalar (SMEM) load.
typedef const __attribute__((address_space(4))) int32_t const_i32;
__device__ __forceinline__ int32_t tab(const int32_t *p, int i) { return ((const_i32 *)p)[i]; }

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
#ifndef LDPC_MIN_ASM
#define LDPC_MIN_ASM 0
#endif
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
#if LDPC_MIN_ASM
    (void)ninf;
    asm("v_med3_f32 %0, %1, |%2|, %3" : "=v"(m2) : "v"(m1), "v"(x), "v"(m2));
    asm("v_min_f32 %0, %1, |%2|" : "=v"(m1) : "v"(m1), "v"(x));
#else
    // builtins, not inline asm: a VALU reading a VGPR written by inline asm gets a conservative
    // s_nop from the hazard recognizer (one per edge in the check phase)
    m2 = __builtin_amdgcn_fmed3f(m1, fabsf(x), m2);
    m1 = __builtin_amdgcn_fmed3f(m1, fabsf(x), ninf);
#endif
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
constexpr int kPartRow = 8;  // uint32 per workgroup row
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
constexpr int ES_P1 = 3, ES_P2 = 4;

#ifdef LDPC_EXP_NOBARRIER  // timing experiment only: results are wrong without the phase barriers
#define LDPC_ITER_SYNC() ((void)0)
#else
#define LDPC_ITER_SYNC() __syncthreads()
#endif

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
};

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
        LDPC_ITER_SYNC();
        if (C.ballots && tid == 0) C.words[Nb] = 0;
        if (last)
            body.template var<true, false>(C, L, errs);
        else if (kEvery)
            body.template var<true, true>(C, L, errs);
        else
            body.template var<false, true>(C, L, errs);
        LDPC_ITER_SYNC();
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

// per-wave compile-time plan
template <class G, int WV>
struct FxPlan {
    static constexpr int R0 = G::CHK_PTR[WV], NR = G::CHK_PTR[WV + 1] - R0;
    static constexpr int C0 = G::VAR_PTR[WV], NC = G::VAR_PTR[WV + 1] - C0;
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
            const int c = G::VAR_COLS[C0 + i];
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
#ifndef LDPC_SEL_ASM
// 1: the select by v_cmp / v_cndmask in asm (measured fastest); 0: the compare-free select (fewer
// VALU pipe cycles but one more instruction per edge: 3.7 % slower, the kernel is bound by the
// per-wave issue and dependency latency rather than by the VALU pipe)
#define LDPC_SEL_ASM 1
#endif
#ifndef LDPC_ZFLAG
#define LDPC_ZFLAG 1  // zero inputs join the sticky NaN flag: one slow/fast branch per check phase (+5%)
#endif
#ifndef LDPC_VAR_PK
#define LDPC_VAR_PK 0  // 1: variable update on v_pk_add_f32 pairs (6 % slower than scalar adds)
#endif
#ifndef LDPC_MIN_SPLIT
#define LDPC_MIN_SPLIT 0  // 1: the row's two minima as two half-row chains + a merge (shorter chain)
#endif
#ifndef LDPC_ADDTID
#define LDPC_ADDTID 1  // check-phase stores as ds_write_addtid_b32 (the slot entry of a row is slot[lane])
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
#if LDPC_ZFLAG
                    nan |= is_zero_sign(ext[X]);  // zero or NaN
#else
                    nan |= ext[X] != ext[X];
#endif
                }
            });
        });
        sfor<P::T.nsh>([&](auto j) {
            constexpr int J = decltype(j)::value;
            rot[J] = L.fz4 + ((L.k4 + (4 * G::Z - 4 * P::T.shv[J])) & ZM4);
        });
        sfor<P::NC>([&](auto i) {
            constexpr int I = decltype(i)::value, COL = G::VAR_COLS[P::C0 + I];
            constexpr int P0 = G::COL_PTR[COL], DV = G::COL_PTR[COL + 1] - P0;
            cllr[I] = L.llr_at(COL * 4 * G::Z + L.k4);
#if LDPC_ZFLAG
            nan |= is_zero_sign(cllr[I]);
#else
            nan |= cllr[I] != cllr[I];
#endif
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
    __device__ __forceinline__ void row(const Ctx &C, const Lane &L, const float (&v)[MAXDC], bool nanflag,
                                        int &errs, float ninf, float pinf, uint32_t sgn, float alv) const {
        constexpr int R = G::CHK_ROWS[P::R0 + I], P0 = G::ROW_PTR[R], DC = G::ROW_PTR[R + 1] - P0;
        // an output is needed for a slot edge always, for a degree-1 edge only to take its decision
        auto needed = [](int e) constexpr { return DEC || G::ROW_SLOT[P0 + e] >= 0; };
        auto emit = [&](auto e, float o) {
            constexpr int E = decltype(e)::value, SL = G::ROW_SLOT[P0 + E];
            if constexpr (SL >= 0) {
#if LDPC_ADDTID
                lds_wr_tid<SL * 256>(o);
#else
                lds_wr(C.lds + SL * 256, L.lane4, o);
#endif
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
#if LDPC_MIN_SPLIT
            if constexpr (DC >= 6) {
                // two independent chains over the halves, then the second smallest of the union =
                // med3(m1a, m1b, min(m2a, m2b)) (both minima are <= their chains' second minima)
                constexpr int H1 = DC / 2;
                float m1b = fabsf(v[H1]), m2b = pinf;
                sfor<H1 - 1>([&](auto e) {
                    two_min_step(m1, m2, v[decltype(e)::value + 1], ninf);
                    two_min_step(m1b, m2b, v[H1 + decltype(e)::value + 1], ninf);
                });
                if constexpr (DC - H1 > H1) two_min_step(m1b, m2b, v[DC - 1], ninf);
                const float t = __builtin_amdgcn_fmed3f(m2, m2b, ninf);  // min(m2, m2b)
                m2 = __builtin_amdgcn_fmed3f(m1, m1b, t);
                m1 = __builtin_amdgcn_fmed3f(m1, m1b, ninf);
            } else {
                sfor<DC - 1>([&](auto e) { two_min_step(m1, m2, v[decltype(e)::value + 1], ninf); });
            }
#else
            sfor<DC - 1>([&](auto e) { two_min_step(m1, m2, v[decltype(e)::value + 1], ninf); });
#endif
            // Fast path: no zero message in the row (then m1 > 0) and no possible NaN in the
            // workgroup (the sticky flag, see var()): torch.sign is +-1 on every message, so
            //   c2v_e = (par ^ sign(x_e)) * (alpha * (|x_e| == m1 ? m2 : m1))
            // bit for bit (a tie at m1 puts m1 in m2 too).  Otherwise MinSumStats (exact
            // torch.sign(0) = 0 and NaN semantics).
#if LDPC_ZFLAG
            // the workgroup's sticky flag (init / var) covers zero and NaN inputs: one branch per
            // phase (check) instead of one per row, and the hot loop holds the fast code only
            if (!SLOW) {
#elif LDPC_EXP_NOSLOW  // timing experiment only: the fast path unconditionally (inexact for zeros / NaN)
            if (true) {
#else
            if (!nanflag && !__any(m1 == 0.0f)) {
#endif
#if LDPC_SEL_ASM
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
#else
                // The select without compares: t = m1 - |x_e| is +0 exactly when |x_e| == m1 and
                // negative otherwise (x - y == 0 only for x == y; a flushed tiny difference is -0),
                // so its arithmetic shift by 31 is the "use s1" mask.  v_sub / v_ashr / v_bitop3
                // with VGPR operands issue at the full VALU rate, where v_cmp, v_cndmask and any
                // op with an SGPR operand take two passes (measured: tools/ubench).  The sign
                // mask and alpha are opaque VGPRs for the same reason.
                const uint32_t par = sign_parity_n<DC>(v) & sgn;
                const uint32_t s1 = __float_as_uint(alv * m1) ^ par, s2 = __float_as_uint(alv * m2) ^ par;
                sfor<DC>([&](auto e) {
                    constexpr int E = decltype(e)::value;
                    if constexpr (needed(E)) {
                        // (opaque: the compiler would turn the mask back into v_cmp + v_cndmask)
                        const uint32_t mk = opaque_vu((uint32_t)((int32_t)__float_as_uint(m1 - fabsf(v[E])) >> 31));
                        const uint32_t sel = (s1 & mk) | (s2 & ~mk);
                        // sel ^ (x & SIGN) as one v_bitop3 (the compiler splits it into and + xor)
                        emit(e, __uint_as_float(__builtin_amdgcn_bitop3_b32(sel, __float_as_uint(v[E]), sgn, 0x78)));
                    }
                });
#endif
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
        bool nanflag = false;
        if constexpr (ALGO == LDPC_ALGO_MINSUM) nanflag = __builtin_amdgcn_readfirstlane(*C.flag) != 0;
#if LDPC_ZFLAG
        if constexpr (ALGO == LDPC_ALGO_MINSUM) {
            if (nanflag)
                rows<DEC, true>(C, L, errs);
            else
                rows<DEC, false>(C, L, errs);
            return;
        }
#endif
        rows<DEC, false>(C, L, errs, nanflag);
    }

    template <bool DEC, bool SLOW>
    __device__ __forceinline__ void rows(const Ctx &C, const Lane &L, int &errs, bool nanflag = false) const {
        float va[MAXDC], vb[MAXDC];
#if LDPC_ADDTID
        addtid_begin(C.lds);
#endif
        const float ninf = opaque_sf(-INFINITY), pinf = opaque_sf(INFINITY);
        const uint32_t sgn = opaque_vu(0x80000000u);
        const float alv = opaque_vf(C.alpha);
        load_row<0>(C, L, va);
        sfor<P::NR>([&](auto i) {
            constexpr int I = decltype(i)::value;
            if constexpr (I % 2 == 0) {
                if constexpr (I + 1 < P::NR) load_row<I + 1>(C, L, vb);
                row<I, DEC, SLOW>(C, L, va, nanflag, errs, ninf, pinf, sgn, alv);
            } else {
                if constexpr (I + 1 < P::NR) load_row<I + 1>(C, L, va);
                row<I, DEC, SLOW>(C, L, vb, nanflag, errs, ninf, pinf, sgn, alv);
            }
        });
#if LDPC_ADDTID
        addtid_end();
#endif
    }

    // ---- variable phase
    static constexpr int dv_of(int i) { return G::COL_PTR[G::VAR_COLS[P::C0 + i] + 1] - G::COL_PTR[G::VAR_COLS[P::C0 + i]]; }

    template <int I>
    __device__ __forceinline__ void load_col(const Ctx &C, float (&c)[MAXDV]) const {
        constexpr int COL = G::VAR_COLS[P::C0 + I], P0 = G::COL_PTR[COL], DV = G::COL_PTR[COL + 1] - P0;
        sfor<DV>([&](auto jj) {
            constexpr int J = decltype(jj)::value, SL = G::COL_SLOT[P0 + J];
            constexpr int SI = P::T.shidx[G::COL_SHIFT[P0 + J]];
            c[J] = lds_rd(C.lds + SL * 256, rot[SI]);
        });
    }

    // v2c_e = llr + sum_{e' != e} c_e' in ascending check order (traditional_decoders.py:235-250):
    // acc[e] = P_e (prefix) then + c_{e+1} + ... ; in pairs, one v_pk_add_f32 adds c to two
    // running sums (two independent IEEE fp32 adds, the same sequence per element)
    template <int I, bool DEC, bool WRITE>
    __device__ __forceinline__ void col(const Ctx &C, const Lane &L, const float (&c)[MAXDV], int &errs,
                                        bool &bad, float &mz) const {
        constexpr int COL = G::VAR_COLS[P::C0 + I], P0 = G::COL_PTR[COL], DV = G::COL_PTR[COL + 1] - P0;
        float Pp = cllr[I];
        f32x2 acc[(DV + 1) / 2];
#if LDPC_VAR_PK
        sfor<DV>([&](auto jj) {
            constexpr int J = decltype(jj)::value;
            const f32x2 cc = {c[J], c[J]};
            sfor<J / 2>([&](auto p) { acc[decltype(p)::value] = acc[decltype(p)::value] + cc; });
            if constexpr (J % 2 == 1) {
                acc[J / 2].x = acc[J / 2].x + c[J];
                acc[J / 2].y = Pp;
            } else {
                acc[J / 2].x = Pp;
            }
            Pp = Pp + c[J];
        });
#else
        // scalar v_add_f32 (measured 6 % faster for the whole kernel than v_pk_add_f32 pairs: the
        // running sums are dependency chains, and a packed add's chain latency is longer)
        float a[DV];
        sfor<DV>([&](auto jj) {
            constexpr int J = decltype(jj)::value;
            sfor<J>([&](auto p) { a[decltype(p)::value] = a[decltype(p)::value] + c[J]; });
            a[J] = Pp;
            Pp = Pp + c[J];
        });
        sfor<DV>([&](auto jj) {
            constexpr int J = decltype(jj)::value;
            if constexpr (J % 2 == 0) acc[J / 2].x = a[J]; else acc[J / 2].y = a[J];
        });
#endif
        if constexpr (WRITE) {
            sfor<DV>([&](auto jj) {
                constexpr int J = decltype(jj)::value, SL = G::COL_SLOT[P0 + J];
                constexpr int SI = P::T.shidx[G::COL_SHIFT[P0 + J]];
                lds_wr(C.lds + SL * 256, rot[SI], J % 2 == 0 ? acc[J / 2].x : acc[J / 2].y);
            });
#if LDPC_ZFLAG
            if constexpr (ALGO == LDPC_ALGO_MINSUM) {  // smallest |v2c| written: a zero sets the flag
                sfor<(DV + 1) / 2>([&](auto pp) {
                    constexpr int Q = decltype(pp)::value;
                    if constexpr (2 * Q + 1 < DV)
                        mz = fminf(mz, fminf(fabsf(acc[Q].x), fabsf(acc[Q].y)));
                    else
                        mz = fminf(mz, fabsf(acc[Q].x));
                });
            }
#endif
        }
        // a NaN v2c implies a NaN or infinite APP of its column (every summand of a v2c is a
        // summand of the APP; +-inf is absorbing), so this flag bounds the fast check path
        if constexpr (ALGO == LDPC_ALGO_MINSUM) bad |= !(fabsf(Pp) < INFINITY);
        if constexpr (DEC) {
            if (C.direct_bits || C.ballots) var_decision(C, L, COL, Pp, errs);
        }
    }

    template <bool DEC, bool WRITE>
    __device__ __forceinline__ void var(const Ctx &C, const Lane &L, int &errs) const {
        bool bad = false;
        float mz = INFINITY;
        if constexpr (P::NC > 0) {
            float ca[MAXDV], cb[MAXDV];
            load_col<0>(C, ca);
            sfor<P::NC>([&](auto i) {
                constexpr int I = decltype(i)::value;
                constexpr bool ahead = I + 1 < P::NC && dv_of(I) + dv_of(I + 1) <= kVarPipe;
                if constexpr (I % 2 == 0) {
                    if constexpr (ahead) load_col<I + 1>(C, cb);
                    col<I, DEC, WRITE>(C, L, ca, errs, bad, mz);
                    if constexpr (I + 1 < P::NC && !ahead) load_col<I + 1>(C, cb);
                } else {
                    if constexpr (ahead) load_col<I + 1>(C, ca);
                    col<I, DEC, WRITE>(C, L, cb, errs, bad, mz);
                    if constexpr (I + 1 < P::NC && !ahead) load_col<I + 1>(C, ca);
                }
            });
        }
        if constexpr (ALGO == LDPC_ALGO_MINSUM) {
#if LDPC_ZFLAG
            bad |= mz == 0.0f;
#endif
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

// ---------------------------------------------------------------- host side
#ifndef LDPC_FLOOD_KERNELS_ONLY  // (defined by kernel-only experiment builds)
namespace {
constexpr size_t kLdsMax = 160 * 1024;

size_t flood_lds_bytes(const ldpc_graph *g, int es) {
    size_t b = (size_t)g->nslots * 64 * sizeof(float) + 8;  // slots + the NaN flag
    if (es != LDPC_ES_OFF) b += (size_t)(g->Nb + 1) * sizeof(uint64_t);
    return std::max<size_t>(b, 2 * 64 * (size_t)g->ft.W * sizeof(uint32_t));
}

size_t align256(size_t b) { return (b + 255) / 256 * 256; }

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

constexpr int kStreamMaxDeg = 32;  // register windows of stream_check_kernel / stream_var_kernel

bool use_stream(const ldpc_graph *g, int es) {
    if (!g->lds_ok || flood_lds_bytes(g, es) > kLdsMax) return true;
    const char *e = std::getenv("LDPC_FLOOD_STREAM");  // force the streaming kernels (tests, A/B)
    return e && std::atoi(e) != 0;
}

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
    hipLaunchKernelGGL(counters_reduce_kernel, dim3(1), dim3(1024), 0, s, w.partials, (B + 63) / 64, counters,
                       es == LDPC_ES_OFF ? nullptr : batch_iters, nullptr);
    LDPC_CHECK_LAUNCH("counters_reduce_kernel");
    return LDPC_OK;
}

// CustomMinSum workspace: the streaming arrays (msg, llrT) + probsT [N][B]
int64_t custom_ws_bytes(const ldpc_graph *g, int64_t B) {
    return (int64_t)(align256((size_t)g->E * B * 4) + 2 * align256((size_t)g->N * B * 4));
}

int run_custom_minsum(const ldpc_graph *g, const float *llr, int64_t B, int iterations, float *probs, void *work,
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

template <int ALGO, int ES>
int launch_flood(const ldpc_graph *g, const float *llr, int64_t B, int max_iter, float alpha, int out_dtype,
                 void *bits, const Outs &O, const EsWs &W, hipStream_t s) {
    const size_t lds = flood_lds_bytes(g, ES);
    auto kern = flood_kernel<ALGO, ES>;
    if (g->fixed_id == 1) kern = flood_fixed_kernel<fixed::BG2_Z4, ALGO, ES>;
    if (g->fixed_id == 2) kern = flood_fixed_kernel<fixed::BG2_Z32, ALGO, ES>;
    LDPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int64_t nwg = (B + g->FG - 1) / g->FG;
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(64 * g->ft.W), lds, s, g->ft, llr, B, max_iter, alpha,
                       out_dtype, bits, O, W);
    LDPC_CHECK_LAUNCH("flood_kernel");
    return LDPC_OK;
}

int reduce_rows(const ldpc_graph *g, int64_t B, const uint32_t *partials, uint64_t *counters, int32_t *batch_iters,
                const int32_t *gate, hipStream_t s) {
    if (!counters && !batch_iters) return LDPC_OK;
    const int64_t nwg = (B + g->FG - 1) / g->FG;
    hipLaunchKernelGGL(counters_reduce_kernel, dim3(1), dim3(1024), 0, s, partials, nwg, counters, batch_iters, gate);
    LDPC_CHECK_LAUNCH("counters_reduce_kernel");
    return LDPC_OK;
}

template <int ALGO>
int run_flood(const ldpc_graph *g, const float *llr, int64_t B, int max_iter, float alpha, int es, int out_dtype,
              void *bits, int32_t *iters_out, uint64_t *counters, int32_t *batch_iters, void *work, hipStream_t s) {
    const FloodWs ws = flood_ws(g, B, max_iter, es, work);
    const bool want = counters || batch_iters;
    const Outs O{iters_out, want ? ws.partials : nullptr};
    if (es == LDPC_ES_OFF) {
        int rc = launch_flood<ALGO, LDPC_ES_OFF>(g, llr, B, max_iter, alpha, out_dtype, bits, O, EsWs{}, s);
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
#endif  // LDPC_FLOOD_KERNELS_ONLY

}  // namespace ldpc

#ifndef LDPC_FLOOD_KERNELS_ONLY
using namespace ldpc;

extern "C" int64_t ldpc_flood_workspace_size(const ldpc_graph *g, int64_t B, int max_iter, int early_stop) {
    if (!g || B < 0 || max_iter < 0) return fail(LDPC_EINVAL, "bad arguments");
    if (B == 0 || max_iter == 0) return 0;
    if (use_stream(g, early_stop)) return stream_ws(g, B, max_iter, nullptr).bytes;
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
                   ? run_stream<LDPC_ALGO_MINSUM>(g, d_llr, B, max_iter, alpha, early_stop, out_dtype, d_bits, d_iters,
                                                  d_counters, d_batch_iters, d_work, s)
                   : run_stream<LDPC_ALGO_BP>(g, d_llr, B, max_iter, alpha, early_stop, out_dtype, d_bits, d_iters,
                                              d_counters, d_batch_iters, d_work, s);
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
#endif  // LDPC_FLOOD_KERNELS_ONLY
