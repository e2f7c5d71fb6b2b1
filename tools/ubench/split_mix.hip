// The f16 two-term split v = v0 + v1 (csrc/gnn.hpp split2h) two ways: v1 = f16(v - f32(v0)) by
// convert / subtract / convert, and v1 from one v_fma_mixlo/mixhi_f16 per value (fma(-v0, 1, v)
// rounded once to f16: the same value, since v - v0 is exact in f32).  Checks the two bit for bit
// over 2^24 inputs (all exponents, subnormals, inf, NaN).  hipcc --offload-arch=gfx950 -O2 split_mix.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
__global__ void k(const uint32_t *in, uint32_t *bad, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * i + 1 >= n) return;
    const float v0 = __uint_as_float(in[2 * i]), v1 = __uint_as_float(in[2 * i + 1]);
    // reference form
    const _Float16 a0 = (_Float16)v0, a1 = (_Float16)v1;
    const _Float16 r0 = (_Float16)(v0 - (float)a0), r1 = (_Float16)(v1 - (float)a1);
    // mix form
    const h2_t h = {(_Float16)v0, (_Float16)v1};
    const uint32_t hp = __builtin_bit_cast(uint32_t, h);
    uint32_t r;
    asm volatile("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hp), "v"(v0));
    asm volatile("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(r) : "v"(hp), "v"(v1));
    const uint32_t ref = (uint32_t)__builtin_bit_cast(uint16_t, r0) | ((uint32_t)__builtin_bit_cast(uint16_t, r1) << 16);
    const bool nan0 = v0 != v0 || (v0 - v0) != 0.0f, nan1 = v1 != v1 || (v1 - v1) != 0.0f;  // inf / NaN: any NaN ok
    const bool ok0 = nan0 ? ((r & 0x7c00u) == 0x7c00u && (r & 0x3ffu)) || (r & 0xffffu) == (ref & 0xffffu) : (r & 0xffffu) == (ref & 0xffffu);
    const bool ok1 = nan1 ? ((r >> 16 & 0x7c00u) == 0x7c00u && (r >> 16 & 0x3ffu)) || (r >> 16) == (ref >> 16) : (r >> 16) == (ref >> 16);
    if (!ok0 || !ok1) atomicAdd(bad, 1u);
}
int main() {
    const int n = 1 << 24;
    uint32_t *h = new uint32_t[n];
    uint64_t s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {  // xorshift bits: every exponent; plus the scaled range the kernels use
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        uint32_t b = (uint32_t)s;
        if (i % 4 == 1) b = (b & 0x807fffffu) | ((uint32_t)(100 + (s >> 40) % 50) << 23);  // |v| in 2^-27 .. 2^22
        if (i % 97 == 0) b = 0x7f800000u | (b & 0x80000000u);
        if (i % 89 == 0) b = 0x7fc00000u;
        h[i] = b;
    }
    uint32_t *din, *dbad;
    (void)hipMalloc(&din, (size_t)n * 4); (void)hipMalloc(&dbad, 4);
    (void)hipMemcpy(din, h, (size_t)n * 4, hipMemcpyHostToDevice);
    (void)hipMemset(dbad, 0, 4);
    k<<<n / 2 / 256, 256>>>(din, dbad, n);
    uint32_t bad = 0;
    (void)hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
    printf("split_mix: %u mismatching pairs of %d\n", bad, n / 2);
    return bad != 0;
}
