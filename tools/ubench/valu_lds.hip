// Microbenchmark: SIMD issue cost of the instructions the flood kernel is built from, on gfx950.
// One workgroup per CU (grid = CU count), W waves per workgroup (W/4 per SIMD); every wave runs a
// loop of 32 independent instructions of one kind (inline asm on 16 / 32 registers, so nothing is
// folded), timed with s_memtime (shader clock).  cycles per wave64 instruction per SIMD =
// (loop cycles) / (instructions per wave x waves per SIMD).
//   build: hipcc --offload-arch=gfx950 -O2 tools/ubench/valu_lds.hip -o tools/ubench/valu_lds
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

enum Op { ADD_F32, PK_ADD_F32, MED3_F32, BITOP3, CNDMASK, CMP_EQ_F32, DS_READ_B32, DS_READ2ST64_B32, DS_WRITE_B32, NOP0, NUM_OPS };
static const char *kName[NUM_OPS] = {"v_add_f32", "v_pk_add_f32", "v_med3_f32", "v_bitop3_b32", "v_cndmask_b32",
                                     "v_cmp_eq_f32(sgpr)", "ds_read_b32", "ds_read2st64_b32", "ds_write_b32", "s_nop 0"};

constexpr int kIters = 256;

template <int OP>
__global__ __launch_bounds__(1024) void kern(float *out, unsigned long long *cyc, float seed) {
    __shared__ float lds[16384];
    const int t = threadIdx.x;
    for (int i = t; i < 16384; i += blockDim.x) lds[i] = seed + i;
    __syncthreads();
    float a0 = seed + t, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b0 = a0 * 2, b1 = a1 * 2, b2 = a2 * 2, b3 = a3 * 2, b4 = a4 * 2, b5 = a5 * 2, b6 = a6 * 2, b7 = a7 * 2;
    const float c = seed * 0.5f;
    int addr = (t & 63) * 4 + (t >> 6) * 2048;
    unsigned long long k0 = 0, k1 = 0, k2 = 0, k3 = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
#define R8(X) X(a0) X(a1) X(a2) X(a3) X(a4) X(a5) X(a6) X(a7) X(b0) X(b1) X(b2) X(b3) X(b4) X(b5) X(b6) X(b7)
        if constexpr (OP == ADD_F32) {
#define X(r) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r) : "v"(c));
            R8(X) R8(X)
#undef X
        } else if constexpr (OP == PK_ADD_F32) {
#define X(r) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*(double *)&r) : "v"(*(double *)&b0));
            // 16 pairs: (a0,a1) (a2,a3) ... as 64-bit register pairs
            double p0 = 0, p1 = 0, p2 = 0, p3 = 0, p4 = 0, p5 = 0, p6 = 0, p7 = 0, q = c;
#undef X
#define X(r) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(r) : "v"(q));
            X(p0) X(p1) X(p2) X(p3) X(p4) X(p5) X(p6) X(p7) X(p0) X(p1) X(p2) X(p3) X(p4) X(p5) X(p6) X(p7)
            X(p0) X(p1) X(p2) X(p3) X(p4) X(p5) X(p6) X(p7) X(p0) X(p1) X(p2) X(p3) X(p4) X(p5) X(p6) X(p7)
#undef X
            a0 += (float)(p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7);
        } else if constexpr (OP == MED3_F32) {
#define X(r) asm volatile("v_med3_f32 %0, %0, |%1|, %2" : "+v"(r) : "v"(c), "v"(b0));
            R8(X) R8(X)
#undef X
        } else if constexpr (OP == BITOP3) {
#define X(r) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r) : "v"(c), "v"(b0));
            R8(X) R8(X)
#undef X
        } else if constexpr (OP == CNDMASK) {
            asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(k0) : "v"(a0), "v"(c));
            asm volatile("s_nop 4");
#define X(r) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(r) : "v"(c), "s"(k0));
            R8(X) R8(X)
#undef X
        } else if constexpr (OP == CMP_EQ_F32) {
#define X(r) asm volatile("v_cmp_eq_f32_e64 %0, |%1|, %2" : "=s"(k1) : "v"(r), "v"(c)); k2 ^= k1;
            R8(X) R8(X)
#undef X
        } else if constexpr (OP == DS_READ_B32) {
#define X(r) asm volatile("ds_read_b32 %0, %1 offset:256" : "=v"(r) : "v"(addr));
            R8(X) R8(X)
#undef X
            asm volatile("s_waitcnt lgkmcnt(0)");
        } else if constexpr (OP == DS_READ2ST64_B32) {
            float2 u0, u1, u2, u3, u4, u5, u6, u7;
#define X(r) asm volatile("ds_read2st64_b32 %0, %1 offset0:2 offset1:3" : "=v"(r) : "v"(addr));
            X(u0) X(u1) X(u2) X(u3) X(u4) X(u5) X(u6) X(u7) X(u0) X(u1) X(u2) X(u3) X(u4) X(u5) X(u6) X(u7)
            X(u0) X(u1) X(u2) X(u3) X(u4) X(u5) X(u6) X(u7) X(u0) X(u1) X(u2) X(u3) X(u4) X(u5) X(u6) X(u7)
#undef X
            asm volatile("s_waitcnt lgkmcnt(0)");
            a0 += u0.x + u1.y + u2.x + u3.y + u4.x + u5.y + u6.x + u7.y;
        } else if constexpr (OP == DS_WRITE_B32) {
#define X(r) asm volatile("ds_write_b32 %0, %1 offset:512" : : "v"(addr), "v"(r) : "memory");
            R8(X) R8(X)
#undef X
            asm volatile("s_waitcnt lgkmcnt(0)");
        } else {
#define X(r) asm volatile("s_nop 0");
            R8(X) R8(X)
#undef X
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + t] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7 + (float)(k2 & 1);
    if ((t & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + (t >> 6)] = t1 - t0;
}

template <int OP>
int run(int cus, int wps, float *out, unsigned long long *cyc) {
    const int W = 4 * wps;
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(kern<OP>, dim3(cus), dim3(64 * W), 0, 0, out, cyc, 1.0f);
        CHECK(hipDeviceSynchronize());
        std::vector<unsigned long long> h(cus * W);
        CHECK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long mx = 0;
        for (auto v : h) mx = v > mx ? v : mx;
        // per SIMD: wps waves x 32 instructions x kIters
        const float cpi = (float)mx / ((float)wps * 32.0f * kIters);
        best = cpi < best ? cpi : best;
    }
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_wave64_instr_per_simd\": %.3f}\n", kName[OP], wps, best);
    return 0;
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    float *out;
    unsigned long long *cyc;
    CHECK(hipMalloc(&out, (size_t)cus * 1024 * 4));
    CHECK(hipMalloc(&cyc, (size_t)cus * 16 * 8));
    for (int wps : {1, 2, 4}) {
        run<ADD_F32>(cus, wps, out, cyc);
        run<PK_ADD_F32>(cus, wps, out, cyc);
        run<MED3_F32>(cus, wps, out, cyc);
        run<BITOP3>(cus, wps, out, cyc);
        run<CNDMASK>(cus, wps, out, cyc);
        run<CMP_EQ_F32>(cus, wps, out, cyc);
        run<DS_READ_B32>(cus, wps, out, cyc);
        run<DS_READ2ST64_B32>(cus, wps, out, cyc);
        run<DS_WRITE_B32>(cus, wps, out, cyc);
        run<NOP0>(cus, wps, out, cyc);
    }
    CHECK(hipFree(out));
    CHECK(hipFree(cyc));
    return 0;
}
