// v_pk_add_f32 vs v_add_f32 on denormal / special operands (is the packed add bit-identical to two
// scalar adds under the default float mode?).  hipcc --offload-arch=gfx950 -O2 pk_denorm.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k(const float *a, const float *b, float *s, float *p, int n) {
    int i = threadIdx.x;
    if (i >= n) return;
    float x = a[i], y = b[i];
    float r;
    asm volatile("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    s[i] = r;
    f2 xa = {x, x}, ya = {y, y}, rr;
    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(rr) : "v"(xa), "v"(ya));
    p[2 * i] = rr.x;
    p[2 * i + 1] = rr.y;
}
int main() {
    const int n = 8;
    float a[n] = {1e-40f, 1e-40f, -1e-39f, 1.0f, 1e-45f, 3e-38f, 0.0f, -0.0f};
    float b[n] = {0.0f, 1e-40f, 5e-40f, 1e-40f, -0.0f, -2.9e-38f, -0.0f, -0.0f};
    float *da, *db, *ds, *dp;
    hipMalloc(&da, 64); hipMalloc(&db, 64); hipMalloc(&ds, 64); hipMalloc(&dp, 128);
    hipMemcpy(da, a, sizeof a, hipMemcpyHostToDevice);
    hipMemcpy(db, b, sizeof b, hipMemcpyHostToDevice);
    k<<<1, 64>>>(da, db, ds, dp, n);
    float s[n], p[2 * n];
    hipMemcpy(s, ds, sizeof s, hipMemcpyDeviceToHost);
    hipMemcpy(p, dp, sizeof p, hipMemcpyDeviceToHost);
    int diff = 0;
    for (int i = 0; i < n; ++i) {
        unsigned us, up;
        memcpy(&us, &s[i], 4);
        memcpy(&up, &p[2 * i], 4);
        printf("%g + %g: scalar %g (0x%08x)  packed %g (0x%08x)\n", a[i], b[i], s[i], us, p[2 * i], up);
        diff += us != up;
    }
    printf("pk_denorm differing=%d\n", diff);
    return 0;
}
