// NaN-propagating ReLU on bf16 bit patterns: v_pk_maximum3_f16 applied to the bf16 bits viewed as
// f16 (one instruction per two values, like the v_pk_max_i16 it would replace).  Checks all 65536
// patterns against torch.relu semantics: NaN stays a bf16 NaN, negatives (and -0) become +0 or -0,
// every other pattern (inf included) keeps its bits.  hipcc --offload-arch=gfx950 -O2 relu_bf16.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));
__global__ void k(const unsigned *in, unsigned *out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    h2 v = __builtin_bit_cast(h2, in[i]);
    h2 r = __builtin_elementwise_maximum(v, (h2)0);
    out[i] = __builtin_bit_cast(unsigned, r);
}
int main() {
    const int n = 32768;  // two patterns per word
    static unsigned h_in[n], h_out[n];
    for (int i = 0; i < n; ++i) h_in[i] = (unsigned)(2 * i) | ((unsigned)(2 * i + 1) << 16);
    unsigned *din, *dout;
    hipMalloc(&din, sizeof h_in); hipMalloc(&dout, sizeof h_out);
    hipMemcpy(din, h_in, sizeof h_in, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(din, dout, n);
    hipMemcpy(h_out, dout, sizeof h_out, hipMemcpyDeviceToHost);
    int bad = 0, nan_changed = 0;
    for (int w = 0; w < n; ++w)
        for (int h = 0; h < 2; ++h) {
            const unsigned b = (h_in[w] >> (16 * h)) & 0xffff, r = (h_out[w] >> (16 * h)) & 0xffff;
            const bool nan = (b & 0x7f80) == 0x7f80 && (b & 0x7f);
            const bool rnan = (r & 0x7f80) == 0x7f80 && (r & 0x7f);
            bool ok;
            if (nan) ok = rnan, nan_changed += r != b;
            else if (b & 0x8000) ok = (r & 0x7fff) == 0;
            else ok = r == b;
            if (!ok && bad++ < 16) printf("bf16 0x%04x -> 0x%04x\n", b, r);
        }
    printf("relu_bf16 f16-view maximum3: %d wrong of 65536 (NaN payloads changed: %d)\n", bad, nan_changed);
    return bad != 0;
}
