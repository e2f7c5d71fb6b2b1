// channel.hip -- on-device QPSK/BPSK + AWGN + LLR demodulation, and BER/FER counters.
//
// Replaces utils/channel.py:
//   qpsk_modulate   (:4-60)    s = 1/sqrt2 - b*sqrt2, I = even bits, Q = odd bits
//   awgn_channel    (:62-88)   n = randn * sqrt((1/snr)/2) per component
//   qpsk_demodulate (:90-154)  llr = 2*r / (1/snr), interleaved I, Q
//   AWGNChannel.transmit (:193-232) BPSK variant
//   compute_ber_fer (:156-190) as integer counters
// The float32 operation sequence is the reference's (each torch op rounds to float32, scalars are
// cast to float32 first), so the only difference from the reference is the normal generator:
// Philox-4x32-10 + Box-Muller here, torch's CPU mt19937 there (parity is statistical; see
// tests/test_channel_gpu.py; the fused arithmetic is pinned against oracle.awgn_llr there, and the
// reference-API functions against the reference's own seeded outputs in tests/test_channel_host.py).
// Compile with -ffp-contract=off so s + n*std does not fuse.
#include <cmath>
#include <cstdint>

#include "common.hpp"

namespace ldpc {
namespace {

struct u4 { uint32_t x, y, z, w; };

__host__ __device__ __forceinline__ u4 philox4x32_10(u4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// uniform in (0, 1): 24 random bits, centred in their interval (never 0, never 1)
__device__ __forceinline__ float u01(uint32_t x) { return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f); }

__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float &n0, float &n1) {
    const float r = sqrtf(-2.0f * logf(u01(a)));
    float sn, cs;
    sincosf(6.28318530717958647692f * u01(b), &sn, &cs);
    n0 = r * cs;
    n1 = r * sn;
}

constexpr uint32_t kStreamTag = 0xC4A77E11u;  // ctr.w of the channel stream

struct ChanParams {
    float inv_sqrt2, sqrt2;  // (float)(1/np.sqrt(2)), (float)np.sqrt(2)
    float noise_std;         // qpsk: (float)sqrt(noise_power/2);  bpsk: (float)(1/sqrt(snr))
    float denom;             // qpsk: (float)(1/snr);               bpsk: (float)(noise_std**2)
};

// one thread = two QPSK symbols = four coded bits of one frame
__global__ __launch_bounds__(256) void qpsk_awgn_kernel(uint32_t k0, uint32_t k1, uint64_t frame_offset,
                                                        ChanParams P, const uint8_t *__restrict__ tx,
                                                        int64_t B, int N, int pairs, float *__restrict__ llr) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t b = gid / pairs;
    const int j = (int)(gid - b * pairs);
    if (b >= B) return;
    const uint64_t fr = frame_offset + (uint64_t)b;
    const u4 r = philox4x32_10(u4{(uint32_t)j, (uint32_t)fr, (uint32_t)(fr >> 32), kStreamTag}, k0, k1);
    float n[4];
    box_muller(r.x, r.y, n[0], n[1]);  // symbol 2j:   real, imag
    box_muller(r.z, r.w, n[2], n[3]);  // symbol 2j+1: real, imag
    const int64_t row = b * (int64_t)N;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int bit = 4 * j + q;  // symbol 2j+q/2, component q&1 (I = even bit, Q = odd bit)
        if (bit >= N) break;
        const float bf = tx ? (float)tx[row + bit] : 0.0f;
        const float s = P.inv_sqrt2 - bf * P.sqrt2;     // qpsk_modulate (channel.py:39)
        const float noise = n[q] * P.noise_std;          // awgn_channel  (channel.py:81-82)
        const float rx = s + noise;                      // channel.py:86
        llr[row + bit] = (2.0f * rx) / P.denom;          // qpsk_demodulate (channel.py:137-143)
    }
}

// BPSK AWGNChannel.transmit: one thread = four bits, four normals
__global__ __launch_bounds__(256) void bpsk_awgn_kernel(uint32_t k0, uint32_t k1, uint64_t frame_offset,
                                                        ChanParams P, const uint8_t *__restrict__ tx,
                                                        int64_t B, int N, int quads, float *__restrict__ llr) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t b = gid / quads;
    const int j = (int)(gid - b * quads);
    if (b >= B) return;
    const uint64_t fr = frame_offset + (uint64_t)b;
    const u4 r = philox4x32_10(u4{(uint32_t)j, (uint32_t)fr, (uint32_t)(fr >> 32), kStreamTag ^ 1u}, k0, k1);
    float n[4];
    box_muller(r.x, r.y, n[0], n[1]);
    box_muller(r.z, r.w, n[2], n[3]);
    const int64_t row = b * (int64_t)N;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int bit = 4 * j + q;
        if (bit >= N) break;
        const float bf = tx ? (float)tx[row + bit] : 0.0f;
        const float sym = 1.0f - 2.0f * bf;               // channel.py:217
        const float rx = sym + n[q] * P.noise_std;         // channel.py:226-227
        llr[row + bit] = (2.0f * rx) / P.denom;           // channel.py:230
    }
}

__global__ void philox_raw_kernel(uint32_t k0, uint32_t k1, uint32_t c2, uint32_t c3, int64_t n,
                                  uint32_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u4 r = philox4x32_10(u4{(uint32_t)i, (uint32_t)((uint64_t)i >> 32), c2, c3}, k0, k1);
    out[4 * i + 0] = r.x;
    out[4 * i + 1] = r.y;
    out[4 * i + 2] = r.z;
    out[4 * i + 3] = r.w;
}

// one wave per frame: {bit errors, frame errors, frames}
template <typename T>
__global__ __launch_bounds__(256) void count_kernel(const T *__restrict__ bits, const uint8_t *__restrict__ ref,
                                                    int64_t B, int N, uint64_t *__restrict__ counters) {
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    uint64_t e = 0;
    if (b < B) {
        const T *row = bits + b * N;
        const uint8_t *rr = ref ? ref + b * N : nullptr;
        for (int v = lane; v < N; v += 64) {
            const int d = row[v] != (T)0;
            const int t = rr ? (rr[v] != 0) : 0;
            e += (uint64_t)(d != t);
        }
    }
    for (int off = 32; off > 0; off >>= 1) e += __shfl_xor(e, off, 64);
    if (lane == 0 && b < B) {
        atomicAdd((unsigned long long *)&counters[0], (unsigned long long)e);
        if (e) atomicAdd((unsigned long long *)&counters[1], 1ull);
        atomicAdd((unsigned long long *)&counters[2], 1ull);
    }
}

}  // namespace
}  // namespace ldpc

using namespace ldpc;

extern "C" int ldpc_awgn_llr(uint64_t seed, uint64_t frame_offset, float snr_db, const uint8_t *d_bits,
                             int64_t B, int N, int bpsk, float *d_llr, void *stream) {
    if (B < 0 || N <= 0) return fail(LDPC_EINVAL, "bad channel shape");
    if (B == 0) return LDPC_OK;
    if (!d_llr) return fail(LDPC_EINVAL, "llr is NULL");
    hipStream_t s = static_cast<hipStream_t>(stream);
    // host double arithmetic exactly as the reference's Python/numpy scalars
    const double snr_linear = std::pow(10.0, (double)snr_db / 10.0);
    ChanParams P;
    P.inv_sqrt2 = (float)(1.0 / std::sqrt(2.0));
    P.sqrt2 = (float)std::sqrt(2.0);
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    if (!bpsk) {
        const double noise_power = 1.0 / snr_linear;
        P.noise_std = (float)std::sqrt(noise_power / 2.0);
        P.denom = (float)(1.0 / snr_linear);
        const int pairs = (N + 3) / 4;
        const int64_t threads = B * pairs;
        hipLaunchKernelGGL(qpsk_awgn_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, k0, k1,
                           frame_offset, P, d_bits, B, N, pairs, d_llr);
    } else {
        const double noise_std = 1.0 / std::sqrt(snr_linear);
        P.noise_std = (float)noise_std;
        P.denom = (float)(noise_std * noise_std);
        const int quads = (N + 3) / 4;
        const int64_t threads = B * quads;
        hipLaunchKernelGGL(bpsk_awgn_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, k0, k1,
                           frame_offset, P, d_bits, B, N, quads, d_llr);
    }
    LDPC_CHECK_LAUNCH("awgn");
    return LDPC_OK;
}

extern "C" int ldpc_philox_raw(uint64_t seed, uint32_t ctr2, uint32_t ctr3, int64_t n_blocks, uint32_t *d_out,
                               void *stream) {
    if (n_blocks < 0) return fail(LDPC_EINVAL, "negative count");
    if (n_blocks == 0) return LDPC_OK;
    hipLaunchKernelGGL(philox_raw_kernel, dim3((unsigned)((n_blocks + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), (uint32_t)seed, (uint32_t)(seed >> 32), ctr2, ctr3,
                       n_blocks, d_out);
    LDPC_CHECK_LAUNCH("philox_raw");
    return LDPC_OK;
}

extern "C" int ldpc_count_errors(const void *d_bits, int bits_dtype, const uint8_t *d_ref, int64_t B, int N,
                                 uint64_t *d_counters, void *stream) {
    if (B < 0 || N <= 0 || !d_counters) return fail(LDPC_EINVAL, "bad count arguments");
    if (B == 0) return LDPC_OK;
    if (!d_bits) return fail(LDPC_EINVAL, "bits is NULL");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((B + 3) / 4));
    if (bits_dtype == LDPC_OUT_F32)
        hipLaunchKernelGGL(count_kernel<float>, grid, dim3(256), 0, s, static_cast<const float *>(d_bits), d_ref,
                           B, N, d_counters);
    else if (bits_dtype == LDPC_OUT_U8)
        hipLaunchKernelGGL(count_kernel<uint8_t>, grid, dim3(256), 0, s, static_cast<const uint8_t *>(d_bits),
                           d_ref, B, N, d_counters);
    else
        return fail(LDPC_EINVAL, "unknown bits dtype");
    LDPC_CHECK_LAUNCH("count_errors");
    return LDPC_OK;
}
