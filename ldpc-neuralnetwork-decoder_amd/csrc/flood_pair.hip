// flood_pair.hip -- the frame-pair flooding kernel (flood_pair.inc) and its launcher.
#include "flood_host.hpp"

namespace ldpc {

#include "flood_pair.inc"

int launch_pair_kernel(int algo, int fixed_id, int64_t nwg, hipStream_t s, const float *llr, int64_t B,
                       int max_iter, float alpha, int out_dtype, void *bits, const Outs &O) {
    const void *kern = nullptr;
    size_t lds = 0;
    if (fixed_id == 1) {
        lds = pair_lds_bytes<fixed::BG2_Z4>();
        kern = algo == LDPC_ALGO_MINSUM ? reinterpret_cast<const void *>(flood_pair_kernel<fixed::BG2_Z4, LDPC_ALGO_MINSUM>)
                                        : reinterpret_cast<const void *>(flood_pair_kernel<fixed::BG2_Z4, LDPC_ALGO_BP>);
    } else if (fixed_id == 2) {
        lds = pair_lds_bytes<fixed::BG2_Z32>();
        kern = algo == LDPC_ALGO_MINSUM ? reinterpret_cast<const void *>(flood_pair_kernel<fixed::BG2_Z32, LDPC_ALGO_MINSUM>)
                                        : reinterpret_cast<const void *>(flood_pair_kernel<fixed::BG2_Z32, LDPC_ALGO_BP>);
    }
    if (!kern) return fail(LDPC_EINVAL, "no frame-pair kernel for this code");
    LDPC_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const float *l = llr;
    int64_t b = B;
    int mi = max_iter;
    float a = alpha;
    int od = out_dtype;
    void *bi = bits;
    Outs o = O;
    void *args[] = {&l, &b, &mi, &a, &od, &bi, &o};
    LDPC_HIP(hipLaunchKernel(kern, dim3((unsigned)nwg), dim3(512), args, lds, s));
    return LDPC_OK;
}

}  // namespace ldpc
