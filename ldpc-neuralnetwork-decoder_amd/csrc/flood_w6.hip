// flood_w6.hip -- the 6-wave flooding kernel (flood_w6.inc) and its launcher.
#include "flood_host.hpp"

namespace ldpc {

#include "flood_w6.inc"

int launch_w6_kernel(int algo, int fixed_id, int64_t nwg, size_t lds, hipStream_t s, const FloodTables &T,
                     const float *llr, int64_t B, int max_iter, float alpha, int out_dtype, void *bits,
                     const Outs &O) {
    const void *kern = nullptr;
    if (fixed_id == 1)
        kern = algo == LDPC_ALGO_MINSUM ? reinterpret_cast<const void *>(flood_w6_kernel<fixed::BG2_Z4, LDPC_ALGO_MINSUM>)
                                        : reinterpret_cast<const void *>(flood_w6_kernel<fixed::BG2_Z4, LDPC_ALGO_BP>);
    else if (fixed_id == 2)
        kern = algo == LDPC_ALGO_MINSUM ? reinterpret_cast<const void *>(flood_w6_kernel<fixed::BG2_Z32, LDPC_ALGO_MINSUM>)
                                        : reinterpret_cast<const void *>(flood_w6_kernel<fixed::BG2_Z32, LDPC_ALGO_BP>);
    if (!kern) return fail(LDPC_EINVAL, "no 6-wave kernel for this code");
    LDPC_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    FloodTables t = T;
    const float *l = llr;
    int64_t b = B;
    int mi = max_iter;
    float a = alpha;
    int od = out_dtype;
    void *bi = bits;
    Outs o = O;
    void *args[] = {&t, &l, &b, &mi, &a, &od, &bi, &o};
    LDPC_HIP(hipLaunchKernel(kern, dim3((unsigned)nwg), dim3(384), args, lds, s));
    return LDPC_OK;
}

}  // namespace ldpc
