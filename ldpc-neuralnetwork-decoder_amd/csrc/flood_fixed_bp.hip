// flood_fixed_bp.hip -- flood_fixed_kernel instances for sum-product (BP) (compile-time schedules of the reference's codes).
// Split out of flood.hip so that the kernel families compile in parallel.
#include "flood_host.hpp"

namespace ldpc {

int launch_fixed_bp(int fixed_id, int es, dim3 grid, dim3 block, size_t lds, hipStream_t s,
                    const FloodTables &T, const float *llr, int64_t B, int max_iter, float alpha,
                    int out_dtype, void *bits, const Outs &O, const EsWs &W) {
    auto pick = [&](auto code) -> const void * {
        using G = decltype(code);
        switch (es) {
            case LDPC_ES_OFF: return reinterpret_cast<const void *>(flood_fixed_kernel<G, LDPC_ALGO_BP, LDPC_ES_OFF>);
            case LDPC_ES_FRAME: return reinterpret_cast<const void *>(flood_fixed_kernel<G, LDPC_ALGO_BP, LDPC_ES_FRAME>);
            case LDPC_ES_BATCH: return reinterpret_cast<const void *>(flood_fixed_kernel<G, LDPC_ALGO_BP, LDPC_ES_BATCH>);
            case ES_P1: return reinterpret_cast<const void *>(flood_fixed_kernel<G, LDPC_ALGO_BP, ES_P1>);
            case ES_P2: return reinterpret_cast<const void *>(flood_fixed_kernel<G, LDPC_ALGO_BP, ES_P2>);
            default: return nullptr;
        }
    };
    const void *kern = fixed_id == 1 ? pick(fixed::BG2_Z4{}) : (fixed_id == 2 ? pick(fixed::BG2_Z32{}) : nullptr);
    if (!kern) return fail(LDPC_EINVAL, "no fixed kernel for this code / stopping mode");
    LDPC_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    FloodTables t = T;
    const float *l = llr;
    int64_t b = B;
    int mi = max_iter;
    float a = alpha;
    int od = out_dtype;
    void *bi = bits;
    Outs o = O;
    EsWs w = W;
    void *args[] = {&t, &l, &b, &mi, &a, &od, &bi, &o, &w};
    LDPC_HIP(hipLaunchKernel(kern, grid, block, args, lds, s));
    return LDPC_OK;
}

}  // namespace ldpc
