// flood_fixed_kernel<BG2_Z32, min-sum, ES off> alone, for ISA inspection (tools/valu_cost.py):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
//     -Ildpc-neuralnetwork-decoder_amd/csrc -x hip --cuda-device-only -S tools/ubench/flood_one.hip -o /tmp/flood_one.s
#include "flood_dev.hpp"
namespace ldpc {
template __global__ void flood_fixed_kernel<fixed::BG2_Z32, LDPC_ALGO_MINSUM, LDPC_ES_OFF>(FloodTables, const float *, int64_t, int, float, int, void *, Outs, EsWs);
}
