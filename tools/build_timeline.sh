# Timeline build of the flooding decoders (-DLDPC_TIMELINE: s_memtime per wave per phase, see
# flood_dev.hpp) into ldpc_neural_decoder/_lib/variants/timeline<suffix>.so; extra flags pass through.
# usage: bash tools/build_timeline.sh [suffix] [-DFOO=1 ...]; select with LDPC_AMD_LIB=<path>
set -e
cd "$(dirname "$0")/../ldpc-neuralnetwork-decoder_amd"
N=timeline${1}; shift || true
mkdir -p build/var_$N ldpc_neural_decoder/_lib/variants
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -DLDPC_TIMELINE $*"
for S in flood.hip flood_fixed_ms.hip flood_fixed_bp.hip; do
  /opt/rocm/bin/hipcc $F -fno-slp-vectorize -x hip -c csrc/$S -o build/var_$N/$S.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ldpc_neural_decoder/_lib/variants/$N.so build/var_$N/*.o \
  $(ls build/*.o | grep -v "/flood.hip.o\|/flood_fixed_ms.hip.o\|/flood_fixed_bp.hip.o")
