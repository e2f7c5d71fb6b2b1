# Build libldpc_amd.so with extra compile flags for one source (default flood.hip) into
# ldpc_neural_decoder/_lib/variants/<name>.so (A/B timing; select with LDPC_AMD_LIB=<path>).
# usage: [SRC=gnn.hip] bash tools/build_variant.sh <name> -DFOO=1 ...
set -e
cd "$(dirname "$0")/../ldpc-neuralnetwork-decoder_amd"
N=$1; shift
S=${SRC:-flood_fixed_ms.hip}
mkdir -p build/var_$N ldpc_neural_decoder/_lib/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function "$@" -x hip -c csrc/$S -o build/var_$N/$S.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ldpc_neural_decoder/_lib/variants/$N.so build/var_$N/$S.o $(ls build/*.o | grep -v "/$S.o")
