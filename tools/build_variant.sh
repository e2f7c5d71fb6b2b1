# Build libldpc_amd.so with extra compile flags for one source (default flood.hip) into
# ab/<name>.so (A/B timing with tools/gpu_ab.sh; select with LDPC_AMD_LIB=<path>).
# usage: [SRC=gnn.hip] bash tools/build_variant.sh <name> -DFOO=1 ...
set -e
cd "$(dirname "$0")/../ldpc-neuralnetwork-decoder_amd"
N=$1; shift
S=${SRC:-flood_fixed_ms.hip}
mkdir -p build/var_$N ../ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function "$@" -x hip -c csrc/$S -o build/var_$N/$S.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../ab/$N.so build/var_$N/$S.o $(ls build/*.o | grep -v "/$S.o")
