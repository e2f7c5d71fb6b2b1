// graph.hpp -- device-resident Tanner graph, quasi-cyclic layout and per-wave schedules.
//
// Replaces the reference's per-call Python index building:
//   traditional_decoders.py:26-40 / 161-175 (_precompute_indices: check_to_var / var_to_check)
//   message_gnn_decoder.py:382-488 (TannerToMessageGraph: check-major edge list, groups)
//
// Layout (see DESIGN.md "Data layout"):
//   The graph is lifted: H = [block (r, c) = cyclic shift s of I_Z, or 0].  A non-QC H is the
//   Z = 1 case.  One wave-wide "lane vector" is FG = 64 / Z frames x Z rows: lane l = f * Z + k.
//   Every block of a column with degree >= 2 owns one LDS "slot" of 64 floats holding, for each
//   lane, the message on the edge (check r*Z + k, var c*Z + (k + s) % Z) of frame f.  Slots are
//   indexed by the CHECK row k, so the check update reads slot[lane] unrotated and the variable
//   update reads slot[f*Z + (t - s) mod Z] (a permutation inside a Z-lane group: no bank
//   conflicts).  Degree-1 columns own no slot: their v2c is the channel LLR forever.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

namespace ldpc {

constexpr int kMaxWaves = 8;     // waves per flood workgroup (runtime W <= this)
constexpr int kMaxUnroll = 24;   // check/var degrees handled by unrolled register code

// Device view of the flooding schedule: per-wave "programs" (int32 streams, read through the
// constant address space so that every word is a scalar load).  Passed by value.
//   check program, per block-row: header dc, then dc edge words
//       slot edge:  slot_byte_offset | (4*shift) << 18
//       degree-1:   0x80000000 | col | (4*shift) << 18      (v2c is the channel LLR)
//   var program, per column with degree != 1: header dv | col << 8, then dv edge words
//       slot_byte_offset | (4*shift) << 18                  (blocks in ascending row order)
//   parity program, per block-row: header dc, then dc words col | shift << 18
//   bit-emission list: the columns each wave writes out
// prog_ptr holds 4 x (W+1) offsets: [chk | var | par | bw] per wave.
struct FloodTables {
    const int32_t *chk_prog, *var_prog, *par_prog, *bw_task, *prog_ptr;
    int Z, FG, Mb, Nb, N, nslots;
    int W;  // waves per workgroup
    uint64_t rep1;  // a 1 at the bottom of every Z-bit segment of a 64-bit ballot
};
constexpr int32_t kExtFlag = (int32_t)0x80000000u;
constexpr int kShiftBit = 18;
constexpr int32_t kLowMask = (1 << kShiftBit) - 1;

struct Block { int r, c, s; };

}  // namespace ldpc

struct ldpc_graph {
    int device = 0;
    int M = 0, N = 0;
    int64_t E = 0;
    int Z = 1, Mb = 0, Nb = 0, FG = 64;
    int max_dc = 0, max_dv = 0;
    int nslots = 0;
    std::vector<int32_t> edge_chk, edge_var;   // check-major
    std::vector<ldpc::Block> blocks;            // row-major (r asc, c asc)
    int32_t *d_tab = nullptr;
    ldpc::FloodTables ft{};
    int fixed_id = 0;      // 0: table-driven kernel; 1/2: compile-time schedule BG2_Z4 / BG2_Z32
    int fixed_match = 0;   // what the graph matched (kept when the variant is forced off)
    bool lds_ok = true;    // the LDS-resident schedule exists (its encoding fits); else stream only
    // streaming decoder (flood.hip, any graph): check-major CSR + per-variable edge lists
    int32_t *d_csr = nullptr;  // chk_ptr[M+1] edge_var[E] var_ptr[N+1] var_edge[E]
    const int32_t *chk_ptr = nullptr, *ev = nullptr, *var_ptr = nullptr, *var_edge = nullptr;
    // checks / variables grouped by degree (stable): the streaming kernels run one launch per
    // degree, so each is compiled for its degree alone (registers, and occupancy, of that degree)
    const int32_t *row_order = nullptr, *col_order = nullptr;
    const int32_t *ext_var = nullptr;   // per edge: its variable if that has degree 1, else -1
    std::vector<int> row_seg, col_seg;  // {degree, offset into *_order, count} triples
};
