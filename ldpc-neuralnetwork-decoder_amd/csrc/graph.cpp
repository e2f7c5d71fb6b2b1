// graph.cpp -- host-side graph construction: QC detection, slot assignment, wave schedules.
//
// Replaces: traditional_decoders.py:26-40 / 161-175 and message_gnn_decoder.py:382-488 (the
// Python M x N loops that build index lists; 18.7 s at Z = 32 in the reference).  Here: O(E)
// per candidate lifting size, once per code, then one upload.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <numeric>
#include <string>
#include <thread>

#include "common.hpp"
#include "gen/fixed_codes.hpp"
#include "graph.hpp"

namespace ldpc {

static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
const char *last_error() { return g_last_error.c_str(); }

namespace {

// Is H (edge list) block-circulant at lifting z?  Fills blocks (row-major) on success.
bool try_lift(int M, int N, const std::vector<int32_t> &ec, const std::vector<int32_t> &ev, int z,
              std::vector<Block> &blocks) {
    if (M % z || N % z) return false;
    const int mb = M / z, nb = N / z;
    std::map<int64_t, std::pair<int, int>> shift_count;  // block -> (shift, count)
    for (size_t e = 0; e < ec.size(); ++e) {
        const int r = ec[e] / z, c = ev[e] / z;
        const int k = ec[e] % z, t = ev[e] % z;
        const int s = ((t - k) % z + z) % z;
        const int64_t key = (int64_t)r * nb + c;
        auto it = shift_count.find(key);
        if (it == shift_count.end()) {
            shift_count.emplace(key, std::make_pair(s, 1));
        } else {
            if (it->second.first != s) return false;
            ++it->second.second;
        }
    }
    blocks.clear();
    for (auto &kv : shift_count) {
        if (kv.second.second != z) return false;
        blocks.push_back({(int)(kv.first / nb), (int)(kv.first % nb), kv.second.first});
    }
    (void)mb;
    return true;  // std::map iterates keys ascending = row-major, c ascending
}

// Longest-processing-time-first assignment of tasks to W waves.
void schedule(const std::vector<int> &tasks, const std::vector<double> &cost, int W,
              std::vector<int32_t> &ptr, std::vector<int32_t> &list) {
    std::vector<int> order(tasks.size());
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return cost[a] > cost[b]; });
    std::vector<std::vector<int>> per(W);
    std::vector<double> load(W, 0.0);
    for (int i : order) {
        int w = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        per[w].push_back(tasks[i]);
        load[w] += cost[i];
    }
    ptr.assign(W + 1, 0);
    list.clear();
    for (int w = 0; w < W; ++w) {
        std::sort(per[w].begin(), per[w].end());
        list.insert(list.end(), per[w].begin(), per[w].end());
        ptr[w + 1] = (int32_t)list.size();
    }
}

// Device CSR tables of the streaming decoder: checks' edges (check-major = edge order) and, for
// every variable, its edge ids in ascending check order (traditional_decoders.py:26-40).
int build_csr(ldpc_graph *g) {
    const int M = g->M, N = g->N;
    const int64_t E = g->E;
    std::vector<int32_t> blob((size_t)(M + 1) + E + (N + 1) + E + M + N + E, 0);
    int32_t *cp = blob.data(), *ev = cp + M + 1, *vp = ev + E, *ve = vp + N + 1, *ro = ve + E, *co = ro + M,
            *xv = co + N;
    for (int64_t e = 0; e < E; ++e) {
        ++cp[g->edge_chk[e] + 1];
        ev[e] = g->edge_var[e];
        ++vp[g->edge_var[e] + 1];
    }
    for (int i = 0; i < M; ++i) cp[i + 1] += cp[i];
    for (int j = 0; j < N; ++j) vp[j + 1] += vp[j];
    std::vector<int32_t> fill(vp, vp + N);
    for (int64_t e = 0; e < E; ++e) ve[fill[g->edge_var[e]]++] = (int32_t)e;  // edges ascend = checks ascend
    // nodes grouped by degree, ascending index inside a degree
    auto group = [](const int32_t *ptr, int n, int32_t *order, std::vector<int> &seg) {
        std::vector<int> idx(n);
        for (int i = 0; i < n; ++i) idx[i] = i;
        std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return ptr[a + 1] - ptr[a] < ptr[b + 1] - ptr[b]; });
        seg.clear();
        for (int k = 0; k < n; ++k) {
            order[k] = idx[k];
            const int d = ptr[idx[k] + 1] - ptr[idx[k]];
            if (seg.empty() || seg[seg.size() - 3] != d) seg.insert(seg.end(), {d, k, 0});
            ++seg.back();
        }
    };
    for (int64_t e = 0; e < E; ++e) {
        const int v = g->edge_var[e];
        xv[e] = vp[v + 1] - vp[v] == 1 ? v : -1;
    }
    group(cp, M, ro, g->row_seg);
    group(vp, N, co, g->col_seg);
    LDPC_HIP(hipMalloc(&g->d_csr, blob.size() * sizeof(int32_t)));
    LDPC_HIP(hipMemcpy(g->d_csr, blob.data(), blob.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    g->chk_ptr = g->d_csr;
    g->ev = g->chk_ptr + M + 1;
    g->var_ptr = g->ev + E;
    g->var_edge = g->var_ptr + N + 1;
    g->row_order = g->var_edge + E;
    g->col_order = g->row_order + M;
    g->ext_var = g->col_order + N;
    return LDPC_OK;
}

int build(ldpc_graph *g) {
    const int M = g->M, N = g->N;
    if (int rc = build_csr(g)) return rc;
    // choose the lifting: the largest z dividing 64 that H is block-circulant for, so that a
    // wave's 64 lanes are exactly FG = 64/z frames x z rows (every lane owns a position; no
    // lane predicates on the hot path).  z = 1 (one frame per lane) always works.
    int best = 1;
    std::vector<Block> blocks, cand;
    try_lift(M, N, g->edge_chk, g->edge_var, 1, blocks);
    for (int z = 2; z <= 64; z *= 2) {
        if (M % z || N % z) continue;
        if (!try_lift(M, N, g->edge_chk, g->edge_var, z, cand)) continue;
        best = z;
        blocks = cand;
    }
    g->Z = best;
    g->FG = 64 / best;
    g->Mb = M / best;
    g->Nb = N / best;
    g->blocks = blocks;
    const int Mb = g->Mb, Nb = g->Nb;

    std::vector<int> dv(Nb, 0), dc(Mb, 0);
    for (auto &b : blocks) { ++dv[b.c]; ++dc[b.r]; }
    g->max_dc = Mb ? *std::max_element(dc.begin(), dc.end()) : 0;
    g->max_dv = Nb ? *std::max_element(dv.begin(), dv.end()) : 0;

    // slots: blocks of columns with degree >= 2
    std::vector<int32_t> slot_of(blocks.size(), -1);
    int nslots = 0;
    for (size_t i = 0; i < blocks.size(); ++i)
        if (dv[blocks[i].c] >= 2) slot_of[i] = nslots++;
    g->nslots = nslots;

    // schedules (cost in VALU-ish units per lane vector), LPT over W waves
    const int W = std::min(kMaxWaves, 4);
    std::vector<std::vector<int>> row_blocks(Mb), col_blocks(Nb);
    for (size_t i = 0; i < blocks.size(); ++i) {
        row_blocks[blocks[i].r].push_back((int)i);  // c ascending (row-major order)
        col_blocks[blocks[i].c].push_back((int)i);  // r ascending
    }
    std::vector<int> rtasks(Mb), vtasks, btasks(Nb);
    std::vector<double> rcost(Mb), vcost, bcost(Nb, 1.0);
    for (int r = 0; r < Mb; ++r) { rtasks[r] = r; rcost[r] = 6.0 * dc[r] + 0.5 * dc[r] * dc[r] + 8; }
    for (int c = 0; c < Nb; ++c) {
        if (dv[c] == 1) continue;
        vtasks.push_back(c);
        vcost.push_back(0.5 * dv[c] * (dv[c] + 1) + 4.0 * dv[c] + 6);
    }
    for (int c = 0; c < Nb; ++c) btasks[c] = c;
    std::vector<int32_t> cw_ptr, cw_task, vw_ptr, vw_task, bw_ptr, bw_task;
    schedule(rtasks, rcost, W, cw_ptr, cw_task);
    schedule(vtasks, vcost, W, vw_ptr, vw_task);
    schedule(btasks, bcost, W, bw_ptr, bw_task);

    // programs
    std::vector<int32_t> chk, var, par, prog_ptr(4 * (W + 1), 0);
    for (int w = 0; w < W; ++w) {
        for (int q = cw_ptr[w]; q < cw_ptr[w + 1]; ++q) {
            const int r = cw_task[q];
            chk.push_back((int32_t)row_blocks[r].size());
            par.push_back((int32_t)row_blocks[r].size());
            for (int i : row_blocks[r]) {
                const Block &bk = blocks[i];
                if (slot_of[i] >= 0)
                    chk.push_back((slot_of[i] * 256) | ((4 * bk.s) << kShiftBit));
                else
                    chk.push_back(kExtFlag | bk.c | ((4 * bk.s) << kShiftBit));
                par.push_back(bk.c | (bk.s << kShiftBit));
            }
        }
        prog_ptr[w + 1] = (int32_t)chk.size();
        prog_ptr[2 * (W + 1) + w + 1] = (int32_t)par.size();
        for (int q = vw_ptr[w]; q < vw_ptr[w + 1]; ++q) {
            const int c = vw_task[q];
            var.push_back((int32_t)col_blocks[c].size() | (c << 8));
            for (int i : col_blocks[c]) var.push_back((slot_of[i] * 256) | ((4 * blocks[i].s) << kShiftBit));
        }
        prog_ptr[(W + 1) + w + 1] = (int32_t)var.size();
        prog_ptr[3 * (W + 1) + w + 1] = bw_ptr[w + 1];
    }
    if ((int64_t)nslots * 256 >= (1 << kShiftBit) || Nb >= (1 << kShiftBit) || g->max_dv >= 256) {
        // far beyond the LDS of a CU anyway: this graph decodes on the streaming kernels only
        g->lds_ok = false;
        LDPC_HIP(hipDeviceSynchronize());
        return LDPC_OK;
    }

    // one int32 blob on the device
    std::vector<int32_t> blob;
    auto put = [&](const std::vector<int32_t> &v) {
        size_t off = blob.size();
        blob.insert(blob.end(), v.begin(), v.end());
        blob.push_back(0);  // keep every table non-empty
        return off;
    };
    const size_t o_c = put(chk), o_v = put(var), o_p = put(par), o_b = put(bw_task), o_pp = put(prog_ptr);
    LDPC_HIP(hipGetDevice(&g->device));
    LDPC_HIP(hipMalloc(&g->d_tab, blob.size() * sizeof(int32_t)));
    LDPC_HIP(hipMemcpy(g->d_tab, blob.data(), blob.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    FloodTables &t = g->ft;
    t.chk_prog = g->d_tab + o_c;
    t.var_prog = g->d_tab + o_v;
    t.par_prog = g->d_tab + o_p;
    t.bw_task = g->d_tab + o_b;
    t.prog_ptr = g->d_tab + o_pp;
    t.Z = g->Z;
    t.FG = g->FG;
    t.Mb = Mb;
    t.Nb = Nb;
    t.N = N;
    t.nslots = nslots;
    t.W = W;
    t.rep1 = 0;
    for (int b = 0; b < 64; b += g->Z) t.rep1 |= 1ull << b;

    // compile-time schedule available for this exact graph (and the default 4 waves)?
    auto matches = [&](auto tag) {
        using G = decltype(tag);
        if (g->Z != G::Z || Mb != G::Mb || Nb != G::Nb || (int)blocks.size() != G::NBLOCKS || W != G::W) return false;
        for (int i = 0; i < G::NBLOCKS; ++i)
            if (blocks[i].r != G::BLK_ROW[i] || blocks[i].c != G::BLK_COL[i] || blocks[i].s != G::BLK_SHIFT[i])
                return false;
        return true;
    };
    g->fixed_match = matches(fixed::BG2_Z4{}) ? 1 : (matches(fixed::BG2_Z32{}) ? 2 : 0);
    const char *fx = std::getenv("LDPC_FLOOD_FIXED");
    g->fixed_id = (fx && std::atoi(fx) == 0) ? 0 : g->fixed_match;

    LDPC_HIP(hipDeviceSynchronize());
    return LDPC_OK;
}

}  // namespace
}  // namespace ldpc

using namespace ldpc;

extern "C" const char *ldpc_last_error(void) { return ldpc::last_error(); }
extern "C" const char *ldpc_version(void) { return "ldpc_amd 0.1.0 (gfx950)"; }

extern "C" int ldpc_graph_create(int M, int N, int64_t E, const int32_t *h_edge_chk,
                                 const int32_t *h_edge_var, ldpc_graph **out) {
    if (!out) return fail(LDPC_EINVAL, "out is NULL");
    *out = nullptr;
    if (M < 0 || N <= 0 || E < 0 || (E > 0 && (!h_edge_chk || !h_edge_var)))
        return fail(LDPC_EINVAL, "bad graph dimensions");
    auto *g = new ldpc_graph();
    g->M = M;
    g->N = N;
    g->E = E;
    g->edge_chk.assign(h_edge_chk, h_edge_chk + E);
    g->edge_var.assign(h_edge_var, h_edge_var + E);
    for (int64_t e = 0; e < E; ++e) {
        if (g->edge_chk[e] < 0 || g->edge_chk[e] >= M || g->edge_var[e] < 0 || g->edge_var[e] >= N) {
            delete g;
            return fail(LDPC_EINVAL, "edge index out of range");
        }
        if (e && (g->edge_chk[e] < g->edge_chk[e - 1] ||
                  (g->edge_chk[e] == g->edge_chk[e - 1] && g->edge_var[e] <= g->edge_var[e - 1]))) {
            delete g;
            return fail(LDPC_EINVAL, "edge list must be check-major, strictly ascending, no duplicates");
        }
    }
    int rc = build(g);
    if (rc != LDPC_OK) {
        ldpc_graph_destroy(g);
        return rc;
    }
    *out = g;
    return LDPC_OK;
}

extern "C" int ldpc_graph_create_qc(const int32_t *h_base, int mb, int nb, int z, ldpc_graph **out) {
    if (!h_base || mb <= 0 || nb <= 0 || z <= 0) return fail(LDPC_EINVAL, "bad base graph");
    std::vector<int32_t> ec, ev;
    for (int r = 0; r < mb; ++r)
        for (int k = 0; k < z; ++k)
            for (int c = 0; c < nb; ++c) {
                const int s = h_base[r * nb + c];
                if (s < 0) continue;
                ec.push_back(r * z + k);
                ev.push_back(c * z + (k + s % z) % z);
            }
    // inside a check row the vars must ascend: blocks are visited c ascending, and each block
    // contributes one var in [c*z, (c+1)*z), so the order is already ascending.
    return ldpc_graph_create(mb * z, nb * z, (int64_t)ec.size(), ec.data(), ev.data(), out);
}

extern "C" int ldpc_graph_destroy(ldpc_graph *g) {
    if (!g) return LDPC_OK;
    if (g->d_tab) (void)hipFree(g->d_tab);
    if (g->d_csr) (void)hipFree(g->d_csr);
    delete g;
    return LDPC_OK;
}

extern "C" int ldpc_graph_info(const ldpc_graph *g, int *M, int *N, int64_t *E, int *Z, int *max_dc,
                               int *max_dv) {
    if (!g) return fail(LDPC_EINVAL, "graph is NULL");
    if (M) *M = g->M;
    if (N) *N = g->N;
    if (E) *E = g->E;
    if (Z) *Z = g->Z;
    if (max_dc) *max_dc = g->max_dc;
    if (max_dv) *max_dv = g->max_dv;
    return LDPC_OK;
}

extern "C" int ldpc_graph_set_variant(ldpc_graph *g, int variant) {
    if (!g) return fail(LDPC_EINVAL, "graph is NULL");
    if (variant < 0 || variant > 1) return fail(LDPC_EINVAL, "variant must be 0 (auto) or 1 (table-driven)");
    g->fixed_id = variant == 1 ? 0 : g->fixed_match;
    return g->fixed_id;
}

extern "C" int ldpc_graph_edges(const ldpc_graph *g, int32_t *h_edge_chk, int32_t *h_edge_var) {
    if (!g) return fail(LDPC_EINVAL, "graph is NULL");
    if (h_edge_chk) std::memcpy(h_edge_chk, g->edge_chk.data(), g->E * sizeof(int32_t));
    if (h_edge_var) std::memcpy(h_edge_var, g->edge_var.data(), g->E * sizeof(int32_t));
    return LDPC_OK;
}
