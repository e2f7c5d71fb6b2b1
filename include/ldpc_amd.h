/*
 * ldpc_amd.h -- C ABI of the MI355X-native LDPC decoding library (libldpc_amd.so).
 *
 * The reference (BananaFalls/LDPC-NeuralNetwork-Decoder) is pure Python/PyTorch and has no
 * FFI of its own; its hot-path interface is the set of Python calls listed next to each entry
 * point below.  The Python package ldpc_neural_decoder (this repo) keeps those Python
 * signatures and binds these symbols with ctypes.
 *
 * Conventions
 *   - Every pointer named d_* is DEVICE memory owned by the caller (e.g. torch tensors on a HIP
 *     device, passed as data_ptr()).  Host pointers are named h_*.
 *   - Work is enqueued on `stream` (a hipStream_t, passed as void*; NULL = the legacy default
 *     stream) and is asynchronous unless stated otherwise.  No entry point allocates device
 *     memory on the decode path: scratch is caller-provided (query its size first).
 *   - Return value: 0 on success, a negative LDPC_E* code on error; the message of the last
 *     error on the calling thread is available from ldpc_last_error().
 *   - Layouts follow the reference: LLRs are float32 (B, N) row-major (utils/channel.py:90-154),
 *     hard decisions are (B, N) row-major, 0/1, either uint8 or float32
 *     (traditional_decoders.py:101,252 returns float32).
 */
#ifndef LDPC_AMD_H
#define LDPC_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    LDPC_OK = 0,
    LDPC_EINVAL = -1,       /* bad argument */
    LDPC_EHIP = -2,         /* HIP runtime error */
    LDPC_EUNSUPPORTED = -3, /* shape/degree outside what the kernels support */
    LDPC_ENOMEM = -4
};

enum { LDPC_ALGO_MINSUM = 0, LDPC_ALGO_BP = 1 };
enum { LDPC_ES_OFF = 0, LDPC_ES_BATCH = 1, LDPC_ES_FRAME = 2 };
enum { LDPC_OUT_U8 = 0, LDPC_OUT_F32 = 1 };

typedef struct ldpc_graph ldpc_graph; /* opaque: a Tanner graph resident on one device */

/* Last error message of the calling thread ("" if none). */
const char *ldpc_last_error(void);
/* Library version string. */
const char *ldpc_version(void);

/* ------------------------------------------------------------------ graph (setup, host-sync)
 * Replaces: the per-decoder Python setup loops
 *   traditional_decoders.py:26-40 / 161-175  (_precompute_indices over a dense H)
 *   message_gnn_decoder.py:382-488           (TannerToMessageGraph edge list + groups)
 * The edge list is check-major (checks ascending, vars ascending inside a check), i.e. the
 * order of TannerToMessageGraph.messages (message_gnn_decoder.py:397-406).  The library
 * detects quasi-cyclic structure (largest lifting Z <= 64 that H is block-circulant for) and
 * builds the per-wave schedules; a non-QC H is handled as Z = 1.
 * Tables are uploaded to the current HIP device; the call synchronizes. */
int ldpc_graph_create(int M, int N, int64_t E, const int32_t *h_edge_chk,
                      const int32_t *h_edge_var, ldpc_graph **out);
/* Base-graph form: replaces load_base_matrix + expand_base_matrix (ldpc_utils.py:97-147),
 * h_base is (mb, nb) int32 with -1 for a zero block; shifts are taken modulo z. */
int ldpc_graph_create_qc(const int32_t *h_base, int mb, int nb, int z, ldpc_graph **out);
int ldpc_graph_destroy(ldpc_graph *g);
/* M, N, E, detected lifting Z, max check degree, max variable degree. */
int ldpc_graph_info(const ldpc_graph *g, int *M, int *N, int64_t *E, int *Z, int *max_dc,
                    int *max_dv);
/* Kernel variant for this graph: 0 = auto (a compile-time schedule when the graph is one of the
 * reference's shipped codes, else table-driven), 1 = always table-driven.  Returns the variant
 * in use (0 table-driven, 1 BG2 Z=4, 2 BG2 Z=32) or a negative error. */
int ldpc_graph_set_variant(ldpc_graph *g, int variant);
/* Check-major edge list of the graph (E entries each) -- the reference's message order. */
int ldpc_graph_edges(const ldpc_graph *g, int32_t *h_edge_chk, int32_t *h_edge_var);

/* ------------------------------------------------------------------ flooding BP / min-sum
 * Replaces: MinSumScaledDecoder.decode  (traditional_decoders.py:177-260, alpha = scaling_factor)
 *           BeliefPropagationDecoder.decode (traditional_decoders.py:42-109, alpha ignored)
 * early_stop: LDPC_ES_OFF, LDPC_ES_BATCH (the reference's rule: stop at the first iteration at
 *   which ALL B frames satisfy H x = 0, traditional_decoders.py:104-107), LDPC_ES_FRAME
 *   (per-frame freeze at the first valid iteration; no reference counterpart).
 * d_llr     (B, N) float32
 * d_bits    (B, N) uint8 or float32 (out_dtype), 0/1, bit = (APP < 0)
 * d_iters   optional (B,) int32: iterations each frame ran (all equal unless LDPC_ES_FRAME)
 * d_batch_iters optional int32 scalar: the reference's returned `iterations`
 * d_counters optional uint64[4] += {bit errors vs the all-zero codeword, frame errors,
 *   frames, sum of per-frame iterations} -- the all-zero transmit of every reference harness
 *   (comparative_evaluation.py:133); counting is fused into the decoder's epilogue.
 * d_work / work_bytes: scratch of ldpc_flood_workspace_size(...) bytes, required for
 *   LDPC_ES_BATCH and whenever d_counters (or d_batch_iters with LDPC_ES_FRAME) is given: the
 *   counters are reduced through per-workgroup rows, not same-address atomics.
 * LDPC_ES_BATCH runs as passes on the stream (first all-valid iteration per workgroup, then the
 *   batch's candidate T, then -- only if some frame is invalid at T -- the exhaustive search);
 *   it never synchronises with the host. */
int64_t ldpc_flood_workspace_size(const ldpc_graph *g, int64_t B, int max_iter, int early_stop);
int ldpc_flood_decode(const ldpc_graph *g, int algo, const float *d_llr, int64_t B, int max_iter,
                      float alpha, int early_stop, int out_dtype, void *d_bits, int32_t *d_iters,
                      int32_t *d_batch_iters, uint64_t *d_counters, void *d_work,
                      int64_t work_bytes, void *stream);

/* ------------------------------------------------------------------ hybrid min-sum
 * Replaces: CustomMinSumMessageGNNDecoder.forward (models/message_gnn_decoder.py:1167-1251) with
 * CustomVariableMessageGNNLayer.variable_layer_update (:611-670) and
 * CustomCheckMessageGNNLayer.check_layer_update (:976-1044).  The reference cannot run these
 * (SURVEY.md section 0); the semantics this build defines from them (total-minus-own variable update,
 * damping 0.5 with the incoming c2v from the second iteration on, unscaled min-sum check update,
 * probs = sigmoid(llr + sum of c2v)) are spelled out in csrc/flood.hip and DESIGN.md.
 * d_llr (B, N) float32 -> d_probs (B, N) float32.  No early stop (the reference has none).
 * d_work: ldpc_custom_minsum_workspace_size(g, B) bytes.  B <= 4194240 per call. */
int64_t ldpc_custom_minsum_workspace_size(const ldpc_graph *g, int64_t B);
int ldpc_custom_minsum_decode(const ldpc_graph *g, const float *d_llr, int64_t B, int iterations,
                              float *d_probs, void *d_work, int64_t work_bytes, void *stream);

/* ------------------------------------------------------------------ channel
 * Replaces: qpsk_modulate -> awgn_channel -> qpsk_demodulate (utils/channel.py:4-154) fused:
 *   s = 1/sqrt2 - b*sqrt2 (I = even bits, Q = odd bits), n ~ N(0, (1/snr)/2) per component,
 *   llr = 2*(s+n) / (1/snr), all in float32 as the reference rounds them.
 * Noise comes from Philox-4x32-10 keyed by `seed`, counter = (frame_offset + b, symbol), so a
 * frame's LLRs depend only on (seed, its global frame index, snr): ranks of a sharded sweep
 * draw disjoint streams by passing disjoint frame_offset.
 * d_bits optional (B, N) uint8 transmitted bits (NULL = the all-zero codeword).
 * bpsk != 0 selects AWGNChannel.transmit instead (utils/channel.py:193-232). */
int ldpc_awgn_llr(uint64_t seed, uint64_t frame_offset, float snr_db, const uint8_t *d_bits,
                  int64_t B, int N, int bpsk, float *d_llr, void *stream);
/* Raw Philox-4x32-10 stream (for known-answer tests): out[4*i + j] = word j of block
 * (counter = {i lo, i hi, ctr2, ctr3}, key = seed). */
int ldpc_philox_raw(uint64_t seed, uint32_t ctr2, uint32_t ctr3, int64_t n_blocks,
                    uint32_t *d_out, void *stream);

/* ------------------------------------------------------------------ BER / FER
 * Replaces: compute_ber_fer (utils/channel.py:156-190) as integer counts:
 * d_counters uint64[3] += {bit errors, frame errors, frames}.  d_ref NULL = all-zero codeword.
 * bits_dtype: LDPC_OUT_U8 / LDPC_OUT_F32 (a decision is "1" iff the value != 0). */
int ldpc_count_errors(const void *d_bits, int bits_dtype, const uint8_t *d_ref, int64_t B, int N,
                      uint64_t *d_counters, void *stream);

/* ------------------------------------------------------------------ message-centred GNN
 * Replaces: MessageGNNDecoder.forward (message_gnn_decoder.py:190-317) with its
 *           MessageGNNLayer.forward (:51-129) and decode_messages (:131-152).
 * The reference aggregates with dense normalized adjacencies D^-1/2 (A+I) D^-1/2 over the
 * messages that share a variable / a check (:410-469); those are group means.  A plan holds
 * the two groupings (message -> variable group, message -> check group) and the kernels
 * compute segment means, O(E*H) instead of the reference's O(E^2*H) bmm.
 *
 * Weights: one contiguous float32 blob (H = hidden, T = message types, L = layers):
 *   w_in[H], b_in[H]                                  input_embedding (Linear(1,H))
 *   per layer l: emb[T*H]                             message_type_embeddings
 *                w1v[H*2H] b1v[H] w2v[H*H] b2v[H]     var_to_check_update.{0,2}
 *                w1c[H*2H] b1c[H] w2c[H*H] b2c[H]     check_to_var_update.{0,2}
 *                wo[H] bo[1]                          output_projection
 * (nn.Linear weights as stored: (out, in) row-major; ldpc_gnn_weights_size gives the count.)
 * d_msg_type (E,) int32 already padded/truncated/clamped to [0,T) (the Python layer does
 *   :68-81).  d_msg_var (E,) int32 message -> variable for the LLR gather and the output sum
 *   (the reference's message_to_var_mapping, or its column-0 quirk: :218-229 / :285-295).
 * precision: 0 = float32 features and fp32-accurate products (H = 64: scaled two-term f16 splits on
 *   the f16 MFMA, each weight matrix group under one power-of-two scale; H = 96..256: the same splits
 *   per weight slice; other widths: fp32 fma chains); 1 = bf16 MLP operands, fp32 accumulate.
 * d_probs (B, N) float32 = sigmoid(llr + sum of each variable's projected messages).
 * d_work: at least ldpc_gnn_workspace_size(plan, H, N, B, precision) bytes. */
typedef struct ldpc_gnn_plan ldpc_gnn_plan;
/* ldpc_gnn_forward_ex flags */
#define LDPC_GNN_EARLY_STOP 1 /* cfg5 per-frame early termination (bf16 path; see below) */
#define LDPC_GNN_FP32_PRODUCTS 2 /* fp32 path, H = 64: every product on the fp32 MFMA (see below) */
int ldpc_gnn_plan_create(int64_t E, int n_vgroups, const int32_t *h_vgroup, int n_cgroups,
                         const int32_t *h_cgroup, ldpc_gnn_plan **out);
/* General adjacencies: the reference runs a dense bmm with whatever (E x E) matrices it is given
 * (message_gnn_decoder.py:106-118), after zero-padding / cropping them to E (:93-104).  A CSR plan
 * takes each side as a CSR matrix (row m: the columns j with A[m][j] != 0, ascending, and the
 * values; h_*_ptr has E + 1 entries): every message then aggregates sum_j A[m][j] c[j] over its
 * own row.  fp32 forward only (precision 0); the bf16 path and training need a group plan. */
int ldpc_gnn_plan_create_csr(int64_t E, const int32_t *h_v_ptr, const int32_t *h_v_col, const float *h_v_val,
                             const int32_t *h_c_ptr, const int32_t *h_c_col, const float *h_c_val,
                             ldpc_gnn_plan **out);
int ldpc_gnn_plan_destroy(ldpc_gnn_plan *p);
/* Hybrid GNN (CustomVariableMessageGNNDecoder.forward, models/message_gnn_decoder.py:798-879 with
 * CustomVariableMessageGNNLayer.forward :672-755).  The reference cannot run it;
 * the semantics this build defines (check-side MLP + the layer's own output head, min-sum variable
 * update on those LLRs with damping 0.5, the decoder's Linear(1, H) back to features, mean-normalised
 * output) are spelled out in csrc/gnn.hip and DESIGN.md.  hidden must be 64; group plans only.
 * Weights: the ldpc_gnn_forward blob.  d_probs (B, N). */
int64_t ldpc_gnn_custom_var_workspace_size(const ldpc_gnn_plan *p, int hidden, int N, int64_t B, int layers);
int ldpc_gnn_custom_var_forward(const ldpc_gnn_plan *p, int hidden, int types, int layers,
                                const float *d_weights, const int32_t *d_msg_type,
                                const int32_t *d_msg_var, const float *d_llr, int N, int64_t B,
                                float *d_probs, void *d_work, int64_t work_bytes, void *stream);
int64_t ldpc_gnn_weights_size(int hidden, int types, int layers);
int64_t ldpc_gnn_workspace_size(const ldpc_gnn_plan *p, int hidden, int N, int64_t B, int layers,
                                int precision);
int ldpc_gnn_forward(const ldpc_gnn_plan *p, int hidden, int types, int layers,
                     const float *d_weights, const int32_t *d_msg_type, const int32_t *d_msg_var,
                     const float *d_llr, int N, int64_t B, int precision, float *d_probs,
                     void *d_work, int64_t work_bytes, void *stream);

/* ldpc_gnn_forward_ex: ldpc_gnn_forward plus flags and a per-frame layer count d_iters (B,) int32
 * (optional).  LDPC_GNN_EARLY_STOP (precision 1 only; a feature with no reference counterpart,
 * BASELINE cfg5): after every layer but the last, each frame still decoding takes the hard
 * decision [llr + sum of the LAST layer's output_projection over its messages > 0] on its current
 * features; a frame whose decision satisfies every parity check stops there, gets its probs from
 * that decision's soft values and d_iters = layers used; the others run on.
 * LDPC_GNN_FP32_PRODUCTS (precision 0): the products of W1_right g and of the MLP run on the fp32 MFMA
 * (H = 64) or as three-term bf16 splits (H = 96..256) instead of as scaled two-term f16 splits.  The
 * splits hold 22 bits of every weight whose row's largest |w| is at least 2^-17 of its matrix group's; a
 * caller whose weights span more (MessageGNNDecoder checks this per weight version) sets the flag to
 * keep fp32 accuracy. */
int ldpc_gnn_forward_ex(const ldpc_gnn_plan *p, int hidden, int types, int layers,
                        const float *d_weights, const int32_t *d_msg_type, const int32_t *d_msg_var,
                        const float *d_llr, int N, int64_t B, int precision, int flags, float *d_probs,
                        int32_t *d_iters, void *d_work, int64_t work_bytes, void *stream);

/* ---- training (fp32, hidden_dim <= 1024, any plan) ---------------------------------------------
 * Replaces torch autograd through MessageGNNDecoder.forward + F.binary_cross_entropy
 * (message_gnn_decoder.py:190-317, :314), as driven by trainer.py:70-102 (zero_grad, forward,
 * loss.backward(), SGD step).
 * ldpc_gnn_forward_train: the fp32 forward (same arguments as ldpc_gnn_forward, precision 0) that
 *   also writes every layer's output features to d_saved (L, B, E, H) float32.
 * ldpc_gnn_backward: given d_grad_probs = dLoss/dprobs (B, N), writes dLoss/dweights into
 *   d_grad_weights, laid out exactly like the weight blob (zeroed first).  The output_projection of
 *   every layer but the last gets zeros (the reference's forward never uses it: its grad is None).
 * Both take a workspace of ldpc_gnn_train_workspace_size(...) bytes. */
int64_t ldpc_gnn_train_workspace_size(const ldpc_gnn_plan *p, int hidden, int N, int64_t B, int layers);
int ldpc_gnn_forward_train(const ldpc_gnn_plan *p, int hidden, int types, int layers,
                           const float *d_weights, const int32_t *d_msg_type, const int32_t *d_msg_var,
                           const float *d_llr, int N, int64_t B, float *d_probs, float *d_saved,
                           void *d_work, int64_t work_bytes, void *stream);
int ldpc_gnn_backward(const ldpc_gnn_plan *p, int hidden, int types, int layers, const float *d_weights,
                      const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N,
                      int64_t B, const float *d_probs, const float *d_grad_probs, const float *d_saved,
                      float *d_grad_weights, void *d_work, int64_t work_bytes, void *stream);
/* Deep supervision (training extension, no reference counterpart; it is what makes the cfg5
 * per-frame early termination fire: the syndrome check decodes every layer's output through the
 * last layer's output_projection, so a model trained on the last layer's loss alone never yields a
 * codeword before the end).
 * ldpc_gnn_layer_probs: probs of every layer l < L - 1 through the LAST layer's output_projection,
 *   p_l[b][v] = sigmoid(llr + sum_{m -> v} (wo_L . x_{l+1}[b][m] + bo_L)) from d_saved, into
 *   d_layer_probs (L - 1, B, N); the output stage's own variable sums (ascending messages).
 *   Workspace: ldpc_gnn_train_workspace_size(...) bytes suffice.
 * ldpc_gnn_backward_ds: ldpc_gnn_backward plus dLoss/d(layer probs) (L - 1, B, N): each layer's
 *   head gradient is added to the feature gradient that arrives from above and to dwo_L / dbo_L.
 *   Both layer pointers null = ldpc_gnn_backward. */
int ldpc_gnn_layer_probs(const ldpc_gnn_plan *p, int hidden, int types, int layers, const float *d_weights,
                         const int32_t *d_msg_var, const float *d_llr, int N, int64_t B, const float *d_saved,
                         float *d_layer_probs, void *d_work, int64_t work_bytes, void *stream);
int ldpc_gnn_backward_ds(const ldpc_gnn_plan *p, int hidden, int types, int layers, const float *d_weights,
                         const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N,
                         int64_t B, const float *d_probs, const float *d_grad_probs, const float *d_saved,
                         const float *d_layer_probs, const float *d_grad_layer_probs, float *d_grad_weights,
                         void *d_work, int64_t work_bytes, void *stream);
/* Saved projections (round 5): the forward keeps every layer's projected group rows W1_s,right g_s +
 * b1_s and group means g_s (the fp32 path's gnn_group_proj_kernel outputs) in d_proj, so that the
 * backward does not recompute them.  hidden_dim 64 with a group plan; elsewhere the area is 0 floats
 * and the _ex functions behave as the ones above.
 * ldpc_gnn_train_proj_floats: float32 elements of d_proj = L * B * (Gv + Gc) * 2 * H, laid out per
 *   layer as [Pv (B, Gv, H) | Pc (B, Gc, H) | gv (B, Gv, H) | gc (B, Gc, H)].
 * ldpc_gnn_forward_train_ex / ldpc_gnn_backward_ds_ex: ldpc_gnn_forward_train / ldpc_gnn_backward_ds
 *   with d_proj (null = recompute in the backward).  The backward only reads d_proj. */
int64_t ldpc_gnn_train_proj_floats(const ldpc_gnn_plan *p, int hidden, int64_t B, int layers);
int ldpc_gnn_forward_train_ex(const ldpc_gnn_plan *p, int hidden, int types, int layers,
                              const float *d_weights, const int32_t *d_msg_type, const int32_t *d_msg_var,
                              const float *d_llr, int N, int64_t B, float *d_probs, float *d_saved, float *d_proj,
                              void *d_work, int64_t work_bytes, void *stream);
int ldpc_gnn_backward_ds_ex(const ldpc_gnn_plan *p, int hidden, int types, int layers, const float *d_weights,
                            const int32_t *d_msg_type, const int32_t *d_msg_var, const float *d_llr, int N,
                            int64_t B, const float *d_probs, const float *d_grad_probs, const float *d_saved,
                            const float *d_proj, const float *d_layer_probs, const float *d_grad_layer_probs,
                            float *d_grad_weights, void *d_work, int64_t work_bytes, void *stream);

/* ---- index-gather neural-BP layers (models/layers.py) ------------------
 * d_idx is the reference's (n_out, K) index tensor transposed to (K, n_out) int32, -1 = padding
 * (a zero value): d_idx[k * n_out + i]; inputs (B, n_in) fp32.
 * ldpc_gather_minsum   CheckLayer.forward (layers.py:14-66): out = prod sign(v + 1e-10) * min |v|
 *                      (|0| -> 1e10); d_argmin (B, n_out) int32 (optional) keeps torch.min's index.
 * ldpc_gather_sum      VariableLayer.forward (layers.py:78-125): out = llr + sum of gathered msgs
 *                      (d_llr NULL: out = the sum alone).  A row ends at its first -1: put the
 *                      padding last (for a sum, padding anywhere adds an exact +0.0).
 * ldpc_residual        ResidualLayer.forward (layers.py:143-168), h_prev = host array of `depth`
 *                      device pointers (depth <= 8).
 * ldpc_output_layer    OutputLayer.forward (layers.py:180-208): soft = sigmoid(final + llr); with
 *                      d_gt, max over n of the elementwise BCE (+ its argmax for the backward).
 * The *_backward entry points write torch autograd's input gradients of the same functions. */
int ldpc_gather_minsum(const float *d_in, int64_t B, int n_in, const int32_t *d_idx, int n_out, int K,
                       float *d_out, int32_t *d_argmin, void *stream);
/* ldpc_check_groups_minsum: the same CheckLayer outputs (no argmin) when the index is a set of
 * checks -- every edge's row holds exactly the other edges of its check (n_in == n_out == n), as
 * create_LLR_mapping builds it.  d_gptr (G + 1) / d_gmem (n) list each check's edges; K is the
 * index's row length (padding K > degree - 1 contributes the 1e10 of a zero entry). */
int ldpc_check_groups_minsum(const float *d_in, int64_t B, int n, const int32_t *d_gptr, const int32_t *d_gmem,
                             int G, int K, float *d_out, void *stream);
int ldpc_gather_minsum_backward(const float *d_grad_out, const float *d_in, int64_t B, int n_in,
                                const int32_t *d_idx, int n_out, int K, const int32_t *d_argmin,
                                float *d_grad_in, void *stream);
int ldpc_gather_sum(const float *d_llr, const float *d_msgs, int64_t B, int n_in, const int32_t *d_idx,
                    int n_out, int K, float *d_out, void *stream);
/* ldpc_var_groups_sum: the same VariableLayer outputs (layers.py:78-125) when the index is a set of
 * contiguous variable groups -- every edge's row holds exactly the other edges of its variable in
 * ascending order, and each variable's edges are a run [gptr[g], gptr[g + 1]) tiling [0, n)
 * (n_in == n_out == n), as create_LLR_mapping builds it.  Sums in the row's order, bit-identical
 * to ldpc_gather_sum.  d_out must not alias d_msgs or d_llr.  LDPC_EUNSUPPORTED when a row does
 * not fit LDS. */
int ldpc_var_groups_sum(const float *d_llr, const float *d_msgs, int64_t B, int n, const int32_t *d_gptr, int G,
                        float *d_out, void *stream);
int ldpc_gather_sum_backward(const float *d_grad_out, int64_t B, int n_in, const int32_t *d_idx, int n_out,
                             int K, float *d_grad_msgs, void *stream);
int ldpc_residual(const float *d_llr, const float *d_w_ch, const float *d_cm, const float *d_w_res,
                  const float *const *h_prev, int depth, int64_t B, int n, float *d_out, void *stream);
int ldpc_residual_backward(const float *d_grad, const float *d_llr, const float *d_w_ch,
                           const float *d_w_res, const float *const *h_prev, int depth, int64_t B, int n,
                           float *d_grad_llr, float *d_grad_w_ch, float *d_grad_w_res,
                           float *const *h_grad_prev, void *stream);
int ldpc_output_layer(const float *d_final, const float *d_llr, const float *d_gt, int64_t B, int n,
                      float *d_soft, float *d_max_loss, int32_t *d_argmax, void *stream);
int ldpc_output_layer_backward(const float *d_soft, const float *d_gt, const float *d_grad_soft,
                               const float *d_grad_loss, const int32_t *d_argmax, int64_t B, int n,
                               float *d_grad_z, void *stream);

/* ---- hybrid layers' per-message updates on index rows (message_gnn_decoder.py:611-670, :976-1044)
 * d_rows (R, W) int64 row-major: row m = [node, incoming message ids..., -1 padding]; ids index the
 * E_in columns of d_x / d_c2v (validated by the caller).  Outputs (B, R) fp32.
 * ldpc_index_rows_minsum  CustomCheckMessageGNNLayer.check_layer_update (:976-1044): the min-sum
 *                         update of the row's other entries, leaving out its last valid entry
 *                         (torch.sign / torch.min semantics; 0 without two valid entries).
 * ldpc_index_rows_varsum  CustomVariableMessageGNNLayer.variable_layer_update (:611-670):
 *                         (llr[b, node] + sum of the valid entries, ascending) - the last one;
 *                         llr[b, node] without valid entries; damp != 0 (iteration > 0):
 *                         0.5 * out + 0.5 * c2v[b, m] (needs R == E_in).  d_llr (B, N_var). */
int ldpc_index_rows_minsum(const float *d_x, int64_t B, int64_t E_in, const int64_t *d_rows, int64_t R, int W,
                           float *d_out, void *stream);
int ldpc_index_rows_varsum(const float *d_llr, int64_t B, int64_t N_var, const float *d_c2v, int64_t E_in,
                           const int64_t *d_rows, int64_t R, int W, int damp, float *d_out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LDPC_AMD_H */
