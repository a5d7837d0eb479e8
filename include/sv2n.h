/*
 * sv2n.h — C-ABI of the SpotV2Net GAT hot path on MI355X (gfx950).
 *
 * This is the drop-in boundary for the edge-featured GATConv layer that the
 * reference stacks in GATModel (reference utils/models.py:86-117, called once
 * per layer at utils/models.py:146).  The reference binds that layer through
 * Python to the third-party PyG 2.3.0 `torch_geometric.nn.GATConv`
 * (imported at utils/models.py:11; pinned by prose at README.md:88), which is
 * not vendored.  Each entry point below replaces one group of PyG/ATen ops of
 * `GATConv.forward` / its autograd backward:
 *
 *   sv2n_edge_logits_fwd   lin_edge(edge_attr) · att_edge            (row a8)
 *                          folded to edge_attr · W̃ for ALL layers in one pass
 *   sv2n_gat_attn_fwd      a_s[src]+a_d[dst]+a_e, add_self_loops('mean'),
 *                          leaky_relu, softmax(index=dst), dropout, message
 *                          passing scatter-add, concat/mean, bias, activation
 *                          (rows a7, a9, a10, a11 and GATModel's act, a4)
 *   sv2n_gat_attn_bwd      autograd backward of all of the above     (row a12)
 *   sv2n_edge_logits_bwd   d(W̃) = edge_attrᵀ · d(a_e)                (row a12)
 *   sv2n_gemm_f32          the dense projections lin_src(x) (row a6) and its
 *                          backward products, on f32-input MFMA
 *   sv2n_gat_prep_*        per-step weight folding (a_src/a_dst rows, W̃_edge)
 *                          and its backward straight into the parameter grads
 *   sv2n_head_*            GATModel's final Linear (a4) fwd/bwd
 *   sv2n_adam_f32          the reference's Adam step over flat buffers (a13)
 *   sv2n_gat_attn_tiled_*  the same attention fwd/bwd for 32 < n <= 256 (C5
 *                          stress shapes), target-row-tiled
 *   sv2n_gat_attn_fused_*  32 < n <= 256 with narrow edge features: the edge
 *                          logits computed inside the attention (no planes)
 *   sv2n_block_rowmask     edge_index -> per-target source bitmask for graph
 *                          batches whose edges are not in canonical order
 *
 * Conventions
 *  - Every pointer argument is a DEVICE pointer unless the comment says
 *    "host".  The caller owns and pre-allocates every buffer; no entry point
 *    allocates, frees or synchronises.  All work is enqueued on `stream`, so
 *    the calls are capturable into a hipGraph.
 *  - Return value: 0 on success, < 0 for an argument error (see
 *    sv2n_strerror), > 0 is a hipError_t from the launch.
 *  - Graph batches are a disjoint union of `num_graphs` graphs with `n`
 *    nodes each (PyG Batch layout): node v of graph g is
 *    row g*n+v.  Edge rows follow `edge_index` ([2, E], int64, row 0 =
 *    source j, row 1 = target i).  When `edge_index` is NULL the canonical
 *    CovarianceLaggedDataset order is implied (reference
 *    utils/dataset.py:212-226: the n(n-1)/2 row-major upper-triangle pairs,
 *    then the same pairs swapped), described by `canon` ([n(n-1)] uint16,
 *    entry = target<<8 | source).
 *  - Attention-logit layouts ("AE"), per layer:
 *      edge order  float [num_graphs*n(n-1)][H] = [E][H], entry [e][h] = edge
 *                  logit of canonical edge e for head h.  Written when
 *                  `edge_index` is NULL (canonical batches, complete graphs):
 *                  both the edge pass and the attention pass touch it in
 *                  contiguous runs (ae_edge_order = 1 on the attention calls);
 *      dense       float [num_graphs][n][n][H], entry [g][i][j][h] = edge
 *                  logit of edge j->i (any edge set, via edge_index).
 *    The diagonal (self loop) is never stored: the attention kernel derives
 *    it as the mean over i's incoming edges, which is PyG's add_self_loops
 *    fill_value='mean' pushed through the linear edge projection.
 *  - Activation codes: 0 identity, 1 relu, 2 tanh, 3 sigmoid
 *    (reference utils/models.py:125-130).
 */
#ifndef SV2N_H
#define SV2N_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SV2N_ABI_VERSION 21
#define SV2N_MAX_LAYERS 8   /* layers folded into one edge pass            */
#define SV2N_MAX_N 32       /* nodes per graph on the one-workgroup-per-graph
                               attention path (sv2n_gat_attn_fwd/bwd)      */
#define SV2N_MAX_N_TILED 256 /* nodes per graph on the tiled attention path
                               (sv2n_gat_attn_tiled_*) and the edge pass   */
#define SV2N_MAX_HEADS 8    /* attention heads per layer                   */
#define SV2N_TICKET_WORDS 288 /* counter words of a two-level in-launch ticket
                                 (Adam counter, head workspace header)     */

/* argument errors (negative return codes) */
#define SV2N_ERR_ARG       (-1)  /* null pointer / non-positive size        */
#define SV2N_ERR_SHAPE     (-2)  /* unsupported n, heads, layers, widths     */
#define SV2N_ERR_ALIGN     (-3)  /* pointer or leading dim not 16-B aligned  */
#define SV2N_ERR_WORKSPACE (-4)  /* workspace too small                      */

int sv2n_abi_version(void);
const char* sv2n_strerror(int code);

/* Edge logits for L layers at once (replaces PyG GATConv.edge_update's
 * `lin_edge(edge_attr).view(-1,H,C)*att_edge).sum(-1)`).
 *   edge_attr [E][D] row-major, 16-B aligned base.
 *   wfold     [D][hl_pad] with column l*H+h = Σ_c W_edge[l][h*C+c][:]·att_edge[l][h][c];
 *             hl_pad ∈ {4,8,16,32} and L*H <= hl_pad (padding columns are ignored).
 *   ae_layers host array of L device pointers, each [num_edges][H] (edge
 *             order) when edge_index is NULL, else [num_graphs][n][n][H].
 * Self loops present in edge_index are skipped (PyG remove_self_loops). */
int sv2n_edge_logits_fwd(const float* edge_attr, int64_t num_edges, int edge_dim,
                         const int64_t* edge_index, const uint16_t* canon,
                         const float* wfold, int hl_pad,
                         float* const* ae_layers, int num_layers, int heads,
                         int64_t num_graphs, int n, hipStream_t stream);

/* dW̃ = edge_attrᵀ·dAE over all layers: dwfold [D][hl_pad] (overwritten);
 * dae_layers in the layout sv2n_edge_logits_fwd wrote.
 * workspace: sv2n_edge_logits_bwd_workspace(edge_dim, hl_pad) floats. */
int64_t sv2n_edge_logits_bwd_workspace(int edge_dim, int hl_pad);
int sv2n_edge_logits_bwd(const float* edge_attr, int64_t num_edges, int edge_dim,
                         const int64_t* edge_index, const uint16_t* canon,
                         const float* const* dae_layers, int num_layers, int heads,
                         int64_t num_graphs, int n,
                         float* workspace, int64_t workspace_floats,
                         float* dwfold, int hl_pad, hipStream_t stream);

/* Fused per-graph attention forward for one layer.
 *   xs      [N][ldx]: columns [0,H*C) = lin_src(x), [H*C, H*C+H) = a_src,
 *           [H*C+H, H*C+2H) = a_dst (the projection GEMM emits all three).
 *   ae      [num_graphs][n][n][H], or [num_graphs*n(n-1)][H] when
 *           ae_edge_order (complete graphs: rowmask must be NULL), or NULL
 *           (edge_attr=None: no edge term).
 *   rowmask [N] uint32 (bit j of row g*n+i: edge j->i present) or NULL for
 *           complete graphs.
 *   bias    [H*C] (concat) or [C] (mean).
 *   keep    [num_graphs][H][32][32] uint8 attention-dropout keep mask (entry
 *           [g][h][i][j] for edge j->i) or NULL; kept probabilities are
 *           scaled by keep_scale.
 *   y       [N][concat ? H*C : C] = act(concat|mean(Σ_j p_ij·xs_j) + bias).
 *   psave   [num_graphs][H][32][32] softmax probabilities (pre-dropout; rows
 *           padded to 32, absent edges 0) whose sign bit records leaky_relu's
 *           negative side (for the backward).
 *   post_u  GATModel's dropout after the layer (utils/models.py:148, ABI 9):
 *           NULL, or [N][OC] uniform draws; then post_out [N][OC] =
 *           y · (post_u >= post_p) / (1 - post_p), 0 <= post_p < 1, written
 *           beside y (the layer's output; y stays the activation the backward
 *           reads). */
int sv2n_gat_attn_fwd(const float* xs, int ldx, const float* ae, int ae_edge_order,
                      const uint32_t* rowmask,
                      const float* bias, const uint8_t* keep, float keep_scale,
                      float* y, float* psave,
                      const float* post_u, float post_p, float* post_out,
                      int64_t num_graphs, int n, int heads, int channels, int concat,
                      int act, float negative_slope, hipStream_t stream);

/* sv2n_gat_attn_fwd for the model's LAST GAT layer with GATModel.linear
 * (out_features 1, utils/models.py:120/:150) and the training loss
 * nn.MSELoss (5_train_SpotV2Net.py:125/:154, upstream gradient 1) fused in
 * (ABI 13): per graph, out_i = Σ_oc drop(y)[i][oc]·head_weight[oc] +
 * head_bias[0], diff_i = out_i - target_i, and the forward writes
 *   dz     [N][OC]  = act'(2/N·diff_i·head_weight[oc]·m)  (m: the post-dropout
 *          mask·scale, 1 without post_u) — the gradient the layer's backward
 *          starts from, so call sv2n_gat_attn_bwd on it with act = 0
 *          (identity) and no post_u; the layer output itself is not stored;
 *   loss[0] = mean(diff²);
 *   g_head_weight[oc] += Σ_i 2/N·diff_i·drop(y)[i][oc], g_head_bias[0] +=
 *          Σ_i 2/N·diff_i (either may be NULL).
 *   loss_sum[0] += loss[0] when loss_sum is not NULL (ABI 16: a running
 *          epoch sum with no separate add launch).
 * Two launches (the attention, then a fixed-order sum of per-graph partials
 * in workspace: sv2n_gat_attn_fwd_head_mse_workspace floats, 16-B aligned).
 * Runs when
 * sv2n_gat_attn_fwd_head_mse_supported: one workgroup per graph (the batch
 * fills the chip, or few work items), OC <= 512.  Replaces the separate
 * sv2n_head_mse_train launch of a training step. */
int sv2n_gat_attn_fwd_head_mse_supported(int64_t num_graphs, int n, int heads, int channels,
                                         int concat);
int64_t sv2n_gat_attn_fwd_head_mse_workspace(int64_t num_graphs, int heads, int channels,
                                             int concat);
int sv2n_gat_attn_fwd_head_mse(const float* xs, int ldx, const float* ae, int ae_edge_order,
                               const uint32_t* rowmask, const float* bias, const uint8_t* keep,
                               float keep_scale, float* dz, float* psave, const float* post_u,
                               float post_p, const float* head_weight, const float* head_bias,
                               const float* target, float* loss, float* loss_sum,
                               float* g_head_weight, float* g_head_bias, float* workspace,
                               int64_t workspace_floats,
                               int64_t num_graphs, int n, int heads, int channels, int concat,
                               int act, float negative_slope, hipStream_t stream);

/* Backward of sv2n_gat_attn_fwd.
 *   dy, y   [N][OC] (OC = concat ? H*C : C); y is the forward output.
 *   dxs     [N][ldx] gradient w.r.t. xs (all ldx columns written; padding 0).
 *   dae     gradient w.r.t. ae in the layout ae_edge_order names
 *           ([num_graphs][n][n][H] with diagonal / absent entries 0, or
 *           [num_graphs*n(n-1)][H]), or NULL when the forward ran without ae.
 *   dbias_partial [num_graphs][OC] per-graph bias-gradient partial sums.
 *   post_u, post_p  the forward's post-layer dropout draws (or NULL): dy is
 *           then the gradient w.r.t. post_out and is masked and scaled first. */
int sv2n_gat_attn_bwd(const float* dy, const float* y, const float* xs, int ldx,
                      const float* psave, const uint8_t* keep, float keep_scale,
                      const float* post_u, float post_p,
                      const uint32_t* rowmask, float* dxs, float* dae, int ae_edge_order,
                      float* dbias_partial,
                      int64_t num_graphs, int n, int heads, int channels, int concat,
                      int act, float negative_slope, hipStream_t stream);

/* sv2n_gat_attn_bwd writing dxs as bf16 (round to nearest even) into
 * dxs_bf16 [N][ld_dxs] (ld_dxs >= ldx, % 8 == 0, 16-B aligned; columns past
 * ldx zero) instead of fp32 (ABI 14): the bf16 execution mode's
 * weight-gradient operand (sv2n_gat_wgrad_node_bf16b), rounded exactly as
 * that GEMM's staging would round the fp32 dxs. */
int sv2n_gat_attn_bwd_bf16dx(const float* dy, const float* y, const float* xs, int ldx,
                             const float* psave, const uint8_t* keep, float keep_scale,
                             const float* post_u, float post_p, const uint32_t* rowmask,
                             uint16_t* dxs_bf16, int ld_dxs, float* dae, int ae_edge_order,
                             float* dbias_partial, int64_t num_graphs, int n, int heads,
                             int channels, int concat, int act, float negative_slope,
                             hipStream_t stream);

/* sv2n_gat_attn_bwd with the edge-logit weight gradient of EVERY layer fused
 * in (ABI 12; replaces sv2n_edge_logits_bwd for canonical batches, reference
 * GATConv lin_edge / att_edge backward, utils/models.py:146): the workgroup
 * of graph g keeps this layer's d-logits in LDS (none are written), reads
 * the other layers' d-logits layer_dae[l] ([E][heads] canonical edge order,
 * as sv2n_gat_attn_bwd writes them; entry `layer` unused) and streams the
 * graph's edge_attr rows once:
 *   edge_partial[g][d][k] = Σ_{e of g} edge_attr[e][d] · dae_l(k)[e][h(k)],
 * k = l·heads + h < num_layers·heads <= hl_pad (columns past that: 0).
 * Sum the partials in graph order with sv2n_edge_partials_reduce to get the
 * [edge_dim][hl_pad] gradient sv2n_edge_logits_bwd returns.  Canonical
 * complete graphs only; sv2n_gat_attn_bwd_edge_supported says whether the
 * shape runs (all heads in one workgroup, hl_pad <= 8, even edge_dim <= 128).
 * edge_attr 16-B aligned; layer_dae is a HOST array of device pointers. */
int sv2n_gat_attn_bwd_edge_supported(int64_t num_graphs, int n, int heads, int channels,
                                     int edge_dim, int hl_pad);
int sv2n_gat_attn_bwd_edge(const float* dy, const float* y, const float* xs, int ldx,
                           const float* psave, const uint8_t* keep, float keep_scale,
                           const float* post_u, float post_p, float* dxs, float* dbias_partial,
                           const float* edge_attr, int edge_dim, const float* const* layer_dae,
                           int num_layers, int layer, int hl_pad, float* edge_partial,
                           int64_t num_graphs, int n, int heads, int channels, int concat, int act,
                           float negative_slope, hipStream_t stream);
/* out[o] = Σ_p partial[p][o], p = 0 .. num_parts-1 in order (deterministic). */
int sv2n_edge_partials_reduce(const float* partial, int64_t num_parts, int64_t width, float* out,
                              hipStream_t stream);

/* C[M][N] = Σ_k A(m,k)·B(n,k), f32 in / f32 accumulate on MFMA (exact f32).
 *   A(m,k) = A[m*lda+k] if a_kmajor else A[k*lda+m]
 *   B(n,k) = B[n*ldb+k] if b_kmajor else B[k*ldb+n]
 *   C[m*ldc+n] is overwritten.
 * Replaces the lin_src projection GEMM (row a6: a_kmajor = b_kmajor = 1) and
 * its backward products dX (a_kmajor=1, b_kmajor=0) and dWᵀ (0, 0).
 * workspace: sv2n_gemm_f32_workspace(M,N,K) floats (split-K partial slabs;
 * 0 => may be NULL). */
int64_t sv2n_gemm_f32_workspace(int64_t M, int64_t N, int64_t K);
int sv2n_gemm_f32(int a_kmajor, int b_kmajor, const float* A, int64_t lda,
                  const float* B, int64_t ldb, float* C, int64_t ldc,
                  int64_t M, int64_t N, int64_t K,
                  float* workspace, int64_t workspace_floats, hipStream_t stream);

/* f32-accurate GEMM on bf16 MFMA for a small "weight" operand B:
 *   C[M][N] = Σ_k A[m][k]·B(n,k),  A fp32 k-major (16-B aligned, lda % 4 == 0)
 * B is passed as its three bf16 planes (Bp [3][N][Kp], Kp =
 * sv2n_split3_kpad(K)), each fp32 value being the exact sum of its three
 * bf16 terms; the six products with combined order <= 2 are accumulated in
 * fp32, so the result matches an exact-f32 GEMM to fp32 rounding (measured
 * max |err| / Σ|a·b| 3.8e-7 vs 3.75e-7 for sv2n_gemm_f32 on the C2 shapes).
 * sv2n_split3 builds the planes: transpose = 0 reads B as [N][K] (row
 * stride ld), transpose = 1 as [K][N]. */
int64_t sv2n_split3_kpad(int64_t K);
int sv2n_split3(const float* in, int64_t rows, int64_t K, int64_t ld, int transpose,
                uint16_t* out, hipStream_t stream);
int sv2n_gemm_f32x3(const float* A, int64_t lda, const uint16_t* Bp, float* C, int64_t ldc,
                    int64_t M, int64_t N, int64_t K, hipStream_t stream);
/* The same product with the consumer's ReLU backward applied as it is stored
 * (ABI 10): C = (Y > 0) ? A·Bᵀ : 0, Y [M][ldy] the activation the layer saved
 * (act_bwd of ReLU, bit for bit).  The backward of a GAT stack writes the
 * previous layer's dZ here instead of its dy (dy·relu'(y) of GATModel's
 * act after every layer, utils/models.py:147), and that layer's
 * sv2n_gat_attn_bwd then runs with act = identity and reads no y.
 * K % 4 == 0 only (else SV2N_ERR_SHAPE; nothing is launched). */
int sv2n_gemm_f32x3_relu(const float* A, int64_t lda, const uint16_t* Bp, float* C, int64_t ldc,
                         int64_t M, int64_t N, int64_t K, const float* Y, int64_t ldy,
                         hipStream_t stream);

/* bf16 execution mode of the same projection (the reference run under
 * torch.autocast(dtype=bfloat16), BASELINE config C3): C = bf16(A)·bf16(B)ᵀ
 * with fp32 accumulation and fp32 output.  A fp32 k-major as in
 * sv2n_gemm_f32x3 (rounded to bf16 while staged); Bp is plane 0 of the
 * sv2n_split3 planes of B (= bf16_rn(B), [N][Kp]); planes 1-2 are not read. */
int sv2n_gemm_bf16(const float* A, int64_t lda, const uint16_t* Bp, float* C, int64_t ldc,
                   int64_t M, int64_t N, int64_t K, hipStream_t stream);
/* sv2n_gemm_bf16 that also leaves bf16(A) in a_bf16 [M][ld_ab] (ld_ab >=
 * K rounded up to 64, % 8 == 0, 16-B aligned; zero past K): written by the
 * GEMM's own operand staging on the large-tile path (ABI 14), for the
 * weight-gradient GEMM of the same layer (sv2n_gat_wgrad_node_bf16b). */
int sv2n_gemm_bf16_export(const float* A, int64_t lda, const uint16_t* Bp, float* C,
                          int64_t ldc, int64_t M, int64_t N, int64_t K, uint16_t* a_bf16,
                          int64_t ld_ab, hipStream_t stream);
/* sv2n_gemm_bf16 with A already bf16 [M][lda] (lda % 8 == 0, 16-B aligned;
 * e.g. sv2n_window_gather_bf16x's x_bf16), ABI 15: the same products, no
 * rounding pass.  Large-tile shapes only (M >= 1024, N >= 384), else
 * SV2N_ERR_SHAPE. */
int sv2n_gemm_bf16_a16(const uint16_t* A, int64_t lda, const uint16_t* Bp, float* C,
                       int64_t ldc, int64_t M, int64_t N, int64_t K, hipStream_t stream);

/* Weight preparation for one GAT layer (replaces, per step, PyG's separate
 * (x_src*att_src).sum(-1) / (x_dst*att_dst).sum(-1) and lin_edge·att_edge
 * reductions by folded weights):
 *   waug [ldx][F] = [ W (H*C rows) ; W_hᵀatt_src_h (H rows) ; W_hᵀatt_dst_h (H rows) ; 0 ]
 *   wfold[d][col0+h] = Σ_c att_edge[h*C+c] · W_edge[h*C+c][d]   (skipped if W_edge NULL) */
int sv2n_gat_prep_fwd(const float* W, const float* att_src, const float* att_dst,
                      int heads, int channels, int in_features, float* waug, int ldx,
                      const float* W_edge, const float* att_edge, int edge_dim,
                      float* wfold, int hl_pad, int col0, hipStream_t stream);

/* All layers' weight preparation in ONE launch: per layer what
 * sv2n_gat_prep_fwd writes (waug, wfold columns), plus the bf16 split planes
 * the f32-accurate GEMM (sv2n_gemm_f32x3) consumes:
 *   planes  [3][ldx][kp]  = split3(waug)        (B of xs = x · waugᵀ; kp = sv2n_split3_kpad(F))
 *   planesT [3][F][kpt]   = split3(waugᵀ)       (B of dx = dxs · waug; kpt = sv2n_split3_kpad(ldx)),
 *                                               skipped when NULL
 * i.e. sv2n_gat_prep_fwd + sv2n_split3 (+ transposed) per layer, fused. */
typedef struct sv2n_prep_layer {
  const float* W;         /* lin_src.weight [H*C][F] */
  const float* att_src;   /* [H*C] */
  const float* att_dst;   /* [H*C] */
  int heads, channels, in_features, ldx;
  float* waug;            /* [ldx][F], or NULL: not written (ABI 19; the planes
                             are the GEMMs' only operand, e.g. in bf16 mode) */
  uint16_t* planes;       /* [nplanes][ldx][kp] */
  uint16_t* planes_t;     /* [nplanes][F][kpt] or NULL */
  const float* W_edge;    /* lin_edge.weight [H*C][edge_dim] or NULL */
  const float* att_edge;  /* [H*C] */
  int edge_dim, hl_pad, col0;
  float* wfold;           /* [edge_dim][hl_pad] */
  int nplanes;            /* planes written per operand: 3 (split, default when 0)
                             or 1 (bf16 mode: plane 0 = bf16_rn(w) only) */
} sv2n_prep_layer;
int sv2n_gat_prep_fwd_all(const sv2n_prep_layer* layers, int num_layers, hipStream_t stream);

/* Backward of the node half of sv2n_gat_prep_fwd plus the bias: from
 * dwaug_t = dWaugᵀ [F][ldx] ACCUMULATE (+=) into gW [H*C][F], g_att_src /
 * g_att_dst [H*C] and g_bias[o] += Σ_b dbias_partial[b][o] (any output NULL
 * = skipped; dwaug_t/W/att_* may be NULL when gW, g_att_src, g_att_dst are).
 * workspace: sv2n_gat_prep_bwd_workspace(heads, in_features) floats (needed
 * when g_att_src or g_att_dst is requested). */
int64_t sv2n_gat_prep_bwd_workspace(int heads, int in_features);
int sv2n_gat_prep_bwd_node(const float* dwaug_t, int ldx, const float* W,
                           const float* att_src, const float* att_dst, int heads,
                           int channels, int in_features, const float* dbias_partial,
                           int num_parts, int bias_len, float* gW, float* g_att_src,
                           float* g_att_dst, float* g_bias, float* workspace,
                           int64_t workspace_floats, hipStream_t stream);

/* The split-K f32 GEMM of sv2n_gemm_f32 alone: C's K slices are left as
 * slabs [count][M][N] (count = sv2n_gemm_f32_slabs_count(M, N, K); a single
 * slice writes slab 0 = C).  The caller sums them (fixed order, as the
 * library's reduce does). */
int sv2n_gemm_f32_slabs_count(int64_t M, int64_t N, int64_t K);
int sv2n_gemm_f32_slabs(int a_kmajor, int b_kmajor, const float* A, int64_t lda, const float* B,
                        int64_t ldb, int64_t M, int64_t N, int64_t K, float* slabs,
                        int64_t slab_floats, hipStream_t stream);

/* Weight gradients of one GAT layer in two launches: the split-K GEMM
 *   T = dWaugᵀ[f][o] = Σ_k x[k][f] · dxs[k][o]        (x [num_nodes][ld_x], dxs [num_nodes][ldx])
 * and one fused epilogue that reduces its K slabs in a fixed order and
 * ACCUMULATES gW (+ the att_src / att_dst fold terms), g_att_src, g_att_dst and
 * g_bias (Σ of dbias_partial [num_parts][bias_len]) — what
 * sv2n_gemm_f32 + sv2n_gat_prep_bwd_node compute, without materialising T.
 * Replaces lin_src / att_src / att_dst / bias autograd of PyG GATConv
 * (torch_geometric/nn/conv/gat_conv.py, reference utils/models.py:146).
 * workspace: sv2n_gat_wgrad_node_workspace floats (no state between calls). */
int64_t sv2n_gat_wgrad_node_workspace(int64_t num_nodes, int in_features, int ldx, int heads,
                                      int channels);
int sv2n_gat_wgrad_node(const float* x, int64_t ld_x, const float* dxs, int ldx,
                        int64_t num_nodes, int in_features, const float* W,
                        const float* att_src, const float* att_dst, int heads, int channels,
                        const float* dbias_partial, int num_parts, int bias_len, float* gW,
                        float* g_att_src, float* g_att_dst, float* g_bias, float* workspace,
                        int64_t workspace_floats, hipStream_t stream);

/* sv2n_gat_wgrad_node in the bf16 execution mode: the GEMM T = xᵀ·dxs runs
 * on bf16 operands (rounded while staged) with fp32 accumulation; the fold,
 * attention-vector and bias epilogue is the fp32 one.  Same arguments;
 * workspace: sv2n_gat_wgrad_node_bf16_workspace floats; x, dxs 16-B aligned
 * with leading dims % 4 == 0. */
int64_t sv2n_gat_wgrad_node_bf16_workspace(int64_t num_nodes, int in_features, int ldx,
                                           int heads, int channels);
int sv2n_gat_wgrad_node_bf16(const float* x, int64_t ld_x, const float* dxs, int ldx,
                             int64_t num_nodes, int in_features, const float* W,
                             const float* att_src, const float* att_dst, int heads, int channels,
                             const float* dbias_partial, int num_parts, int bias_len, float* gW,
                             float* g_att_src, float* g_att_dst, float* g_bias, float* workspace,
                             int64_t workspace_floats, hipStream_t stream);

/* sv2n_gat_wgrad_node_bf16 on operands already in bf16 (ABI 14): x_bf16
 * [num_nodes][ld_xb] (sv2n_gemm_bf16_export of the layer's projection) and
 * dxs_bf16 [num_nodes][ld_db] (sv2n_gat_attn_bwd_bf16dx); ld % 8 == 0, 16-B
 * aligned, in_features % 4 == 0, gW required.  Same results as
 * sv2n_gat_wgrad_node_bf16 on the fp32 operands; same workspace. */
int sv2n_gat_wgrad_node_bf16b(const uint16_t* x_bf16, int64_t ld_xb, const uint16_t* dxs_bf16,
                              int64_t ld_db, int64_t num_nodes, int in_features, int ldx,
                              const float* W, const float* att_src, const float* att_dst,
                              int heads, int channels, const float* dbias_partial, int num_parts,
                              int bias_len, float* gW, float* g_att_src, float* g_att_dst,
                              float* g_bias, float* workspace, int64_t workspace_floats,
                              hipStream_t stream);

/* Backward of the edge fold: ACCUMULATE gW_edge[h*C+c][d] += dwfold[d][col0+h]·att_edge[h*C+c]
 * and g_att_edge[h*C+c] += Σ_d W_edge[h*C+c][d]·dwfold[d][col0+h]. */
int sv2n_gat_prep_bwd_edge(const float* dwfold, int hl_pad, int col0,
                           const float* W_edge, const float* att_edge, int heads,
                           int channels, int edge_dim, float* gW_edge,
                           float* g_att_edge, hipStream_t stream);

/* sv2n_gat_prep_bwd_edge for every layer in ONE launch (ABI 7; the layers'
 * gradient buffers are disjoint, each result as the per-layer call's). */
typedef struct sv2n_edge_grad_layer {
  const float* W_edge;    /* lin_edge.weight [H*C][edge_dim] */
  const float* att_edge;  /* [H*C] */
  float* gW_edge;         /* [H*C][edge_dim] or NULL */
  float* g_att_edge;      /* [H*C] or NULL */
  int heads, channels, col0;
} sv2n_edge_grad_layer;
int sv2n_gat_prep_bwd_edge_all(const float* dwfold, int hl_pad, int edge_dim,
                               const sv2n_edge_grad_layer* layers, int num_layers,
                               hipStream_t stream);

/* torch.optim.Adam step (amsgrad=False) over flat buffers of n floats
 * (16-B aligned); *step is the already-incremented device step count. */
int sv2n_adam_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                  int64_t n, const float* step, float lr, float beta1, float beta2,
                  float eps, float weight_decay, hipStream_t stream);

/* Adam step that also advances the device step counter (t = *step + 1 is used
 * and stored) and zeroes grad after reading it (the next backward accumulates
 * into zeros).  counter: SV2N_TICKET_WORDS uint32 ticket words (two-level
 * tickets), zero before the first call (left zero by every call). */
int sv2n_adam_f32_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                       float* step, uint32_t* counter, float lr, float beta1, float beta2,
                       float eps, float weight_decay, hipStream_t stream);

/* Edge logits for edge features in the reference's covariance layout (ABI
 * 18; utils/dataset.py:228-243 and :279-282): row s -> t of edge_attr is
 * [cov_t'(s,t) | var_t'(s) | var_t'(t)] for t' < seq_length (edge_dim =
 * 3·seq_length), cov the same for both directions, var a per-node series.
 * Canonical complete graphs of n <= 32 nodes (canon as for
 * sv2n_edge_logits_fwd), L·H <= 16 logit columns, seq_length <= 64.  The
 * outputs are those of sv2n_edge_logits_fwd / _bwd (ae per layer [E][H] in
 * edge order; dwfold [edge_dim][hl_pad]) computed from the covariance columns
 * of the upper rows and one variance series per node: ≈ 1/6 of edge_attr is
 * read.  The caller guarantees the layout (its builder wrote it); other
 * edge_attr gives other logits.  The backward's workspace:
 * sv2n_edge_logits_bwd_cv_workspace floats. */
int sv2n_edge_logits_fwd_cv(const float* edge_attr, int64_t num_graphs, int n, int seq_length,
                            const uint16_t* canon, const float* wfold, int hl_pad,
                            float* const* ae_layers, int num_layers, int heads, hipStream_t stream);
int64_t sv2n_edge_logits_bwd_cv_workspace(int seq_length, int hl_pad);
int sv2n_edge_logits_bwd_cv(const float* edge_attr, int64_t num_graphs, int n, int seq_length,
                            const uint16_t* canon, const float* const* dae_layers, int num_layers,
                            int heads, float* workspace, int64_t workspace_floats, float* dwfold,
                            int hl_pad, hipStream_t stream);

/* Dropout uniforms for the captured training step (ABI 17; replaces the
 * torch.rand draw behind F.dropout, reference utils/models.py:148, inside
 * spotv2net_amd.train.TrainStep): u[i] = word i%4 of Philox4x32-10 with key
 * = seed and counter = (i/4 low, i/4 high, salt, (uint32)*step), scaled as
 * (word >> 8)·2^-24 in [0, 1).  *step is a device float (the optimizer's step
 * count), so a graph replay draws new values with no host work; u 16-B
 * aligned. */
int sv2n_dropout_uniform(float* u, int64_t n, uint64_t seed, const float* step, uint32_t salt,
                         hipStream_t stream);

/* Output head (GATModel.linear, reference utils/models.py:120/:150):
 *   out[i][o] = Σ_c x[i][c]·weight[o][c] + bias[o]      x [rows][in], weight [out][in]
 * in_features <= 1024, out_features <= 16.  The backward writes dx and
 * ACCUMULATES into g_weight / g_bias (either may be NULL).
 * workspace: sv2n_head_bwd_workspace(rows, in, out) floats, 16-B aligned; its
 * first SV2N_TICKET_WORDS (288) floats are ticket counters that must be zero
 * before the first call (every call leaves them zero), the rest per-workgroup
 * partial slabs
 * reduced in a fixed order inside the launch (deterministic). */
int sv2n_head_fwd(const float* x, int64_t num_rows, int in_features, const float* weight,
                  const float* bias, int out_features, float* out, hipStream_t stream);
int64_t sv2n_head_bwd_workspace(int64_t num_rows, int in_features, int out_features);
int sv2n_head_bwd(const float* x, int64_t num_rows, int in_features, const float* weight,
                  int out_features, const float* dout, float* dx, float* g_weight,
                  float* g_bias, float* workspace, int64_t workspace_floats,
                  hipStream_t stream);

/* Head fused with the training loss (5_train_SpotV2Net.py:154, nn.MSELoss
 * mean): forward writes diff = out - target (kept for the backward), the
 * prediction to yhat when non-NULL, and loss[0] = mean(diff²); backward
 * scales diff by 2/(rows·out)·grad_loss[0] (grad_loss: device scalar, the
 * upstream gradient of the loss) and is otherwise sv2n_head_bwd.
 * workspace: sv2n_head_mse_workspace(...) floats, same counter rule. */
int64_t sv2n_head_mse_workspace(int64_t num_rows, int in_features, int out_features);
int sv2n_head_mse_fwd(const float* x, int64_t num_rows, int in_features, const float* weight,
                      const float* bias, int out_features, const float* target, float* yhat,
                      float* diff, float* loss, float* loss_sum, float* workspace,
                      int64_t workspace_floats, hipStream_t stream);
int sv2n_head_mse_bwd(const float* x, int64_t num_rows, int in_features, const float* weight,
                      int out_features, const float* diff, const float* grad_loss, float* dx,
                      float* g_weight, float* g_bias, float* workspace,
                      int64_t workspace_floats, hipStream_t stream);

/* Head + MSE forward and backward in ONE launch for a training step whose
 * upstream loss gradient is 1 (loss.backward()): loss[0] = mean(diff²), dx =
 * 2/(rows·out)·diff·weight, and g_weight / g_bias ACCUMULATE Σ 2/(rows·out)·
 * diff ⊗ [x, 1] (either may be NULL).  Equals sv2n_head_mse_fwd followed by
 * sv2n_head_mse_bwd with grad_loss = 1.  loss_sum (ABI 16; also in
 * sv2n_head_mse_fwd): when not NULL, loss_sum[0] += loss[0] in the same
 * launch (an epoch's running sum without an add launch).  workspace:
 * sv2n_head_mse_train_workspace(...) floats, same counter rule. */
int64_t sv2n_head_mse_train_workspace(int64_t num_rows, int in_features, int out_features);
int sv2n_head_mse_train(const float* x, int64_t num_rows, int in_features, const float* weight,
                        const float* bias, int out_features, const float* target, float* loss,
                        float* loss_sum, float* dx, float* g_weight, float* g_bias,
                        float* workspace, int64_t workspace_floats, hipStream_t stream);

/* sv2n_head_mse_train in two launches (ABI 19; the wave-per-rows form only:
 * out_features <= 4 and out_features * ceil(in_features / 64) <= 32, else
 * SV2N_ERR_SHAPE).  _rows writes dx and the per-block partials into the
 * workspace; _reduce (same workspace, num_rows and widths, any stream ordered
 * after _rows) sums them into loss, loss_sum, g_weight, g_bias.  The caller
 * runs _reduce after the layer backwards, which need only dx, instead of the
 * one-launch form's ticket chain ahead of them.  Bitwise equal to the
 * one-launch sv2n_head_mse_train.  ABI 20: _reduce takes the workspace size
 * too and refuses one smaller than sv2n_head_mse_train_workspace (a mismatch
 * with the _rows launch would otherwise read past the caller's buffer). */
int sv2n_head_mse_train_rows(const float* x, int64_t num_rows, int in_features,
                             const float* weight, const float* bias, int out_features,
                             const float* target, float* dx, float* workspace,
                             int64_t workspace_floats, hipStream_t stream);
int sv2n_head_mse_train_reduce(const float* workspace, int64_t workspace_floats,
                               int64_t num_rows, int in_features, int out_features, float* loss,
                               float* loss_sum, float* g_weight, float* g_bias,
                               hipStream_t stream);

/* Fused attention for dense-block graphs of 32 < n <= 256 nodes (any n <= 256
 * works; n <= 32 is faster on sv2n_gat_attn_fwd/bwd).  Same semantics and
 * arguments as sv2n_gat_attn_fwd/bwd except:
 *   ae       the layer's edge logits as head planes [H][num_edges] in edge
 *            order (sv2n_edge_logits_fwd_planes), or NULL (no edge term);
 *   eid      [N][n] int32 edge id of (target row, source j), -1 if absent
 *            (sv2n_block_eid), or NULL for the canonical edge order;
 *   rowmask  [N][ceil(n/32)] uint32 words (bit j%32 of word j/32 of row g*n+i:
 *            edge j->i present) or NULL for complete graphs;
 *   keep     [num_graphs][H][n][n] uint8 or NULL;
 *   channels <= 64;
 *   dae      (backward) head planes [H][num_edges]: every present edge's
 *            entry is written, input self loops are left untouched;
 *   nothing is saved for the backward: it recomputes the attention from xs
 *   and ae (pass the forward's ae again);
 *   concat = 0 needs a workspace of sv2n_gat_attn_tiled_workspace(...)
 *   floats (per-head aggregates before the mean). */
int64_t sv2n_gat_attn_tiled_workspace(int64_t num_graphs, int n, int heads, int channels,
                                      int concat);
int sv2n_gat_attn_tiled_fwd(const float* xs, int ldx, const float* ae, int64_t num_edges,
                            const int32_t* eid, const uint32_t* rowmask, const float* bias,
                            const uint8_t* keep, float keep_scale, float* y, float* workspace,
                            int64_t workspace_floats, int64_t num_graphs, int n, int heads,
                            int channels, int concat, int act, float negative_slope,
                            hipStream_t stream);
int sv2n_gat_attn_tiled_bwd(const float* dy, const float* y, const float* xs, int ldx,
                            const float* ae, int64_t num_edges, const int32_t* eid,
                            const uint8_t* keep, float keep_scale, const uint32_t* rowmask,
                            float* dxs, float* dae, float* dbias_partial, int64_t num_graphs,
                            int n, int heads, int channels, int concat, int act,
                            float negative_slope, hipStream_t stream);

/* Edge-fused attention for dense-block graphs of 32 < n <= 256 nodes with
 * narrow edge features (n 256, edge_dim 12, 8 heads x 16).
 * Replaces, per GATConv layer, PyG's lin_edge + edge_update + softmax +
 * dropout + propagate + bias (torch_geometric/nn/conv/gat_conv.py, reference
 * utils/models.py:146) AND this library's separate edge pass: the logit of
 * (i <- j, h) is edge_attr[e]·wfold[:, col0+h] + a_src[j,h] + a_dst[i,h],
 * computed where it is consumed in the forward and again in the backward.
 *   sv2n_gat_attn_fused_supported: 1 if (n, heads, channels, edge_dim) are
 *            taken (heads <= 8, channels in {4,8,12,16}, edge_dim in {3,6,12})
 *   edge_attr [num_edges][edge_dim] fp32; canonical order (eid NULL) needs
 *            num_edges = num_graphs*n*(n-1) and 16-B alignment; block
 *            layouts pass eid [N][n] (sv2n_block_eid; -1 = absent edge)
 *   wfold, hl_pad, col0: the layer's columns of the edge fold
 *            (sv2n_gat_prep_fwd_all), col0 + heads <= hl_pad
 *   xs       [N][ldx] projection output (ldx % 4 == 0, 16-B aligned)
 *   keep     [num_graphs][heads][n][n] uint8 attention-dropout mask or NULL
 *   y        [N][OC] layer output (activation applied)
 *   agg, stats: training only (both or neither): agg [N][heads*channels] the
 *            pre-bias head aggregates, stats [N][4*heads] (row max, 1/sum,
 *            self-loop logit, edge count) — the backward's inputs
 * Backward: dxs [N][ldx] is overwritten (xs, a_src, a_dst, padding columns);
 * dbias_partial [num_graphs*ceil(n/32)][OC] overwritten (sum them);
 * dwfold columns col0..col0+heads-1 overwritten (the layer's dW̃);
 * workspace sv2n_gat_attn_fused_bwd_workspace floats, no state between calls. */
int sv2n_gat_attn_fused_supported(int n, int heads, int channels, int edge_dim);
int sv2n_gat_attn_fused_fwd(const float* xs, int ldx, const float* edge_attr, int edge_dim,
                            const float* wfold, int hl_pad, int col0, const int32_t* eid,
                            const float* bias, const uint8_t* keep, float keep_scale, float* y,
                            float* agg, float* stats, int64_t num_graphs, int n, int heads,
                            int channels, int concat, int act, float negative_slope,
                            hipStream_t stream);
int64_t sv2n_gat_attn_fused_bwd_workspace(int64_t num_graphs, int n, int heads, int channels,
                                          int edge_dim);
int sv2n_gat_attn_fused_bwd(const float* dy, const float* y, const float* agg,
                            const float* stats, const float* xs, int ldx,
                            const float* edge_attr, int edge_dim, const float* wfold,
                            int hl_pad, int col0, const int32_t* eid, const uint8_t* keep,
                            float keep_scale, float* dxs, float* dbias_partial, float* dwfold,
                            float* workspace, int64_t workspace_floats, int64_t num_graphs,
                            int n, int heads, int channels, int concat, int act,
                            float negative_slope, hipStream_t stream);

/* Edge logits / their weight gradient with the per-layer output in head
 * planes [H][num_edges] (edge order), the layout of the tiled attention:
 * ae_layers[l][h*E + e] = edge_attr[e] · wfold[:, l*H + h] for every edge
 * (input self loops included; their values are never read).  The backward
 * skips input self loops when edge_index is given (NULL: none present). */
int sv2n_edge_logits_fwd_planes(const float* edge_attr, int64_t num_edges, int edge_dim,
                                const float* wfold, int hl_pad, float* const* ae_layers,
                                int num_layers, int heads, hipStream_t stream);
int sv2n_edge_logits_bwd_planes(const float* edge_attr, int64_t num_edges, int edge_dim,
                                const int64_t* edge_index, const float* const* dae_layers,
                                int num_layers, int heads, float* workspace,
                                int64_t workspace_floats, float* dwfold, int hl_pad,
                                hipStream_t stream);

/* eid[t*n + j] = e for every non-self edge e: s->t, j = s - g*n (eid
 * [num_nodes][n] int32 must be filled with -1 by the caller). */
int sv2n_block_eid(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes, int n,
                   int32_t* eid, hipStream_t stream);

/* rowmask[t*W + j/32] |= 1<<(j%32), W = ceil(n/32), j = s - g*n, for every
 * non-self edge s->t (rowmask [num_nodes][W] must be zeroed by the caller).
 * Edges must stay inside their n-node block; n <= SV2N_MAX_N_TILED. */
int sv2n_block_rowmask(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes,
                       int n, uint32_t* rowmask, hipStream_t stream);

/* sv2n_block_rowmask that also validates, with no host round trip: adds to
 * *violations (int32, device) the number of edges the dense-block kernels
 * cannot take — an end outside [0, num_nodes), source and target in
 * different n-node blocks, or a repeated (target, source) pair.  The host
 * reads the count later (deferred error) instead of synchronising per batch. */
int sv2n_block_rowmask_checked(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes,
                               int n, uint32_t* rowmask, int32_t* violations,
                               hipStream_t stream);

/* Device-side CovarianceLaggedDataset window builder (reference
 * utils/dataset.py:200-282; multi-output targets :385-405): for window b with
 * first matrix st_b = starts[b] + start_offset (starts int64, device; the
 * offset is WindowDataset's cut, so a batch index vector is passed as is —
 * ABI 9), fills the PyG batch layout
 *   x         [B*n][n*S]      x[b*n+v][c*S+t] = vol[st_b+t][v][c]
 *   edge_attr [B*n(n-1)][3S]  canonical edge order (canon = target<<8|source):
 *             [0*S+t] upper-triangle volvol[t][min][max], [1*S+t] volvol[t][s][s],
 *             [2*S+t] volvol[t][g][g]
 *   y         [B*n*F]         y[(b*n+v)*F+k] = vol[st_b+S+k][v][v]
 * vol / volvol: [T][n][n] fp32 series, T = num_matrices.  A window outside
 * the series (starts[b] < 0, st_b < 0 or st_b + S + F > T) reads nothing and
 * its x / edge_attr / y rows are written as NaN (ABI 8; a negative starts[b]
 * since ABI 12, so a negative batch index never reads before the offset). */
int sv2n_window_gather(const float* vol, const float* volvol, int n, int64_t num_matrices,
                       const int64_t* starts, int64_t start_offset,
                       int64_t num_windows, int seq_length, int future_steps,
                       const uint16_t* canon, float* x, float* edge_attr, float* y,
                       hipStream_t stream);

/* sv2n_window_gather with the series' diagonal given (ABI 11): diag [T][n],
 * diag[t][v] = volvol[t][v][v] (contiguous fp32, built once per series), or
 * NULL (read from volvol).  Same outputs bit for bit; the diagonal reads of
 * the LDS row kernel become one 120-B run per matrix instead of one 128-B
 * line per element. */
int sv2n_window_gather_diag(const float* vol, const float* volvol, const float* diag, int n,
                            int64_t num_matrices, const int64_t* starts, int64_t start_offset,
                            int64_t num_windows, int seq_length, int future_steps,
                            const uint16_t* canon, float* x, float* edge_attr, float* y,
                            hipStream_t stream);
/* sv2n_window_gather_diag that also writes bf16(x) (round to nearest even)
 * into x_bf16 [num_windows·n][ld_xb] (ld_xb >= n·seq_length, % 4 == 0, zero
 * past n·seq_length; NaN rows for windows outside the series) — the bf16
 * execution mode's projection operand (sv2n_gemm_bf16_a16) and its weight
 * gradient's (sv2n_gat_wgrad_node_bf16b) straight from the data builder
 * (ABI 15).  x may be NULL (ABI 21): only the twin is written, for a
 * consumer that reads x through it alone.  Row-kernel shapes only
 * (n·seq_length % 4 == 0, 3·S·(n+1) floats of LDS <= 64 KiB, future_steps
 * <= 256); else SV2N_ERR_SHAPE. */
int sv2n_window_gather_bf16x(const float* vol, const float* volvol, const float* diag, int n,
                             int64_t num_matrices, const int64_t* starts, int64_t start_offset,
                             int64_t num_windows, int seq_length, int future_steps,
                             const uint16_t* canon, float* x, uint16_t* x_bf16, int64_t ld_xb,
                             float* edge_attr, float* y, hipStream_t stream);
/* The window gather for a consumer that reads edge_attr only through the
 * covariance-layout edge passes (sv2n_edge_logits_fwd_cv / _bwd_cv; ABI 19):
 * x, y (and bf16(x) when x_bf16 is not NULL, as sv2n_window_gather_bf16x)
 * in full, but of edge_attr only the covariance columns [0, S) of the upper
 * rows, the source-variance columns [S, 2S) of upper row 0 and the
 * target-variance columns [2S, 3S) of the upper rows of the pairs (0, w),
 * and the covariance columns of the first (16 - P % 16) % 16 lower rows
 * (the even-S passes' last tile of 16 upper rows runs into them with zero
 * d-logits): what those passes read (≈ 1/6 of the edge bytes).  The rest of edge_attr
 * is left as it was; any other reader of it is the caller's error.  Windows
 * outside the series give NaN rows as in sv2n_window_gather_diag.  x may be
 * NULL when x_bf16 is not (ABI 21, as sv2n_window_gather_bf16x).  Row-kernel
 * shapes only (see sv2n_window_gather_bf16x); else SV2N_ERR_SHAPE. */
int sv2n_window_gather_cv(const float* vol, const float* volvol, const float* diag, int n,
                          int64_t num_matrices, const int64_t* starts, int64_t start_offset,
                          int64_t num_windows, int seq_length, int future_steps,
                          const uint16_t* canon, float* x, uint16_t* x_bf16, int64_t ld_xb,
                          float* edge_attr, float* y, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SV2N_H */
