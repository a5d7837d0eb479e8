// C-ABI entry points of the per-graph GAT attention for graphs of n <= 32
// nodes — the dense-block form of PyG 2.3.0 GATConv message passing that
// SpotV2Net runs on its fully connected 30-asset graphs
// (reference utils/models.py:146 -> GATConv.forward).
//
// The kernels live in sv2n_attn_canon.hip (one 256-thread workgroup per graph,
// canonical edge order or row-mask block layouts, every H <= SV2N_MAX_HEADS).
// Saved probabilities / keep masks use a padded [g][h][32][32] layout (16-B
// aligned rows); the sign bit of a saved probability records leaky_relu's
// negative side for the backward.
#include "sv2n_common.h"

namespace sv2n {
void attn_canon_fwd(int64_t B, hipStream_t st, const float* xs, int ldx, const float* ae,
                    int ae_edge_order, const uint32_t* rowmask, const float* bias,
                    const uint8_t* keep, float keep_scale, float* y, float* psave,
                    const float* post_u, float post_p, float* post_out, int n, int H, int C,
                    int concat, int act, float slope, const HeadFuse& hf);
bool attn_canon_head_ok(int64_t B, int n, int H, int C, bool concat);
void attn_canon_bwd(int64_t B, hipStream_t st, const float* dy, const float* y, const float* xs,
                    int ldx, const float* psave, const uint8_t* keep, float keep_scale,
                    const float* post_u, float post_p, const uint32_t* rowmask, float* dxs, float* dae, int ae_edge_order,
                    float* dbias, int n, int H, int C, int concat, int act, float slope,
                    const EdgeTail& et, unsigned short* dxb = nullptr, int ldb = 0);
bool attn_canon_edge_tail_ok(int64_t B, int n, int H, int C, int D, int hlp);
}  // namespace sv2n

using namespace sv2n;

static int check_attn_args(int64_t B, int n, int H, int C, int ldx, int act) {
  if (B <= 0 || C <= 0) return SV2N_ERR_ARG;
  if (n < 1 || n > SV2N_MAX_N || H < 1 || H > SV2N_MAX_HEADS || act < 0 || act > 3)
    return SV2N_ERR_SHAPE;
  if (ldx < H * C + 2 * H) return SV2N_ERR_SHAPE;
  return 0;
}

extern "C" int sv2n_gat_attn_fwd(const float* xs, int ldx, const float* ae, int ae_edge_order,
                                 const uint32_t* rowmask, const float* bias, const uint8_t* keep,
                                 float keep_scale, float* y, float* psave, const float* post_u,
                                 float post_p, float* post_out, int64_t num_graphs, int n,
                                 int heads, int channels, int concat, int act,
                                 float negative_slope, hipStream_t stream) {
  if (!xs || !y || !psave) return SV2N_ERR_ARG;
  if (int rc = check_attn_args(num_graphs, n, heads, channels, ldx, act)) return rc;
  if (ae_edge_order && (rowmask || n < 2)) return SV2N_ERR_ARG;  // complete graphs only
  if (post_u && (!post_out || !(post_p >= 0.f && post_p < 1.f))) return SV2N_ERR_ARG;
  attn_canon_fwd(num_graphs, stream, xs, ldx, ae, ae_edge_order, rowmask, bias, keep,
                 keep_scale, y, psave, post_u, post_p, post_out, n, heads, channels, concat, act,
                 negative_slope, HeadFuse{});
  return (int)hipGetLastError();
}

extern "C" int sv2n_gat_attn_fwd_head_mse_supported(int64_t num_graphs, int n, int heads,
                                                    int channels, int concat) {
  if (num_graphs <= 0 || channels <= 0 || heads < 1 || heads > SV2N_MAX_HEADS) return 0;
  return attn_canon_head_ok(num_graphs, n, heads, channels, concat != 0) ? 1 : 0;
}

extern "C" int64_t sv2n_gat_attn_fwd_head_mse_workspace(int64_t num_graphs, int heads,
                                                        int channels, int concat) {
  if (num_graphs <= 0 || heads < 1 || channels < 1) return 0;
  return num_graphs * ((concat ? heads * channels : channels) + 2);  // per-graph partials
}

extern "C" int sv2n_gat_attn_fwd_head_mse(
    const float* xs, int ldx, const float* ae, int ae_edge_order, const uint32_t* rowmask,
    const float* bias, const uint8_t* keep, float keep_scale, float* dz, float* psave,
    const float* post_u, float post_p, const float* head_weight, const float* head_bias,
    const float* target, float* loss, float* loss_sum, float* g_head_weight, float* g_head_bias,
    float* workspace, int64_t workspace_floats, int64_t num_graphs, int n, int heads,
    int channels, int concat, int act, float negative_slope, hipStream_t stream) {
  if (!xs || !dz || !psave || !head_weight || !target || !loss || !workspace)
    return SV2N_ERR_ARG;
  if ((uintptr_t)workspace & 15) return SV2N_ERR_ALIGN;
  if (int rc = check_attn_args(num_graphs, n, heads, channels, ldx, act)) return rc;
  if (ae_edge_order && (rowmask || n < 2)) return SV2N_ERR_ARG;
  if (post_u && !(post_p >= 0.f && post_p < 1.f)) return SV2N_ERR_ARG;
  if (!attn_canon_head_ok(num_graphs, n, heads, channels, concat != 0)) return SV2N_ERR_SHAPE;
  if (workspace_floats <
      sv2n_gat_attn_fwd_head_mse_workspace(num_graphs, heads, channels, concat))
    return SV2N_ERR_WORKSPACE;
  HeadFuse hf{};
  hf.w = head_weight;
  hf.b = head_bias;
  hf.target = target;
  hf.part = workspace;
  hf.inv_n2 = (float)(2.0 / ((double)num_graphs * n));
  hf.gw = g_head_weight;
  hf.gb = g_head_bias;
  hf.loss = loss;
  hf.loss_sum = loss_sum;
  attn_canon_fwd(num_graphs, stream, xs, ldx, ae, ae_edge_order, rowmask, bias, keep,
                 keep_scale, dz, psave, post_u, post_p, nullptr, n, heads, channels, concat, act,
                 negative_slope, hf);
  return (int)hipGetLastError();
}

extern "C" int sv2n_gat_attn_bwd(const float* dy, const float* y, const float* xs, int ldx,
                                 const float* psave, const uint8_t* keep, float keep_scale,
                                 const float* post_u, float post_p, const uint32_t* rowmask,
                                 float* dxs, float* dae, int ae_edge_order, float* dbias_partial,
                                 int64_t num_graphs, int n, int heads, int channels, int concat,
                                 int act, float negative_slope, hipStream_t stream) {
  if (!dy || !y || !xs || !psave || !dxs || !dbias_partial) return SV2N_ERR_ARG;
  if (int rc = check_attn_args(num_graphs, n, heads, channels, ldx, act)) return rc;
  if (ae_edge_order && (rowmask || n < 2)) return SV2N_ERR_ARG;  // complete graphs only
  if (post_u && !(post_p >= 0.f && post_p < 1.f)) return SV2N_ERR_ARG;
  attn_canon_bwd(num_graphs, stream, dy, y, xs, ldx, psave, keep, keep_scale, post_u, post_p,
                 rowmask, dxs,
                 dae, ae_edge_order, dbias_partial, n, heads, channels, concat, act,
                 negative_slope, EdgeTail{});
  return (int)hipGetLastError();
}

extern "C" int sv2n_gat_attn_bwd_bf16dx(const float* dy, const float* y, const float* xs,
                                        int ldx, const float* psave, const uint8_t* keep,
                                        float keep_scale, const float* post_u, float post_p,
                                        const uint32_t* rowmask, uint16_t* dxs_bf16, int ld_dxs,
                                        float* dae, int ae_edge_order, float* dbias_partial,
                                        int64_t num_graphs, int n, int heads, int channels,
                                        int concat, int act, float negative_slope,
                                        hipStream_t stream) {
  if (!dy || !y || !xs || !psave || !dxs_bf16 || !dbias_partial) return SV2N_ERR_ARG;
  if (int rc = check_attn_args(num_graphs, n, heads, channels, ldx, act)) return rc;
  if (ld_dxs < ldx || (ld_dxs & 7)) return SV2N_ERR_SHAPE;
  if ((uintptr_t)dxs_bf16 & 15) return SV2N_ERR_ALIGN;
  if (post_u && !(post_p >= 0.f && post_p < 1.f)) return SV2N_ERR_ARG;
  if (ae_edge_order && (rowmask || n < 2)) return SV2N_ERR_ARG;
  attn_canon_bwd(num_graphs, stream, dy, y, xs, ldx, psave, keep, keep_scale, post_u, post_p,
                 rowmask, nullptr, dae, ae_edge_order, dbias_partial, n, heads, channels, concat,
                 act, negative_slope, EdgeTail{}, reinterpret_cast<unsigned short*>(dxs_bf16),
                 ld_dxs);
  return (int)hipGetLastError();
}

extern "C" int sv2n_gat_attn_bwd_edge_supported(int64_t num_graphs, int n, int heads, int channels,
                                                int edge_dim, int hl_pad) {
  if (num_graphs <= 0 || channels <= 0 || heads < 1 || heads > SV2N_MAX_HEADS) return 0;
  return attn_canon_edge_tail_ok(num_graphs, n, heads, channels, edge_dim, hl_pad) ? 1 : 0;
}

extern "C" int sv2n_gat_attn_bwd_edge(const float* dy, const float* y, const float* xs, int ldx,
                                      const float* psave, const uint8_t* keep, float keep_scale,
                                      const float* post_u, float post_p, float* dxs,
                                      float* dbias_partial, const float* edge_attr, int edge_dim,
                                      const float* const* layer_dae, int num_layers, int layer,
                                      int hl_pad, float* edge_partial, int64_t num_graphs, int n,
                                      int heads, int channels, int concat, int act,
                                      float negative_slope, hipStream_t stream) {
  if (!dy || !y || !xs || !psave || !dxs || !dbias_partial || !edge_attr || !edge_partial ||
      !layer_dae)
    return SV2N_ERR_ARG;
  if (int rc = check_attn_args(num_graphs, n, heads, channels, ldx, act)) return rc;
  if (post_u && !(post_p >= 0.f && post_p < 1.f)) return SV2N_ERR_ARG;
  if (num_layers < 1 || num_layers > SV2N_MAX_LAYERS || layer < 0 || layer >= num_layers ||
      num_layers * heads > hl_pad)
    return SV2N_ERR_SHAPE;
  if (!attn_canon_edge_tail_ok(num_graphs, n, heads, channels, edge_dim, hl_pad))
    return SV2N_ERR_SHAPE;
  if ((uintptr_t)edge_attr % 16) return SV2N_ERR_ALIGN;
  EdgeTail et{};
  et.ea = edge_attr;
  for (int l = 0; l < num_layers; ++l) {
    if (l == layer) continue;
    if (!layer_dae[l]) return SV2N_ERR_ARG;
    et.dae[l] = layer_dae[l];
  }
  et.part = edge_partial;
  et.D = edge_dim;
  et.L = num_layers;
  et.own = layer;
  et.hlp = hl_pad;
  attn_canon_bwd(num_graphs, stream, dy, y, xs, ldx, psave, keep, keep_scale, post_u, post_p,
                 nullptr, dxs, nullptr, 1, dbias_partial, n, heads, channels, concat, act,
                 negative_slope, et);
  return (int)hipGetLastError();
}
