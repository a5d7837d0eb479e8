"""SpotV2Net GAT hot-path benchmark (BASELINE.json metric, config C2).

Workload: one training step (forward + MSELoss + backward + Adam, reference
5_train_SpotV2Net.py:150-159) of GATModel with the C2 configuration — 30-node
fully connected graphs, seq_length 42 (F = 1260 node / D = 126 edge
features), 2 GAT layers [100, 50], 4 heads, concat_heads — over a
device-resident synthetic batch of 512 window graphs per GPU, fp32.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

value = graphs processed by ALL ranks / max-over-ranks wall time (weak
scaling: 512 graphs per GPU).  The JSON line also carries the fwd-only rate,
the dominant kernel's roofline point (HIP events on its launch stream) and the
CPU baseline (oracle restatement of PyG GATConv, rank 0 at N = 1 only).
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import platform
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "graphs/sec (30-node dense GAT, batch=512) at 1/2/4/8 MI355X vs PyG-CPU"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
F32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32, dense
# the split GEMM computes each f32 product as 6 bf16 MFMA products: its
# f32-equivalent ceiling is the dense bf16 MFMA peak (~2.5 PF) / 6
BF16X3_PEAK_TFLOPS = round(2500.0 / 6, 1)
BF16_MFMA_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA (no sparsity)

S, N_NODES, HEADS, HIDDEN, BATCH = 42, 30, 4, [100, 50], 512

# BASELINE.json configs.  c2 is the headline workload (the
# driver's default run); the others are measured with --config.
CONFIGS = {
    "c1": dict(S=42, n=30, heads=1, hidden=[500], concat=False, batch=32, dropout_att=0.0,
               dropout=0.0,
               desc="C1: 1 GAT layer, 1 head, hidden [500], 30-node dense graphs, S=42"),
    "c2": dict(S=42, n=30, heads=4, hidden=[100, 50], concat=True, batch=512, dropout_att=0.0,
               dropout=0.0,
               desc="C2 train step (fwd+MSE+bwd+Adam): 30-node dense GAT graphs, "
                    "870 edges + self loops, seq_length 42 (F=1260, D=126), "
                    "GAT [100,50] x 4 heads concat, relu"),
    # config/GNN_param.yaml:26-39 as-is: dropout_att 0.0, dropout 0.1
    "c3": dict(S=42, n=30, heads=6, hidden=[500], concat=True, batch=128, dropout_att=0.0,
               dropout=0.1,
               desc="C3: config/GNN_param.yaml model (S=42, hidden [500], 6 heads, "
                    "dropout_att 0.0, dropout 0.1, batch 128)"),
    "c5": dict(S=4, n=256, heads=8, hidden=[16, 16, 16], concat=True, batch=1024,
               dropout_att=0.0, dropout=0.0,
               desc="C5 stress: 256-node dense graphs (65,280 edges), S=4 (F=1024, D=12), "
                    "3 GAT layers [16,16,16] x 8 heads concat"),
}


def build_model(dev, cfg=None):
    from spotv2net_amd import GATModel
    cfg = cfg or CONFIGS["c2"]
    torch.manual_seed(5154)  # config/GNN_param.yaml:23
    return GATModel(cfg["n"] * cfg["S"], 3 * cfg["S"], cfg["heads"], 1, cfg["hidden"],
                    dropout_att=cfg["dropout_att"], dropout=cfg["dropout"],
                    concat_heads=cfg["concat"], activation="relu", negative_slope=0.2).to(dev)


def time_replays(fn, k, sync_group=True):
    if sync_group and dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    if sync_group and dist.is_initialized():
        dist.barrier()
    return time.perf_counter() - t0


def _coll_device(dev):
    """Where a collective's tensors live: the GPU under nccl (RCCL), the host
    under gloo."""
    return dev if dist.get_backend() == "nccl" else torch.device("cpu")


def max_over_ranks(x: float, dev) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], device=_coll_device(dev), dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def replicas_identical(flat: torch.Tensor, dev) -> bool:
    """Every rank's parameters bit for bit equal: the elementwise MAX and MIN
    over ranks of the parameters' int32 bit patterns both equal this rank's."""
    bits = flat.detach().view(torch.int32).to(_coll_device(dev))
    hi, lo = bits.clone(), bits.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    ok = torch.tensor([int(torch.equal(hi, bits) and torch.equal(lo, bits))],
                      device=_coll_device(dev), dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    return bool(ok.item())


# --------------------------------------------------------------------------
# per-kernel timing (HIP events on the stream the kernels are launched on)
# --------------------------------------------------------------------------
def kernel_table(model, data, reps=50):
    from spotv2net_amd import ops
    from spotv2net_amd.layout import analyze_edge_index
    dev = data.x.device
    stream = torch.cuda.current_stream(dev)
    B = data.x.shape[0] // N_NODES
    layout = analyze_edge_index(data.edge_index, data.x.shape[0], N_NODES)
    L = len(model.gat_layers)
    with torch.no_grad():
        W = [c.projection_weight().contiguous() for c in model.gat_layers]
        wf = torch.cat([c.edge_fold() for c in model.gat_layers], 1)
    x0 = data.x
    N0 = x0.shape[0]
    xs0 = ops.gemm_f32(x0, True, W[0], True, N0, W[0].shape[0], x0.shape[1])
    conv0 = model.gat_layers[0]
    lib = ops._lib.load()
    sh = stream.cuda_stream
    E, D = data.edge_attr.shape
    wfp, hp = ops.pad_columns(wf)
    ae = [torch.empty(E, HEADS, device=dev) for _ in range(L)]  # canonical: edge order
    ptrs = ops._lib.ptr_array([a.data_ptr() for a in ae])

    def edge_fwd():
        lib.sv2n_edge_logits_fwd(data.edge_attr.data_ptr(), E, D, None, layout.canon.data_ptr(),
                                 wfp.data_ptr(), hp, ptrs, L, HEADS, B, N_NODES, sh)

    edge_fwd()
    y0 = torch.empty(N0, conv0.out_dim, device=dev)
    ps0 = torch.empty(B, HEADS, 32, 32, device=dev)

    def attn_fwd():
        lib.sv2n_gat_attn_fwd(xs0.data_ptr(), xs0.stride(0), ae[0].data_ptr(), 1, None,
                              conv0.bias.data_ptr(), None, 1.0, y0.data_ptr(), ps0.data_ptr(),
                              None, 0.0, None, B, N_NODES, HEADS, conv0.out_channels, 1, 1, 0.2, sh)

    dy0 = torch.randn_like(y0)
    dxs0 = torch.empty_like(xs0)
    dae0 = torch.empty_like(ae[0])
    dbp = torch.empty(B, conv0.out_dim, device=dev)

    # as the step runs it: layer 1's dx GEMM stores dZ = relu'(y0)·dy0
    # (sv2n_gemm_f32x3_relu), so layer 0's backward runs with act = identity
    # and reads no y
    def attn_bwd():
        lib.sv2n_gat_attn_bwd(dy0.data_ptr(), y0.data_ptr(), xs0.data_ptr(), xs0.stride(0),
                              ps0.data_ptr(), None, 1.0, None, 0.0, None, dxs0.data_ptr(),
                              dae0.data_ptr(),
                              1, dbp.data_ptr(), B, N_NODES, HEADS, conv0.out_channels, 1, 0, 0.2,
                              sh)

    ws_n = lib.sv2n_edge_logits_bwd_workspace(D, hp)
    ws = torch.empty(ws_n, device=dev)
    dwf = torch.empty(D, hp, device=dev)

    def edge_bwd():
        lib.sv2n_edge_logits_bwd(data.edge_attr.data_ptr(), E, D, None, layout.canon.data_ptr(),
                                 ptrs, L, HEADS, B, N_NODES, ws.data_ptr(), ws_n,
                                 dwf.data_ptr(), hp, sh)

    # the covariance-layout edge passes, launched as the step launches them
    # (stack.stack_forward -> sv2n::edge_logits_cv, stack_backward ->
    # sv2n::edge_logits_bwd_cv: the main pass and its partial-slab reduce)
    S_cv = D // 3
    ae_cv = [torch.empty(E, HEADS, device=dev) for _ in range(L)]
    ptrs_cv = ops._lib.ptr_array([a.data_ptr() for a in ae_cv])
    ws_cv_n = lib.sv2n_edge_logits_bwd_cv_workspace(S_cv, hp)
    ws_cv = torch.empty(ws_cv_n, device=dev)
    dwf_cv = torch.empty(D, hp, device=dev)

    def edge_fwd_cv():
        lib.sv2n_edge_logits_fwd_cv(data.edge_attr.data_ptr(), B, N_NODES, S_cv,
                                    layout.canon.data_ptr(), wfp.data_ptr(), hp, ptrs_cv, L,
                                    HEADS, sh)

    def edge_bwd_cv():
        lib.sv2n_edge_logits_bwd_cv(data.edge_attr.data_ptr(), B, N_NODES, S_cv,
                                    layout.canon.data_ptr(), ptrs_cv, L, HEADS, ws_cv.data_ptr(),
                                    ws_cv_n, dwf_cv.data_ptr(), hp, sh)

    # what the covariance-layout passes must move (cv_edge_bytes): the upper
    # rows' covariance columns, one variance series per node, and the logits
    # (written forward, read backward)
    cv_read = cv_edge_bytes_per_graph(N_NODES, S_cv) * B
    cv_logits = 4.0 * E * L * HEADS

    out0 = torch.empty_like(xs0)
    # the layer-0 projection as the step runs it: the f32-accurate split GEMM
    # (sv2n_gemm_f32x3) on the weight's pre-split bf16 planes
    planes0 = ops.weight_planes(W[0], False)

    def gemm_fwd():
        lib.sv2n_gemm_f32x3(x0.data_ptr(), x0.stride(0), planes0.data_ptr(), out0.data_ptr(),
                            out0.stride(0), N0, W[0].shape[0], x0.shape[1], sh)

    # the layer-0 weight-gradient GEMM (split-K, bf16x3 on MFMA; its slab reduce
    # and epilogue are separate launches of sv2n_gat_wgrad_node)
    Fd, Nd = x0.shape[1], W[0].shape[0]
    nslab = lib.sv2n_gemm_f32_slabs_count(Fd, Nd, N0)
    slabs = torch.empty(nslab * Fd * Nd, device=dev)

    def gemm_dwt():
        lib.sv2n_gemm_f32_slabs(0, 0, x0.data_ptr(), x0.stride(0), dxs0.data_ptr(),
                                dxs0.stride(0), Fd, Nd, N0, slabs.data_ptr(), slabs.numel(), sh)

    # algorithmic work: the H·C projection columns plus the node
    # logits (4·n·H·C per graph), not the GEMM's padded / augmented columns
    M0, K0 = N0, x0.shape[1]
    HC0 = conv0.heads * conv0.out_channels
    N0c = W[0].shape[0]
    # (fn, bound, algorithmic flops, algorithmic bytes, peak for the arithmetic used)
    rows = {
        "gemm_l0_fwd": (gemm_fwd, "mfma", 2.0 * M0 * HC0 * K0 + 4.0 * M0 * HC0,
                        4.0 * (M0 * K0 + HC0 * K0 + M0 * HC0), BF16X3_PEAK_TFLOPS),
        # bf16x3 weight-gradient kernel (k_gemm_tt3y): dW = xᵀ·dxs over the H·C columns
        "gemm_l0_dwT": (gemm_dwt, "mfma", 2.0 * M0 * HC0 * K0,
                        4.0 * (M0 * K0 + M0 * N0c + HC0 * K0), BF16X3_PEAK_TFLOPS),
        "edge_logits_fwd": (edge_fwd, "hbm", 2.0 * E * D * L * HEADS, 4.0 * (E * D + E * L * HEADS),
                            None),
        "edge_logits_bwd": (edge_bwd, "hbm", 2.0 * E * D * L * HEADS, 4.0 * (E * D + E * L * HEADS),
                            None),
        "edge_logits_fwd_cv": (edge_fwd_cv, "hbm", 2.0 * E * D * L * HEADS / 6,
                               cv_read + cv_logits, None),
        "edge_logits_bwd_cv": (edge_bwd_cv, "hbm", 2.0 * E * D * L * HEADS / 6,
                               cv_read + cv_logits, None),
        "gat_attn_fwd_l0": (attn_fwd, "hbm", 2.0 * B * N_NODES * N_NODES * HEADS * conv0.out_channels,
                            4.0 * (xs0.numel() + ae[0].numel() + y0.numel() + ps0.numel()), None),
        # dZ, xs and psave read; dxs, d ae and the bias partials written
        "gat_attn_bwd_l0": (attn_bwd, "hbm", 4.0 * B * N_NODES * N_NODES * HEADS * conv0.out_channels,
                            4.0 * (y0.numel() + 2 * xs0.numel() + ps0.numel() + ae[0].numel() +
                                   dbp.numel()),
                            None),
    }
    return time_rows(rows, stream, reps, order=["edge_logits_fwd_cv", "edge_logits_fwd",
                                                "gemm_l0_fwd", "gat_attn_fwd_l0",
                                                "gat_attn_bwd_l0", "gemm_l0_dwT", "edge_logits_bwd",
                                                "edge_logits_bwd_cv"])


def cv_edge_bytes_per_graph(n: int, S: int) -> float:
    """edge_attr bytes a covariance-layout edge pass must read per graph
    (sv2n_edge.hip k_edge_fwd_cv / k_edge_bwd_cv): the S covariance columns
    of the n(n-1)/2 upper rows and one S-long variance series per node
    (utils/dataset.py:228-243: the swapped row repeats the covariance, the
    variances are node series)."""
    return 4.0 * (n * (n - 1) // 2 * S + n * S)


def time_rows(rows, stream, reps, order):
    """Per-launch HIP-event times of the rows' kernels launched in ``order``
    (their order in the training step), ``reps`` rounds back to back: each
    kernel runs among the others as in the step, at the clock that mix
    sustains.  Launched back to back with itself an MFMA-dense kernel runs at
    a lower sustained clock (C2 L0 projection ~103 us against 86-97 in the
    traced training steps, `profiles/r03_c2_gemm_in_step_trace.txt`) and an
    edge pass finds part of edge_attr still in the Infinity Cache; both
    figures are reported (``avg_us`` in step order, ``avg_us_back_to_back``)."""
    res = {}
    for name, (fn, bound, flops, nbytes, peak) in rows.items():
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        res[name] = dict(avg_us_back_to_back=e0.elapsed_time(e1) * 1e3 / reps, bound=bound,
                         flops=flops, bytes=nbytes, peak_tflops=peak)
    evs = {name: [] for name in order}
    for _ in range(reps):
        for name in order:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            rows[name][0]()
            b.record(stream)
            evs[name].append((a, b))
    torch.cuda.synchronize()
    for name, r in res.items():
        us = sum(a.elapsed_time(b) for a, b in evs[name]) * 1e3 / len(evs[name])
        r.update(avg_us=us, tflops=r["flops"] / us / 1e6, gbs=r["bytes"] / us / 1e3)
    return res


def kernel_table_tiled(model, data, cfg, reps=10):
    """C5 (32 < n <= 256, narrow edge_attr): the layer-0 edge-fused attention
    forward and backward (sv2n_gat_attn_fused_*: prep + main + finish) and the
    layer-0 projection / weight-gradient GEMMs, HIP events on the launch stream.
    Algorithmic bytes per launch: every tensor the call must read or write,
    once — edge_attr, xs, the layer output and the saved aggregates /
    statistics (forward); edge_attr, xs, dy, y, agg, statistics and dxs
    (backward)."""
    from spotv2net_amd import ops
    dev = data.x.device
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    n, H = cfg["n"], cfg["heads"]
    N0 = data.x.shape[0]
    B = N0 // n
    lib = ops._lib.load()
    with torch.no_grad():
        W0 = model.gat_layers[0].projection_weight().contiguous()
        wf = torch.cat([c.edge_fold() for c in model.gat_layers], 1)
    conv0 = model.gat_layers[0]
    C = conv0.out_channels
    HC = H * C
    ldx = (HC + 2 * H + 3) // 4 * 4
    xs0 = torch.zeros(N0, ldx, device=dev)
    xs0[:, :W0.shape[0]] = ops.gemm_f32(data.x, True, W0, True, N0, W0.shape[0], data.x.shape[1])
    E, D = data.edge_attr.shape
    wfp, hp = ops.pad_columns(wf)
    y0 = torch.empty(N0, HC, device=dev)
    agg0 = torch.empty(N0, HC, device=dev)
    st0 = torch.empty(N0, 4 * H, device=dev)
    dy0 = torch.randn_like(y0)
    dxs0 = torch.empty_like(xs0)
    NT = (n + 31) // 32
    dbp = torch.empty(B * NT, HC, device=dev)
    dwf = torch.zeros(D, hp, device=dev)
    ws_n = lib.sv2n_gat_attn_fused_bwd_workspace(B, n, H, C, D)
    ws = torch.empty(ws_n, device=dev)

    def attn_fwd():
        lib.sv2n_gat_attn_fused_fwd(xs0.data_ptr(), ldx, data.edge_attr.data_ptr(), D,
                                    wfp.data_ptr(), hp, 0, None, conv0.bias.data_ptr(), None, 1.0,
                                    y0.data_ptr(), agg0.data_ptr(), st0.data_ptr(), B, n, H, C,
                                    1, 1, 0.2, sh)

    def attn_bwd():
        lib.sv2n_gat_attn_fused_bwd(dy0.data_ptr(), y0.data_ptr(), agg0.data_ptr(),
                                    st0.data_ptr(), xs0.data_ptr(), ldx,
                                    data.edge_attr.data_ptr(), D, wfp.data_ptr(), hp, 0, None,
                                    None, 1.0, dxs0.data_ptr(), dbp.data_ptr(), dwf.data_ptr(),
                                    ws.data_ptr(), ws_n, B, n, H, C, 1, 1, 0.2, sh)

    x0 = data.x
    planes0 = ops.weight_planes(W0, False)
    out0 = torch.empty(N0, W0.shape[0], device=dev)

    def gemm_fwd():
        lib.sv2n_gemm_f32x3(x0.data_ptr(), x0.stride(0), planes0.data_ptr(), out0.data_ptr(),
                            out0.stride(0), N0, W0.shape[0], x0.shape[1], sh)

    Fd, Nd = x0.shape[1], ldx
    nslab = lib.sv2n_gemm_f32_slabs_count(Fd, Nd, N0)
    slabs = torch.empty(nslab * Fd * Nd, device=dev)

    def gemm_dwt():
        lib.sv2n_gemm_f32_slabs(0, 0, x0.data_ptr(), x0.stride(0), dxs0.data_ptr(),
                                dxs0.stride(0), Fd, Nd, N0, slabs.data_ptr(), slabs.numel(), sh)

    attn_fwd()  # the backward reads the training forward's outputs
    eab, xsb, rowb, stb = 4.0 * E * D, 4.0 * N0 * ldx, 4.0 * N0 * HC, 4.0 * N0 * 4 * H
    M0, K0 = N0, x0.shape[1]
    Nc = HC   # algorithmic columns, not the augmented / padded ones
    # (fn, bound, algorithmic flops, algorithmic bytes, peak)
    rows = {
        "gat_attn_fused_fwd_l0": (attn_fwd, "hbm", 0.0, eab + xsb + 2 * rowb + stb, None),
        "gat_attn_fused_bwd_l0": (attn_bwd, "hbm", 0.0, eab + 2 * xsb + 3 * rowb + stb, None),
        "gemm_l0_fwd": (gemm_fwd, "mfma", 2.0 * M0 * Nc * K0 + 4.0 * M0 * Nc,
                        4.0 * (M0 * K0 + Nc * K0 + M0 * Nc), BF16X3_PEAK_TFLOPS),
        "gemm_l0_dwT": (gemm_dwt, "mfma", 2.0 * M0 * Nc * K0, 4.0 * (M0 * K0 + M0 * Nd + Nc * K0),
                        BF16X3_PEAK_TFLOPS),
    }
    return time_rows(rows, stream, reps, order=["gemm_l0_fwd", "gat_attn_fused_fwd_l0",
                                                "gat_attn_fused_bwd_l0", "gemm_l0_dwT"])


def kernel_table_c3(model, cfg, precision, reps=20):
    """C3 (the yaml model: F 1260, 6 heads x 500, mean, B 128) in its execution
    mode: the layer's projection GEMM, its weight-gradient GEMM with the fold
    epilogue (sv2n_gat_wgrad_node[_bf16], slab reduce included), and the
    attention forward / backward, HIP events on the launch stream.  Flops:
    2·M·N·K of the GEMM; bytes: every operand once."""
    from spotv2net_amd import ops, synthetic_batch
    from spotv2net_amd.layout import canonical_edge_index
    dev = next(model.parameters()).device
    B, n, H = cfg["batch"], cfg["n"], cfg["heads"]
    data = synthetic_batch(B, cfg["S"], n=n, seed=99, device=dev)
    conv = model.gat_layers[0]
    C = conv.out_channels
    HC = H * C
    lib = ops._lib.load()
    sh = torch.cuda.current_stream(dev).cuda_stream
    x = data.x
    N, F = x.shape
    with torch.no_grad():
        W = conv.projection_weight().contiguous()
    ldx = W.shape[0]
    bf16 = precision == "bf16"
    planes = ops.weight_planes(W, False)
    xs = torch.empty(N, ldx, device=dev)

    # bf16 mode as the C3 loop runs it: the window gather leaves bf16(x)
    # beside x, the projection reads it (sv2n_gemm_bf16_a16), the weight
    # gradient reads bf16 x and bf16 dxs (sv2n_gat_wgrad_node_bf16b), the
    # attention backward writes bf16 dxs
    kb = (F + 63) // 64 * 64
    xb = torch.zeros(N, kb, device=dev, dtype=torch.bfloat16)
    xb[:, :F] = x.to(torch.bfloat16)

    def gemm_fwd():
        if bf16:
            lib.sv2n_gemm_bf16_a16(xb.data_ptr(), kb, planes.data_ptr(), xs.data_ptr(),
                                   xs.stride(0), N, ldx, F, sh)
        else:
            lib.sv2n_gemm_f32x3(x.data_ptr(), x.stride(0), planes.data_ptr(), xs.data_ptr(),
                                xs.stride(0), N, ldx, F, sh)

    gemm_fwd()
    dxs = torch.randn(N, ldx, device=dev) * 1e-3
    att_s = conv.att_src.detach().reshape(-1).contiguous()
    att_d = conv.att_dst.detach().reshape(-1).contiguous()
    dbp = torch.randn(B, C, device=dev)
    gW = torch.zeros(HC, F, device=dev)
    ga, gd, gb = (torch.zeros(HC, device=dev), torch.zeros(HC, device=dev),
                  torch.zeros(C, device=dev))
    ws_fn = lib.sv2n_gat_wgrad_node_bf16_workspace if bf16 else lib.sv2n_gat_wgrad_node_workspace
    ws_n = ws_fn(N, F, ldx, H, C)
    ws = torch.empty(ws_n, device=dev)

    ldb = (ldx + 7) // 8 * 8
    dxb = dxs.new_zeros(N, ldb).to(torch.bfloat16)
    dxb[:, :ldx] = dxs.to(torch.bfloat16)

    def wgrad():
        if bf16:
            lib.sv2n_gat_wgrad_node_bf16b(
                xb.data_ptr(), kb, dxb.data_ptr(), ldb, N, F, ldx,
                conv.lin_src.weight.data_ptr(), att_s.data_ptr(), att_d.data_ptr(), H, C,
                dbp.data_ptr(), B, C, gW.data_ptr(), ga.data_ptr(), gd.data_ptr(), gb.data_ptr(),
                ws.data_ptr(), ws_n, sh)
        else:
            lib.sv2n_gat_wgrad_node(
                x.data_ptr(), x.stride(0), dxs.data_ptr(), ldx, N, F,
                conv.lin_src.weight.data_ptr(), att_s.data_ptr(), att_d.data_ptr(), H, C,
                dbp.data_ptr(), B, C, gW.data_ptr(), ga.data_ptr(), gd.data_ptr(), gb.data_ptr(),
                ws.data_ptr(), ws_n, sh)

    E = data.edge_attr.shape[0]
    ae = torch.randn(E, H, device=dev)
    y = torch.empty(N, C, device=dev)
    ps = torch.empty(B, H, 32, 32, device=dev)

    def attn_fwd():
        lib.sv2n_gat_attn_fwd(xs.data_ptr(), ldx, ae.data_ptr(), 1, None, conv.bias.data_ptr(),
                              None, 1.0, y.data_ptr(), ps.data_ptr(), None, 0.0, None, B, n, H,
                              C, 0, 1, 0.2, sh)

    attn_fwd()
    dy = torch.randn_like(y)
    dxs2 = torch.empty_like(xs)
    dae = torch.empty_like(ae)
    dbp2 = torch.empty(B, C, device=dev)

    dxb2 = torch.empty_like(dxb)

    def attn_bwd():
        if bf16:
            lib.sv2n_gat_attn_bwd_bf16dx(dy.data_ptr(), y.data_ptr(), xs.data_ptr(), ldx,
                                         ps.data_ptr(), None, 1.0, None, 0.0, None,
                                         dxb2.data_ptr(), ldb, dae.data_ptr(), 1, dbp2.data_ptr(),
                                         B, n, H, C, 0, 1, 0.2, sh)
        else:
            lib.sv2n_gat_attn_bwd(dy.data_ptr(), y.data_ptr(), xs.data_ptr(), ldx, ps.data_ptr(),
                                  None, 1.0, None, 0.0, None, dxs2.data_ptr(), dae.data_ptr(), 1,
                                  dbp2.data_ptr(), B, n, H, C, 0, 1, 0.2, sh)

    peak = BF16_MFMA_PEAK_TFLOPS if bf16 else BF16X3_PEAK_TFLOPS
    gflop = 2.0 * N * HC * F + 4.0 * N * HC   # algorithmic: H·C columns
    rows = {
        # bf16: x read as its bf16 twin
        "gemm_fwd": (gemm_fwd, "mfma", gflop, (2.0 * N * kb if bf16 else 4.0 * N * F)
                     + 4.0 * N * ldx + (2 if bf16 else 6) * ldx * F, peak),
        # bf16: both operands bf16 in memory; gW (and the fold's W) read and written
        "wgrad_node": (wgrad, "mfma", gflop,
                       (2.0 * (N * kb + N * ldb) if bf16 else 4.0 * (N * F + N * ldx))
                       + 4.0 * 3 * HC * F, peak),
        "gat_attn_fwd": (attn_fwd, "hbm", 2.0 * B * n * n * HC,
                         4.0 * (xs.numel() + ae.numel() + y.numel() + ps.numel()), None),
        "gat_attn_bwd": (attn_bwd, "hbm", 4.0 * B * n * n * HC,
                         4.0 * (2 * y.numel() + 2 * xs.numel() + ps.numel() + ae.numel()), None),
    }
    return time_rows(rows, torch.cuda.current_stream(dev), reps,
                     order=["gemm_fwd", "gat_attn_fwd", "gat_attn_bwd", "wgrad_node"])


def roofline_entry(table, traffic=None):
    # dominant = largest time per training step (gemm rows run once per step at L0)
    name = max(table, key=lambda k: table[k]["avg_us"])
    r = table[name]
    if r["bound"] == "mfma":
        ach, peak, unit = r["tflops"], r.get("peak_tflops") or F32_MFMA_PEAK_TFLOPS, "TFLOP/s"
    else:
        ach, peak, unit = r["gbs"], HBM_PEAK_GBS, "GB/s"
    return name, {"kernel": name, "bound": r["bound"], "achieved": round(ach, 2), "peak": peak,
                  "unit": unit, "frac": round(ach / peak, 4), "avg_us": round(r["avg_us"], 2),
                  "avg_us_back_to_back": round(r.get("avg_us_back_to_back", r["avg_us"]), 2),
                  "timing": "HIP events per launch, the table's kernels launched in their "
                            "training-step order (bench.time_rows)",
                  "traffic": traffic}


def load_traffic(kernel):
    """HBM bytes per launch from a committed rocprofv3 --pmc pass
    (tools/pmc_traffic.py writes profiles/pmc_traffic.json), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


# --------------------------------------------------------------------------
# CPU baseline: PyG-semantics oracle, same model/config, host cores
# --------------------------------------------------------------------------
def usable_cores() -> int:
    """CPUs this process may actually run on: the affinity mask, further
    capped by a cgroup-v2 CPU quota when one is set (a GPU box's share of a
    large host; os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, int(n or 1))


def _cpu_name() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "cpu"


def _cpu_rate(cfg, state, batch: int, train: bool, warmup: int = 3, steps: int = 20,
              seed: int = 4321) -> float:
    """SURVEY §8(d) CPU protocol: the oracle GATModel with PyG 2.3.0's
    unfolded op sequence (lin_edge materialised, scatter softmax, index_add
    aggregation), `warmup` + `steps` iterations timed with perf_counter."""
    from oracle.pyg_gatconv import OracleGATModel
    from spotv2net_amd import Data, synthetic_batch
    ref = OracleGATModel(cfg["n"] * cfg["S"], 3 * cfg["S"], cfg["heads"], 1, cfg["hidden"],
                         dropout_att=cfg["dropout_att"], dropout=cfg["dropout"],
                         concat_heads=cfg["concat"])
    if state is not None:
        ref.load_state_dict(state)
    data = synthetic_batch(batch, cfg["S"], n=cfg["n"], seed=seed)
    d = Data(x=data.x, edge_index=data.edge_index, edge_attr=data.edge_attr)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    ref.train(train)

    def step():
        if train:
            loss = torch.nn.functional.mse_loss(ref(d), data.y_x)
            opt.zero_grad()
            loss.backward()
            opt.step()
        else:
            with torch.no_grad():
                ref(d)

    for _ in range(warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    return steps * batch / (time.perf_counter() - t0)


def cpu_baseline(model, cfg, batch: int) -> dict:
    """The reference's CPU path (PyG-semantics restatement; PyG itself is
    absent) on this box's host cores, rank 0 at N = 1: the benched config's
    train step (value) and forward, and the C1 config (B = 32) beside it."""
    cores = usable_cores()
    torch.set_num_threads(cores)
    state = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    t0 = time.perf_counter()
    # bounded sample (~10-30 s of CPU work): SURVEY 8(d)'s 3 + 20 steps at
    # small batches, 1 + 5 at the benched config's 512 graphs per step
    wu, st = (1, 5) if batch >= 256 else (3, 20)
    train = _cpu_rate(cfg, state, batch, True, warmup=wu, steps=st)
    fwd = _cpu_rate(cfg, state, batch, False, warmup=wu, steps=st)
    c1 = CONFIGS["c1"]
    c1_train = _cpu_rate(c1, None, c1["batch"], True)
    c1_fwd = _cpu_rate(c1, None, c1["batch"], False)
    el = time.perf_counter() - t0
    return {"value": round(train, 2), "unit": "graphs/s", "cores": cores, "kind": "port",
            "fwd_value": round(fwd, 2), "c1_train_value": round(c1_train, 2),
            "c1_fwd_value": round(c1_fwd, 2), "host_cpu_count": os.cpu_count(),
            "sample": f"oracle PyG-2.3.0-semantics GATModel (unfolded lin_edge, scatter softmax), "
                      f"{cfg['desc'].split(':')[0]} model at B={batch} and C1 at B=32, train "
                      f"(fwd+MSE+bwd+Adam) and forward, {wu} warm-up + {st} timed steps each "
                      f"(C1: 3 + 20), {cores} threads = the CPUs this process may run on "
                      f"(affinity / cgroup quota; {os.cpu_count()} on the host), "
                      f"{el:.1f}s, torch {torch.__version__} CPU, {_cpu_name()}"}


def step_roofline(cfg, train_gps: float, fwd_gps: float, dtype: str,
                  cov_var: bool = False) -> dict:
    """SURVEY §8(d) whole-step rule: graphs/s ÷ min(HBM-bound, compute-bound)
    graphs/s, from the algorithmic bytes and folded flops per graph (fwd);
    a train step counts 3x the forward flops.  ``cov_var``: the step's edge
    passes read edge_attr in the reference's covariance layout; the edge
    bytes they actually read per graph (cv_edge_bytes_per_graph) and the HBM
    bound under them are stated beside the rule's full-row figure."""
    n, S, H = cfg["n"], cfg["S"], cfg["heads"]
    F0, D, E0 = n * S, 3 * S, n * (n - 1)
    hidden = cfg["hidden"]
    L = len(hidden)
    flops, fin = 0.0, F0
    for l, C in enumerate(hidden):
        concat = cfg["concat"] and l < L - 1 and L > 1
        flops += 2 * n * fin * H * C + 2 * (E0 + n) * D * H + 4 * n * H * C + 2 * (E0 + n) * H * C
        fin = H * C if (concat and H > 1) else C
    out_ch = 1
    nbytes = 4.0 * (n * F0 + E0 * D + n * out_ch)
    peak_tf = BF16_MFMA_PEAK_TFLOPS if dtype == "bf16" else F32_MFMA_PEAK_TFLOPS
    hbm_gps = HBM_PEAK_GBS * 1e9 / nbytes
    fwd_bound = min(hbm_gps, peak_tf * 1e12 / flops)
    train_bound = min(hbm_gps, peak_tf * 1e12 / (3 * flops))
    res = {"bytes_per_graph": nbytes, "fwd_flops_per_graph": flops,
           "compute_peak_TFLOPs": peak_tf, "hbm_bound_gps": round(hbm_gps, 1),
           "fwd_bound_gps": round(fwd_bound, 1), "train_bound_gps": round(train_bound, 1),
           "fwd_frac": round(fwd_gps / fwd_bound, 4), "train_frac": round(train_gps / train_bound, 4)}
    if cov_var:
        ea_cv = cv_edge_bytes_per_graph(n, S)
        cv_bytes = 4.0 * (n * F0 + n * out_ch) + ea_cv
        res.update(edge_bytes_per_graph_rule=4.0 * E0 * D, edge_bytes_per_graph_read=ea_cv,
                   bytes_per_graph_cv=cv_bytes,
                   hbm_bound_gps_cv=round(HBM_PEAK_GBS * 1e9 / cv_bytes, 1),
                   edge_bytes_note="the step's edge passes read the covariance columns of the "
                                   "upper rows and one variance series per node (covariance "
                                   "layout); bytes_per_graph keeps SURVEY 8(d)'s full-row count")
    return res


def _ref_model(dev, cfg, args, world):
    """The model as the reference loop sees it: GATModel, wrapped in
    DistributedDataParallel at N > 1 (its gradient all-reduce is what makes
    the loop data-parallel; GATModel returns its gradients to autograd)."""
    model = build_model(dev, cfg).set_precision(args.precision)
    if world > 1:
        from torch.nn.parallel import DistributedDataParallel as DDP
        model = DDP(model, device_ids=[dev.index], broadcast_buffers=False)
    return model


def reference_loop_rate(dev, cfg, batches, args, world, canonical: bool = True,
                        fused_adam: bool = False, steps=None) -> float:
    """5_train_SpotV2Net.py:127, :142-160 as written, eager Python:
    ``torch.optim.Adam(model.parameters(), lr)`` (``fused_adam``: the one-word
    change ``fused=True``), per step a NEW batch object with a new edge_index,
    ``data = data.to(device)``, ``model(data)``, ``nn.MSELoss``, ``zero_grad``,
    ``backward``, ``step`` and the per-step ``loss.item()`` sync.

    ``batches``: the loader's batches, cycled.  Device-resident batches make
    ``.to(device)`` a no-op (the data already in HBM, as ``value`` assumes);
    host batches make it the reference's H2D copy of every batch (pageable
    memory, as its DataLoader yields without ``pin_memory``).  The batches
    carry what sv2n ``collate`` attaches to a batch of the reference's graphs:
    ``nodes_per_graph`` and, ``canonical``, the verified canonical edge order
    (False: the same batches without it, analysed on the device every step,
    block-layout kernels).  GATModel replays its forward and backward as
    hipGraphs from the second call of a signature on (graphed.py).  At N > 1
    the model is wrapped in DDP (one gradient all-reduce per step)."""
    from spotv2net_amd import Batch
    model = _ref_model(dev, cfg, args, world)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True) if fused_adam \
        else torch.optim.Adam(model.parameters(), lr=1e-3)
    crit = torch.nn.MSELoss()
    extra = {"canonical_edges": True} if canonical else {}
    loader = [Batch(x=b.x, edge_index=b.edge_index, edge_attr=b.edge_attr, y_x=b.y_x,
                    batch=b.batch, ptr=b.ptr, nodes_per_graph=cfg["n"], **extra)
              for b in batches]
    it = [0]

    def step():
        src = loader[it[0] % len(loader)]
        it[0] += 1
        data = src.to(dev)
        if data.edge_index is src.edge_index:   # device-resident: a DataLoader still
            data.edge_index = src.edge_index.clone()   # yields a new edge_index tensor
        y_x_hat = model(data)
        loss = crit(y_x_hat, data.y_x)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss.item()

    steps = steps or args.steps
    for _ in range(max(3, args.warmup)):
        step()
    el = max_over_ranks(time_replays(step, steps), dev)
    return world * args.batch * steps / el


def run_c3_loop(args, dev, cfg) -> dict:
    """C3 as BASELINE.json states it: config/GNN_param.yaml's model and
    hyper-parameters (S 42, hidden [500], 6 heads, dropout 0.1, Adam 1e-3,
    batch 128, split 0.8) over the full training loop of 5_train_SpotV2Net.py
    (train pass with shuffling + test pass per epoch) on 2,157 windows — the
    count CovarianceLaggedDataset yields from 10,556 matrices after the
    [8357:] cut (utils/dataset.py:200, :288).  Timed: ``--epochs`` epochs
    after ``--warmup-epochs``, in bf16 mode and, for comparison, fp32 mode."""
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    from spotv2net_amd.train import Fit
    V, W = synthetic_series(10556, cfg["n"], seed=1234, device=dev)
    ds = WindowDataset(V, W, cfg["S"], cut=8357)
    from spotv2net_amd import stack

    def one(prec):
        model = build_model(dev, cfg).set_precision(prec)
        f = Fit(model, ds, args.batch, lr=1e-3, split=0.8,
                generator=torch.Generator().manual_seed(5154), use_graph=not args.no_graph)
        for _ in range(args.warmup_epochs):
            f.run_epoch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.epochs):
            rec = f.run_epoch()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        steps = args.epochs * (-(-f.n_train // args.batch))
        return f, {"graphs_per_s": args.epochs * len(ds) / el,
                   "train_graphs_per_s_upper": args.epochs * f.n_train / el,
                   "seconds": el, "train_steps": steps, "epoch_record": rec,
                   "history": f.history, "cov_var_only_gather": f._cv_only,
                   "cov_var_edge_passes": bool(stack.LAST_PATH.get("cov_var"))}

    out = {}
    precs = [args.precision] + ([] if args.no_compare else
                                ["f32" if args.precision == "bf16" else "bf16"])
    for prec in precs:
        f, out[prec] = one(prec)
    variants = {}
    if not args.no_compare:
        # what the line owes to the edge features' covariance layout: the same
        # loop (a) gathering every edge_attr column (the passes unchanged), and
        # (b) through the generic edge passes, which read every edge row
        old_only, old_cv = stack.cov_var_edges_only, stack.COV_VAR_EDGES
        try:
            stack.cov_var_edges_only = lambda *a: False
            variants["full_gather"] = one(args.precision)[1]
            stack.COV_VAR_EDGES = "off"
            variants["generic_edges"] = one(args.precision)[1]
        finally:
            stack.cov_var_edges_only, stack.COV_VAR_EDGES = old_only, old_cv
    return {"windows": len(ds), "n_train": f.n_train, "n_test": f.n_test, "runs": out,
            "variants": variants}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="graphs per GPU (config default)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches (no hipGraph)")
    ap.add_argument("--cpu-batch", type=int, default=None,
                    help="graphs per CPU-baseline step (default: the benched batch, at most "
                         "445,440 edges = 512 C2 graphs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-table", action="store_true")
    ap.add_argument("--no-rotating", action="store_true",
                    help="skip value_rotating (the step over rotating distinct batches)")
    ap.add_argument("--rotate", type=int, default=3,
                    help="distinct device-resident batches value_rotating cycles through")
    ap.add_argument("--no-ref-loop", action="store_true",
                    help="skip the eager reference-loop (new batch per step) measurement")
    ap.add_argument("--precision", default=None, choices=("f32", "bf16"),
                    help="execution mode (default: f32; bf16 for --config c3)")
    ap.add_argument("--epochs", type=int, default=3, help="c3: timed epochs (yaml num_epochs)")
    ap.add_argument("--warmup-epochs", type=int, default=1, help="c3: untimed epochs")
    ap.add_argument("--no-compare", action="store_true",
                    help="c3: skip the run in the other precision")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="process group at N > 1: nccl (= RCCL over xGMI, one GPU per rank) "
                         "or gloo (host-staged; e.g. several ranks sharing one GPU)")
    args = ap.parse_args(argv)
    if args.precision is None:
        args.precision = "bf16" if args.config == "c3" else "f32"

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "gloo":
        # ranks may share a GPU (the -m gpu test runs two on the box's one card)
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from spotv2net_amd import synthetic_batch
    from spotv2net_amd.train import ForwardStep, TrainStep, broadcast_params_

    cfg = CONFIGS[args.config]
    if args.batch is None:
        args.batch = cfg["batch"]
    if args.config == "c3" and world == 1:
        return main_c3(args, dev, cfg)
    model = build_model(dev, cfg).set_precision(args.precision)
    if world > 1:  # identical replicas: broadcast rank 0's weights
        broadcast_params_(model, 0)
    data = synthetic_batch(args.batch, cfg["S"], n=cfg["n"], seed=1234 + rank, device=dev)

    step = TrainStep(model, data, lr=1e-3, use_graph=not args.no_graph)
    for _ in range(args.warmup):
        step()
    el = time_replays(step, args.steps)
    el = max_over_ranks(el, dev)
    value = world * args.batch * args.steps / el
    loss = float(step.loss.item())

    # the timed step's parameters, checked before anything else trains a copy
    replicas_ok = replicas_identical(step.flat_params, dev) if world > 1 else None

    # the batch's edge_attr is in the reference's covariance layout (written
    # by window_batch, layout.mark_cov_var), so the step's edge passes read
    # ≈ 1/6 of it; the same step over every edge row, for comparison (on a
    # copy of the model: TrainStep re-flattens the parameters it trains)
    from spotv2net_amd import stack
    cov_var = bool(stack.LAST_PATH.get("cov_var"))
    value_generic = None
    if cov_var:
        old = stack.COV_VAR_EDGES
        stack.COV_VAR_EDGES = "off"
        try:
            gstep = TrainStep(copy.deepcopy(model), data, lr=1e-3, use_graph=not args.no_graph)
            for _ in range(args.warmup):
                gstep()
            gel = max_over_ranks(time_replays(gstep, args.steps), dev)
            value_generic = world * args.batch * args.steps / gel
            del gstep
        finally:
            stack.COV_VAR_EDGES = old

    # a new batch every step, as the reference's loop (5_train_SpotV2Net.py:142-143):
    # ROTATE distinct device-resident batches (more bytes than the 256 MB
    # Infinity Cache holds, so no step finds its inputs left there by the
    # previous one), one captured graph per batch over the same parameters
    rot = None
    if not args.no_rotating and not args.no_graph:
        rot_batches = [data] + [synthetic_batch(args.batch, cfg["S"], n=cfg["n"],
                                                seed=7000 + 100 * rank + i, device=dev)
                                for i in range(args.rotate - 1)]
        rot_bytes = sum(b.x.numel() * 4 + b.edge_attr.numel() * 4 for b in rot_batches)
        rstep = TrainStep(copy.deepcopy(model), rot_batches[0], lr=1e-3)
        for b in rot_batches[1:]:
            rstep.add_shape(b)
        k = len(rot_batches)
        it = [0]

        def rstep_call():
            rstep(it[0] % k)
            it[0] += 1

        for _ in range(max(args.warmup, k)):
            rstep_call()
        rel = max_over_ranks(time_replays(rstep_call, args.steps), dev)
        rot = {"value": world * args.batch * args.steps / rel, "batches": k,
               "bytes_per_batch": rot_bytes / k, "bytes_total": rot_bytes,
               "cov_var": bool(stack.LAST_PATH.get("cov_var"))}
        del rstep, rot_batches

    ref = {}
    if not args.no_ref_loop:
        # the loader's batches: two distinct device-resident ones, alternating
        # (new contents every step at recycled addresses)
        dev_batches = [data, synthetic_batch(args.batch, cfg["S"], n=cfg["n"],
                                             seed=5678 + rank, device=dev)]
        ref["ref_loop_graphs_per_s"] = reference_loop_rate(dev, cfg, dev_batches, args, world)
        ref["ref_loop_fused_adam_graphs_per_s"] = reference_loop_rate(
            dev, cfg, dev_batches, args, world, fused_adam=True)
        ref["ref_loop_block_layout_graphs_per_s"] = reference_loop_rate(
            dev, cfg, dev_batches, args, world, canonical=False)
        del dev_batches
        # literal: host batches, the H2D copy of each inside the step
        host_batches = [synthetic_batch(args.batch, cfg["S"], n=cfg["n"], seed=9100 + 10 * rank + i)
                        for i in range(3)]
        ref["ref_loop_literal_graphs_per_s"] = reference_loop_rate(
            dev, cfg, host_batches, args, world, steps=min(args.steps, 20))
        del host_batches
    model.eval()
    fstep = ForwardStep(model, data, use_graph=not args.no_graph)
    for _ in range(max(1, args.warmup)):
        fstep()
    fel = max_over_ranks(time_replays(fstep, args.steps), dev)
    fwd_value = world * args.batch * args.steps / fel
    model.train()

    result = None
    if rank == 0:
        table = {}
        roof = None
        if not args.no_kernel_table and args.config == "c2":
            table = kernel_table(model, data)
            kname, roof = roofline_entry(table)
            roof["traffic"] = load_traffic(kname)
        elif not args.no_kernel_table and args.config == "c5":
            table = kernel_table_tiled(model, data, cfg)
            kname, roof = roofline_entry(table)
            roof["traffic"] = load_traffic("c5:" + kname)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            # the benched batch (C2: 512 graphs); at most as many
            # edges as 512 C2 graphs for the other configs
            cpu_batch = max(1, min(args.cpu_batch or args.batch, args.batch,
                                   445440 // (cfg["n"] * (cfg["n"] - 1))))
            cpu = cpu_baseline(model, cfg, cpu_batch)
        result = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "graphs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (standardized symmetric vol / vol-of-vol matrices, "
                    "CovarianceLaggedDataset layout), device-resident, random-init weights",
            "config": {"workload": cfg["desc"], "name": args.config,
                       "graphs_per_gpu": args.batch, "global_batch": args.batch * world,
                       "parallelism": f"dp{world}", "hipgraph": not args.no_graph},
            "edge_features": ("reference covariance layout [cov | var_src | var_dst] per lag "
                              "(utils/dataset.py:228-243), read as such by the edge passes"
                              if cov_var else "generic rows"),
            "value_generic_edges": (round(value_generic, 1) if value_generic else None),
            "value_rotating": (round(rot["value"], 1) if rot else None),
            "rotating": ({k: v for k, v in rot.items() if k != "value"} if rot else None),
            "step_edge_passes": ("edge_logits_fwd_cv / edge_logits_bwd_cv" if cov_var
                                 else "edge_logits_fwd / edge_logits_bwd"),
            "fwd_graphs_per_s": round(fwd_value, 1),
            **{k: round(v, 1) for k, v in ref.items()},
            "ref_loop_is": "5_train_SpotV2Net.py:142-160 unchanged (new batch per step, "
                           "data.to(device), MSELoss, zero_grad, backward, torch.optim.Adam, "
                           "loss.item()); DDP-wrapped at N > 1. ref_loop: two device-resident "
                           "batches alternating, default Adam; fused_adam: Adam(fused=True); "
                           "block_layout: no canonical mark; literal: pageable host batches, "
                           "the H2D copy inside the step",
            "replicas_bit_identical": replicas_ok,
            "backend": args.backend if world > 1 else None,
            "step_roofline": step_roofline(cfg, value, fwd_value, args.precision, cov_var),
            "final_loss": loss,
            "roofline": roof,
            "cpu_baseline": cpu,
            "speedup_vs_cpu": (round(value / cpu["value"], 1) if cpu else None),
            "kernels": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv)
                            for kk, vv in v.items()
                            if kk in ("avg_us", "avg_us_back_to_back", "tflops", "gbs", "bound")}
                        for k, v in table.items()},
            "peaks_assumed": {"hbm_GBs": HBM_PEAK_GBS, "f32_mfma_TFLOPs": F32_MFMA_PEAK_TFLOPS,
                              "bf16x3_f32eq_TFLOPs": BF16X3_PEAK_TFLOPS},
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main_c3(args, dev, cfg):
    res = run_c3_loop(args, dev, cfg)
    main_run = res["runs"][args.precision]
    value = main_run["graphs_per_s"]
    cpu = None
    roof, table = None, {}
    if not args.no_kernel_table:
        table = kernel_table_c3(build_model(dev, cfg), cfg, args.precision)
        kname, roof = roofline_entry(table)
        roof["traffic"] = load_traffic(f"c3_{args.precision}:" + kname)
    if not args.no_cpu_baseline:
        model = build_model(dev, cfg)
        cpu = cpu_baseline(model, cfg, min(args.cpu_batch or 16, 16))
    result = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "graphs/s",
        "n_gpus": 1,
        "steps": main_run["train_steps"],
        "warmup": args.warmup_epochs,
        "ms_per_step": round(main_run["seconds"] / main_run["train_steps"] * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic standardized vol / vol-of-vol series of 10,556 matrices on the "
                "device, windows gathered on the device per batch; random-init weights",
        "config": {"workload": cfg["desc"] + "; full train loop (train + test pass per epoch, "
                   "shuffle, ragged last batch) over 2,157 windows, split 0.8",
                   "name": "c3", "graphs_per_gpu": args.batch, "global_batch": args.batch,
                   "parallelism": "dp1", "hipgraph": not args.no_graph,
                   "epochs_timed": args.epochs},
        "value_is": "windows processed (train + test) per second over whole epochs",
        "edge_features": ("reference covariance layout [cov | var_src | var_dst] per lag "
                          "(utils/dataset.py:228-243): the window gather writes only the "
                          "columns the covariance-layout edge passes read "
                          "(sv2n_window_gather_cv)" if main_run["cov_var_only_gather"] else
                          ("reference covariance layout, full gather"
                           if main_run["cov_var_edge_passes"] else "generic rows")),
        "value_full_gather": (round(res["variants"]["full_gather"]["graphs_per_s"], 1)
                              if "full_gather" in res["variants"] else None),
        "value_generic_edges": (round(res["variants"]["generic_edges"]["graphs_per_s"], 1)
                                if "generic_edges" in res["variants"] else None),
        "c3_loop": {k: {kk: (round(vv, 2) if isinstance(vv, float) else vv)
                        for kk, vv in v.items() if kk != "history"}
                    for k, v in res["runs"].items()},
        "loss_curves": {k: [(round(r["train_loss"], 6), round(r["test_loss"], 6))
                            for r in v["history"]] for k, v in res["runs"].items()},
        "step_roofline": step_roofline(cfg, main_run["train_graphs_per_s_upper"], value,
                                       args.precision),
        "roofline": roof,
        "kernels": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv)
                        for kk, vv in v.items()
                            if kk in ("avg_us", "avg_us_back_to_back", "tflops", "gbs", "bound")}
                    for k, v in table.items()},
        "cpu_baseline": cpu,
        "peaks_assumed": {"hbm_GBs": HBM_PEAK_GBS, "f32_mfma_TFLOPs": F32_MFMA_PEAK_TFLOPS,
                          "bf16_mfma_TFLOPs": BF16_MFMA_PEAK_TFLOPS,
                          "bf16x3_f32eq_TFLOPs": BF16X3_PEAK_TFLOPS},
    }
    print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
