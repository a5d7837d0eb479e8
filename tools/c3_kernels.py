"""Per-kernel timings of the C3 training step's non-GEMM launches (the yaml
model: F 1260, 6 heads x 500, mean, B 128), HIP events on the launch stream:
weight prep, window gather, fused head + MSE, weight-gradient node (GEMM +
reduce + epilogue + att kernel) and its parts.

usage: python tools/c3_kernels.py [--precision bf16|f32] [--reps 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps, stream):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-diag", action="store_true",
                    help="window gather reading the diagonal from volvol (no [T][n] copy)")
    args = ap.parse_args()
    from spotv2net_amd import GATModel, WindowDataset, ops
    from spotv2net_amd.data import synthetic_series
    from spotv2net_amd.stack import layer_params  # noqa: F401
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    torch.manual_seed(5154)
    m = GATModel(1260, 126, 6, 1, [500], dropout=0.1, concat_heads=True).to(dev)
    conv = m.gat_layers[0]
    bf16 = args.precision == "bf16"
    out = {}
    c = conv
    prep_args = ([c.lin_src.weight], [c.att_src], [c.att_dst], [c.lin_edge.weight], [c.att_edge],
                 [6], [500], 8, [False], True, bf16)
    out["prep_fwd_all"] = timeit(lambda: torch.ops.sv2n.gat_prep(*prep_args), args.reps, stream)
    V, W = synthetic_series(10556, 30, seed=1234, device=dev)
    ds = WindowDataset(V, W, 42, cut=8357)
    if args.no_diag:
        ds.diag = None
    b = ds.empty_batch(128)
    idx = torch.randperm(len(ds))[:128].to(dev)
    out["window_gather"] = timeit(lambda: ds.fill(b, idx), args.reps, stream)
    x = torch.randn(3840, 500, device=dev)
    y = torch.randn(3840, device=dev)
    gw, gb = torch.zeros_like(m.linear.weight), torch.zeros_like(m.linear.bias)
    out["head_mse_train"] = timeit(lambda: torch.ops.sv2n.head_mse_train(
        x, m.linear.weight.detach(), m.linear.bias.detach(), y, gw, gb), args.reps, stream)
    xin = b.x
    ldx = (3000 + 12 + 3) // 4 * 4
    dxs = torch.randn(3840, ldx, device=dev) * 1e-3
    dbp = torch.randn(128, 500, device=dev)
    gW = torch.zeros(3000, 1260, device=dev)
    ga, gd, gbb = (torch.zeros(6, 500, device=dev) for _ in range(3))
    gbb = torch.zeros(500, device=dev)
    out["wgrad_node"] = timeit(lambda: torch.ops.sv2n.gat_wgrad(
        xin, dxs, c.lin_src.weight.detach(), c.att_src.detach(), c.att_dst.detach(), dbp, 6, 500,
        bf16, gW, ga, gd, gbb), args.reps, stream)
    out["wgrad_bias_only"] = timeit(lambda: torch.ops.sv2n.gat_wgrad(
        None, dxs, c.lin_src.weight.detach(), c.att_src.detach(), c.att_dst.detach(), dbp, 6, 500,
        bf16, None, None, None, gbb), args.reps, stream)
    out["wgrad_no_att"] = timeit(lambda: torch.ops.sv2n.gat_wgrad(
        xin, dxs, c.lin_src.weight.detach(), c.att_src.detach(), c.att_dst.detach(), dbp, 6, 500,
        bf16, gW, None, None, gbb), args.reps, stream)
    planes = ops.weight_planes(c.projection_weight().detach().contiguous(), False)
    out["project"] = timeit(lambda: torch.ops.sv2n.project(xin, planes, c.projection_weight()
                                                           .detach().contiguous(), False, bf16),
                            args.reps, stream)
    print(args.precision, " ".join(f"{k} {v:.1f}" for k, v in out.items()), flush=True)


if __name__ == "__main__":
    main()
