"""Phase timeline of the canonical attention kernels (diagnostic build).

Build:  make STAMPS=1 LIB=spotv2net_amd/libsv2n_stamps.so BUILD=build/stamps
Run:    SV2N_LIB=spotv2net_amd/libsv2n_stamps.so python tools/stamps.py [B | c3 | l1]

Launches the C2 layer-0 attention forward and backward once each (after a
warm-up) through the C-ABI and prints, per phase, the median and max over
waves of the s_memtime deltas (shader cycles) plus the wall span of the
launch from s_memrealtime (10 ns ticks): where a workgroup's time goes."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from spotv2net_amd import ops, synthetic_batch  # noqa: E402


def read(lib, nwg):
    buf = (ctypes.c_ulonglong * (4096 * 4 * 16))()
    torch.cuda.synchronize()
    assert lib.sv2n_diag_stamps(buf, 4096 * 4 * 16) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4, 16)[:nwg].astype(np.int64)


def report(name, st, phases, rt0, rt1):
    print(f"== {name}")
    span = (st[:, :, rt1].max() - st[:, :, rt0].min()) * 10 / 1000.0
    life = (st[:, :, rt1] - st[:, :, rt0]) * 10 / 1000.0
    starts = (st[:, :, rt0] - st[:, :, rt0].min()) * 10 / 1000.0
    print(f"   launch span {span:.1f} us; wave life median {np.median(life):.1f} max {life.max():.1f} us;"
          f" start offsets median {np.median(starts):.1f} max {starts.max():.1f} us")
    for a, b, label in phases:
        d = st[:, :, b] - st[:, :, a]
        print(f"   {label:28s} median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}  max {d.max():8.0f} cyc")


def main_c3(B=128):
    """C3 shape: 6 heads x 500, head mean, F 1260 (ldx 3012), split launches."""
    dev = torch.device("cuda", 0)
    lib = ops._lib.load()
    lib.sv2n_diag_stamps.restype = ctypes.c_int
    lib.sv2n_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    sh = torch.cuda.current_stream(dev).cuda_stream
    n, H, C, ldx = 30, 6, 500, 3012
    torch.manual_seed(0)
    xs = torch.randn(B * n, ldx, device=dev) * 0.1
    ae = torch.randn(B * n * (n - 1), H, device=dev)
    bias = torch.randn(C, device=dev)
    y = torch.empty(B * n, C, device=dev)
    ps = torch.empty(B, H, 32, 32, device=dev)
    dy = torch.randn_like(y)
    dxs = torch.empty_like(xs)
    dae = torch.empty_like(ae)
    dbp = torch.empty(B, C, device=dev)

    def fwd():
        assert lib.sv2n_gat_attn_fwd(xs.data_ptr(), ldx, ae.data_ptr(), 1, None, bias.data_ptr(),
                                     None, 1.0, y.data_ptr(), ps.data_ptr(), None, 0.0, None, B,
                                     n, H, C, 0, 1, 0.2, sh) == 0

    def bwd():
        assert lib.sv2n_gat_attn_bwd(dy.data_ptr(), y.data_ptr(), xs.data_ptr(), ldx,
                                     ps.data_ptr(), None, 1.0, None, 0.0, None, dxs.data_ptr(),
                                     dae.data_ptr(), 1, dbp.data_ptr(), B, n, H, C, 0, 1, 0.2,
                                     sh) == 0

    for _ in range(5):
        fwd()
        bwd()
    fwd()
    report("fwd C3", read(lib, B * 4),
           [(1, 2, "prologue loads -> AE staged"), (2, 3, "softmax"), (3, 4, "barrier"),
            (4, 5, "aggregation + stores")], 0, 6)
    bwd()
    report("bwd C3", read(lib, B * 6),
           [(1, 2, "prologue -> chunk 0 wait"), (2, 3, "stage chunk 0"), (3, 4, "compute 0 + wait 1"),
            (4, 5, "stage chunk 1"), (5, 6, "compute 1 + wait 2"), (6, 7, "stage chunk 2"),
            (7, 8, "compute 2 + wait 3"), (8, 9, "stage chunk 3"), (9, 10, "compute 3 + softmax bwd"),
            (10, 11, "barrier"), (11, 12, "d ae + tail")], 0, 13)


def main(B=512):
    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS["c2"]
    model = bench.build_model(dev, cfg)
    data = synthetic_batch(B, cfg["S"], n=cfg["n"], seed=1234, device=dev)
    lib = ops._lib.load()
    lib.sv2n_diag_stamps.restype = ctypes.c_int
    lib.sv2n_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    sh = torch.cuda.current_stream(dev).cuda_stream
    n, H = bench.N_NODES, bench.HEADS
    conv0 = model.gat_layers[0]
    with torch.no_grad():
        W0 = conv0.projection_weight().contiguous()
    x0 = data.x
    N0 = x0.shape[0]
    xs0 = ops.gemm_f32(x0, True, W0, True, N0, W0.shape[0], x0.shape[1])
    ae = torch.randn(B * n * (n - 1), H, device=dev)
    y0 = torch.empty(N0, conv0.out_dim, device=dev)
    ps0 = torch.empty(B, H, 32, 32, device=dev)
    dy0 = torch.randn_like(y0)
    dxs0 = torch.empty_like(xs0)
    dae0 = torch.empty_like(ae)
    dbp = torch.empty(B, conv0.out_dim, device=dev)

    def fwd():
        lib.sv2n_gat_attn_fwd(xs0.data_ptr(), xs0.stride(0), ae.data_ptr(), 1, None,
                              conv0.bias.data_ptr(), None, 1.0, y0.data_ptr(), ps0.data_ptr(),
                              None, 0.0, None, B, n, H, conv0.out_channels, 1, 1, 0.2, sh)

    def bwd():
        lib.sv2n_gat_attn_bwd(dy0.data_ptr(), y0.data_ptr(), xs0.data_ptr(), xs0.stride(0),
                              ps0.data_ptr(), None, 1.0, None, 0.0, None, dxs0.data_ptr(),
                              dae0.data_ptr(),
                              1, dbp.data_ptr(), B, n, H, conv0.out_channels, 1, 1, 0.2, sh)

    for _ in range(5):
        fwd()
        bwd()
    fwd()
    report("fwd L0", read(lib, B),
           [(1, 2, "prologue loads -> AE staged"), (2, 3, "softmax"), (3, 4, "barrier"),
            (4, 5, "aggregation + stores")], 0, 6)
    bwd()
    report("bwd L0", read(lib, B),
           [(1, 2, "prologue -> chunk 0 wait"), (2, 3, "stage chunk 0"), (3, 4, "compute 0 + wait 1"),
            (4, 5, "stage chunk 1"), (5, 6, "compute 1 + wait 2"), (6, 7, "stage chunk 2"),
            (7, 8, "compute 2 + wait 3"), (8, 9, "stage chunk 3"), (9, 10, "compute 3 + softmax bwd"),
            (10, 11, "barrier"), (11, 12, "d ae + tail")], 0, 13)


def main_l1(B=512):
    """The C2 model's last layer with the output head + MSE fused in
    (k_fwd<HEAD>): phases up to the aggregation, then the head's output /
    residual, the dZ stores and the per-graph partials."""
    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS["c2"]
    model = bench.build_model(dev, cfg)
    lib = ops._lib.load()
    lib.sv2n_diag_stamps.restype = ctypes.c_int
    lib.sv2n_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    n, H = bench.N_NODES, bench.HEADS
    conv1 = model.gat_layers[1]
    C, ldx = conv1.out_channels, (H * conv1.out_channels + 2 * H + 3) // 4 * 4
    torch.manual_seed(0)
    N = B * n
    xs = torch.randn(N, ldx, device=dev) * 0.1
    ae = torch.randn(B * n * (n - 1), H, device=dev)
    tgt = torch.randn(N, device=dev)
    gw = torch.zeros_like(model.linear.weight)
    gb = torch.zeros_like(model.linear.bias)

    def fwd():
        torch.ops.sv2n.gat_attn_fwd_head_mse(
            xs, ae, None, conv1.bias, None, 1.0, None, 0.0, model.linear.weight.view(-1),
            model.linear.bias, tgt, gw, gb, B, n, H, C, bool(conv1.concat), 1, 0.2, True)

    for _ in range(5):
        fwd()
    fwd()
    report("fwd L1 + head + MSE", read(lib, B),
           [(1, 2, "prologue loads -> AE staged"), (2, 3, "softmax"), (3, 4, "barrier"),
            (4, 7, "aggregation + head output"), (7, 8, "dZ stores"), (8, 5, "partials")], 0, 6)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "l1":
        main_l1()
    elif len(sys.argv) > 1 and sys.argv[1] == "c3":
        main_c3()
    else:
        main(int(sys.argv[1]) if len(sys.argv) > 1 else 512)
