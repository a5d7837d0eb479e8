"""Timing ablations of the edge-fused attention forward at the C5 layer-0
shape (B 1024, n 256, D 12, 8 heads x 16): the product kernel and variants
built with parts removed (SV2N_FATTN_ABLATE, sv2n_attn_fused.hip).  Build the
variants on the CPU first:  python tools/fattn_ablate.py --build
Timings only: the variants compute wrong results by construction."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "spotv2net_amd", "csrc", "sv2n_attn_fused.hip")
# (round 3 replaced the backward by the head-per-wave kernel; its round-2
# ablations 4-6 belonged to the three-phase kernel and are gone)
VARIANTS = {0: "product", 1: "no edge_attr loads", 2: "no softmax/MFMA", 3: "no logit math",
            7: "bwd: product"}


def so(k):
    return os.path.join(ROOT, "tools", f"fattn_abl{k}.so")


def build():
    for k in VARIANTS:
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "--offload-arch=gfx950", "-I" + os.path.join(ROOT, "include"),
                        f"-DSV2N_FATTN_ABLATE={k}", SRC, "-o", so(k)], check=True)


def run():
    import torch
    dev = torch.device("cuda", 0)
    B, n, D, H, C = int(os.environ.get("B", 1024)), 256, 12, 8, 16
    N, E = B * n, B * n * (n - 1)
    ldx = (H * C + 2 * H + 3) // 4 * 4
    g = torch.Generator(device=dev).manual_seed(0)
    xs = torch.randn(N, ldx, device=dev, generator=g)
    ea = torch.randn(E, D, device=dev, generator=g)
    wf = torch.randn(D, 32, device=dev, generator=g) * 0.1
    y = torch.empty(N, H * C, device=dev)
    agg = torch.empty(N, H * C, device=dev)
    st = torch.empty(N, 4 * H, device=dev)
    bias = torch.zeros(H * C, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    dy = torch.randn(N, H * C, device=dev, generator=g)
    dxs = torch.empty(N, ldx, device=dev)
    NS = (n + 31) // 32
    dbp = torch.empty(B * NS, H * C, device=dev)
    dwf = torch.zeros(D, 32, device=dev)
    for k, what in VARIANTS.items():
        lib = ctypes.CDLL(so(k))
        if k >= 4:
            fb = lib.sv2n_gat_attn_fused_bwd
            fb.restype = ctypes.c_int
            P, I, F, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64
            fb.argtypes = [P, P, P, P, P, I, P, I, P, I, I, P, P, F, P, P, P, P, L, L, I, I, I, I,
                           I, F, P]
            lib.sv2n_gat_attn_fused_bwd_workspace.restype = L
            lib.sv2n_gat_attn_fused_bwd_workspace.argtypes = [L, I, I, I, I]
            wsn = lib.sv2n_gat_attn_fused_bwd_workspace(B, n, H, C, D)
            ws = torch.empty(wsn, device=dev)

            def call():
                rc = fb(dy.data_ptr(), y.data_ptr(), agg.data_ptr(), st.data_ptr(), xs.data_ptr(),
                        ldx, ea.data_ptr(), D, wf.data_ptr(), 32, 0, None, None, 1.0,
                        dxs.data_ptr(), dbp.data_ptr(), dwf.data_ptr(), ws.data_ptr(), wsn, B, n,
                        H, C, 1, 1, 0.2, stream)
                assert rc == 0, rc
        else:
            call = None
        f = lib.sv2n_gat_attn_fused_fwd
        f.restype = ctypes.c_int
        P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        f.argtypes = [P, I, P, I, P, I, I, P, P, P, F, P, P, P, ctypes.c_int64, I, I, I, I, I, F, P]

        def fcall():
            rc = f(xs.data_ptr(), ldx, ea.data_ptr(), D, wf.data_ptr(), 32, 0, None,
                   bias.data_ptr(), None, 1.0, y.data_ptr(), agg.data_ptr(), st.data_ptr(), B, n,
                   H, C, 1, 1, 0.2, stream)
            assert rc == 0, rc
        fcall()  # a training forward fills y / agg / stats
        call = call or fcall
        for _ in range(3):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        print(f"variant {k} ({what}): {us:9.1f} us  ({4 * E * D / us / 1e3:7.0f} GB/s of edge_attr)",
              flush=True)


if __name__ == "__main__":
    build() if "--build" in sys.argv else run()
