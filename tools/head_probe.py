"""Round 5 probe: k_head_mse_train_w launch time against the row count
(C 500, out 1 — the C3 head), each N replayed as a hipGraph of 50 launches.
A flat curve at small N is the partial reduction's fixed latency."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spotv2net_amd import library  # noqa: F401


def main():
    dev = torch.device("cuda:0")
    C = 500
    w = torch.randn(1, C, device=dev) * 0.05
    b = torch.zeros(1, device=dev)
    for N in (240, 960, 3840, 15360, 61440):
        x = torch.randn(N, C, device=dev)
        t = torch.randn(N, device=dev)
        gw = torch.zeros(1, C, device=dev)
        gb = torch.zeros(1, device=dev)
        ls = torch.zeros((), device=dev)
        op = torch.ops.sv2n.head_mse_train
        for _ in range(3):
            op(x, w, b, t, gw, gb, ls)
        torch.cuda.synchronize()
        s = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(50):
                op(x, w, b, t, gw, gb, ls)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 200
        mb = 2 * N * C * 4 / 1e6
        print(f"N {N:6d}  {us:7.2f} us/launch  {mb:7.2f} MB  {mb / us:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
