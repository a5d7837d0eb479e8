"""Window gather (sv2n_window.hip k_window_rows) timed alone on BASELINE C3's
shape: 128 random windows of S 42 over n 30, per output variant, beside a
device copy of the same bytes.  Usage: python tools/window_micro.py"""
import sys

import torch

sys.path.insert(0, ".")


def main():
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    dev = torch.device("cuda:0")
    V, W = synthetic_series(10556, 30, seed=1234, device=dev)
    ds = WindowDataset(V, W, 42, cut=8357)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    g = torch.Generator().manual_seed(0)
    idx = torch.randperm(len(ds), generator=g)[:B].to(dev)
    variants = {
        "cv+twin_only": dict(bf16_x=True, cov_var_only=True, twin_only=True),
        "cv+twin+x": dict(bf16_x=True, cov_var_only=True),
        "full+twin+x": dict(bf16_x=True),
        "full+x": dict(),
    }
    reps = 200
    for name, kw in variants.items():
        b = ds.empty_batch(B, **kw)
        for _ in range(10):
            ds.fill(b, idx)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(reps):
            ds.fill(b, idx)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / reps
        print(f"{name:14s} {us:8.2f} us/launch", flush=True)
    nbytes = 19 << 20
    a = torch.empty(nbytes // 4, device=dev)
    c = torch.empty_like(a)
    for _ in range(10):
        c.copy_(a)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        c.copy_(a)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / reps
    print(f"copy 19 MiB    {us:8.2f} us ({2 * nbytes / us / 1e6:.0f} GB/s r+w)", flush=True)


if __name__ == "__main__":
    main()
