"""Host-side profile (cProfile) of the reference-shaped loop
(5_train_SpotV2Net.py:142-160) at C2: which Python calls the GPU waits for.
usage: python tools/ref_loop_cprofile.py [--steps 300] [--canonical 1]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--canonical", type=int, default=1)
    args = ap.parse_args()
    from spotv2net_amd import Batch, GATModel, synthetic_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(5154)
    model = GATModel(1260, 126, 4, 1, [100, 50], concat_heads=True).to(dev)
    data = synthetic_batch(512, 42, seed=1234, device=dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    crit = torch.nn.MSELoss()
    extra = {"canonical_edges": True} if args.canonical else {}

    def step():
        b = Batch(x=data.x, edge_index=data.edge_index.clone(), edge_attr=data.edge_attr,
                  y_x=data.y_x, batch=data.batch, ptr=data.ptr, nodes_per_graph=30, **extra)
        loss = crit(model(b), b.y_x)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss.item()

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    el = time.perf_counter() - t0
    print(f"plain: {el / args.steps * 1e6:.1f} us/step, {512 * args.steps / el:.0f} graphs/s")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        step()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(45)


if __name__ == "__main__":
    main()
