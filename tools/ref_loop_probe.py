"""Where the reference-shaped loop (5_train_SpotV2Net.py:142-160: new Batch per
step, model(b), nn.MSELoss, zero_grad, backward, torch.optim.Adam step,
loss.item()) spends its time on the GPU box: host time per phase (no syncs
inside the step), whole-step wall time, and the same loop with the GPU work
drained before each phase (the GPU-side time of that phase).

usage: python tools/ref_loop_probe.py [--steps 50] [--batch 512]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--fused-adam", type=int, default=1)
    ap.add_argument("--modes", default="free,drained")
    ap.add_argument("--canonical", type=int, default=0,
                    help="mark the batch canonical as collate() does for canonical edge order")
    args = ap.parse_args()
    from spotv2net_amd import Batch, GATModel, synthetic_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(5154)
    model = GATModel(1260, 126, 4, 1, [100, 50], concat_heads=True).to(dev)
    data = synthetic_batch(args.batch, 42, seed=1234, device=dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=bool(args.fused_adam))
    crit = torch.nn.MSELoss()
    ph = {k: 0.0 for k in ("batch", "fwd", "loss", "zero", "bwd", "opt", "item")}

    def step(sync_each=False):
        t = [time.perf_counter()]

        def mark():
            if sync_each:
                torch.cuda.synchronize()
            t.append(time.perf_counter())
        b = Batch(x=data.x, edge_index=data.edge_index.clone(), edge_attr=data.edge_attr,
                  y_x=data.y_x, batch=data.batch, ptr=data.ptr, nodes_per_graph=30)
        if args.canonical:
            b.canonical_edges = True
        mark()
        out = model(b)
        mark()
        loss = crit(out, b.y_x)
        mark()
        opt.zero_grad()
        mark()
        loss.backward()
        mark()
        opt.step()
        mark()
        v = loss.item()
        mark()
        return t, v

    for _ in range(5):
        step()
    for mode in [m == "drained" for m in args.modes.split(",")]:
        acc = dict.fromkeys(ph, 0.0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            t, _ = step(sync_each=mode)
            for k, a, b in zip(acc, t[:-1], t[1:]):
                acc[k] += b - a
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(("drained" if mode else "free-running"),
              f"step {el / args.steps * 1e6:.1f} us ({args.batch * args.steps / el:.0f} graphs/s):",
              ", ".join(f"{k} {v / args.steps * 1e6:.1f}" for k, v in acc.items()), flush=True)


if __name__ == "__main__":
    main()
