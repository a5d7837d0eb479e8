"""Host-side anatomy of the reference loop's step (5_train_SpotV2Net.py:142-160,
as bench.reference_loop_rate runs it: device-resident canonical batches, a new
edge_index per step): wall time per phase with no syncs inside the step, and
the host time of the pieces inside model() and backward() (graph replays,
Function.apply, gradient copy), measured by wrapping them.

usage: python tools/ref_loop_host.py [--steps 200] [--fused-adam 0]"""
import argparse
import collections
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--fused-adam", type=int, default=0)
    ap.add_argument("--wrap", type=int, default=1)
    args = ap.parse_args()
    from spotv2net_amd import Batch, GATModel, graphed, model as model_mod, synthetic_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(5154)
    model = GATModel(1260, 126, 4, 1, [100, 50], concat_heads=True).to(dev)
    datas = [synthetic_batch(args.batch, 42, seed=1234 + i, device=dev) for i in range(2)]
    # fused=False would also switch off the foreach default: pass it only when set
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, **({"fused": True} if args.fused_adam else {}))
    crit = torch.nn.MSELoss()
    acc = collections.defaultdict(float)
    marks = {}

    def wrap(obj, name, label):
        f = getattr(obj, name)

        def w(*a, **k):
            t = time.perf_counter()
            marks.setdefault(label if label not in marks else label + "#2", t)
            try:
                return f(*a, **k)
            finally:
                acc[label] += time.perf_counter() - t
        setattr(obj, name, w)

    if args.wrap:
        wrap(model_mod, "_layout_of", "model.layout_of")
        wrap(graphed, "forward", "model.graphed_forward")
        wrap(graphed, "_switches", "graphed.switches")
        wrap(torch.cuda.CUDAGraph, "replay", "graph.replay")
        wrap(graphed._Entry, "load_layout", "entry.load_layout")
        orig_bwd = graphed._Replay.backward

        def bwd(ctx, dout):
            t = time.perf_counter()
            marks.setdefault("replay.backward", t)
            try:
                return orig_bwd(ctx, dout)
            finally:
                acc["replay.backward"] += time.perf_counter() - t
        graphed._Replay.backward = staticmethod(bwd)
    it = [0]

    def step(ph):
        marks.clear()
        t = [time.perf_counter()]
        d = datas[it[0] % 2]
        it[0] += 1
        b = Batch(x=d.x, edge_index=d.edge_index.clone(), edge_attr=d.edge_attr, y_x=d.y_x,
                  batch=d.batch, ptr=d.ptr, nodes_per_graph=30, canonical_edges=True)
        t.append(time.perf_counter())
        out = model(b)
        t.append(time.perf_counter())
        loss = crit(out, b.y_x)
        t.append(time.perf_counter())
        opt.zero_grad()
        t.append(time.perf_counter())
        loss.backward()
        t.append(time.perf_counter())
        opt.step()
        t.append(time.perf_counter())
        loss.item()
        t.append(time.perf_counter())
        for k, a, c in zip(("batch", "fwd", "loss", "zero", "bwd", "opt", "item"), t, t[1:]):
            ph[k] += c - a
        # host clock of the first call of each wrapped piece, from the step start
        for k, v in marks.items():
            ph["@" + k] += v - t[0]
        ph["@opt_done"] += t[-2] - t[0]

    ph = collections.defaultdict(float)
    for _ in range(10):
        step(ph)
    ph.clear()
    acc.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(ph)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n = args.steps
    print(f"fused_adam={args.fused_adam} wrap={args.wrap}: step {el / n * 1e6:.1f} us "
          f"({args.batch * n / el:.0f} graphs/s)")
    print("  phases: " + ", ".join(f"{k} {v / n * 1e6:.1f}" for k, v in ph.items()))
    print("  inside: " + ", ".join(f"{k} {v / n * 1e6:.1f}" for k, v in sorted(acc.items())))


if __name__ == "__main__":
    main()
