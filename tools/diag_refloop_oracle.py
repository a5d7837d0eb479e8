"""Diagnostic: the reference loop on the GPU (graph replay and eager) against
the PyG-semantics oracle in fp32 and fp64, step by step: loss, gradient
error per parameter (scaled), and how many gradient entries differ in sign
from the fp64 oracle's (Adam's first steps move a weight by ~lr·sign(g))."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    from helpers import float64_twin, twin_model
    from spotv2net_amd import Batch, Data, synthetic_batch
    dev = torch.device("cuda", 0)
    mine, ref = twin_model(seed=5154, num_node_features=1260, num_edge_features=126, num_heads=4,
                           output_node_channels=1, dim_hidden_layers=[100, 50], concat_heads=True)
    ref64 = float64_twin(ref)
    mine = mine.to(dev)
    eager = copy.deepcopy(mine)
    eager.graph_replay = False
    data = synthetic_batch(32, 42, seed=1234, device=dev)
    cpu = synthetic_batch(32, 42, seed=1234)
    cpu64 = Data(x=cpu.x.double(), edge_index=cpu.edge_index, edge_attr=cpu.edge_attr.double(),
                 y_x=cpu.y_x.double())
    models = {"graphed": mine, "eager": eager, "oracle32": ref, "oracle64": ref64}
    opts = {k: torch.optim.Adam(m.parameters(), lr=1e-3) for k, m in models.items()}
    for step in range(3):
        losses, grads = {}, {}
        for k, m in models.items():
            if k in ("graphed", "eager"):
                b = Batch(x=data.x, edge_index=data.edge_index.clone(), edge_attr=data.edge_attr,
                          y_x=data.y_x, batch=data.batch, ptr=data.ptr, nodes_per_graph=30,
                          canonical_edges=True)
            else:
                b = cpu64 if k == "oracle64" else cpu
            loss = torch.nn.functional.mse_loss(m(b), b.y_x)
            opts[k].zero_grad()
            loss.backward()
            losses[k] = loss.item()
            grads[k] = {n: p.grad.detach().double().cpu().clone() for n, p in m.named_parameters()}
            opts[k].step()
        print(f"step {step + 1} losses " + " ".join(f"{k} {v:.9f}" for k, v in losses.items()))
        for n in grads["oracle64"]:
            g64 = grads["oracle64"][n]
            sc = max(1.0, g64.abs().max().item())
            row = []
            for k in ("graphed", "eager", "oracle32"):
                g = grads[k][n]
                err = (g - g64).abs().max().item() / sc
                flips = int(((g > 0) != (g64 > 0)).sum().item())
                row.append(f"{k} err {err:.2e} flips {flips}")
            small = int((g64.abs() < 1e-7).sum().item())
            print(f"   {n:34s} |g|max {g64.abs().max().item():.2e} tiny {small:5d}  " + "; ".join(row))


if __name__ == "__main__":
    main()
