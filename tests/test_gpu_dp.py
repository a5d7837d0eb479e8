"""Data-parallel training step on the GPU (BASELINE config C4):
TrainStep's distributed branch — captured forward+backward graph, ONE
all-reduce of the flat gradient buffer, captured Adam graph — run on HIP by
two ranks.

The box has one MI355X, so both ranks share ``cuda:0`` under a ``gloo``
group (RCCL refuses two ranks on one device; gloo all-reduces through a host
copy, ``train.allreduce_mean_``).  What runs on the GPU is exactly the C4
code path of ``bench.py --gpus N`` apart from the transport.  Each rank trains
its own shard of C2-shaped graphs (30 nodes, S = 42, GAT [100, 50] x 4 heads
concat); the reference being data-parallelised is the step of
5_train_SpotV2Net.py:142-160."""
import os
import socket

import pytest
import torch

from helpers import assert_close

pytestmark = pytest.mark.gpu

S, B_LOCAL, STEPS, LR = 42, 64, 3, 1e-3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(seed):
    from spotv2net_amd import GATModel
    torch.manual_seed(seed)
    return GATModel(30 * S, 3 * S, 4, 1, [100, 50], concat_heads=True)


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spotv2net_amd import synthetic_batch
        from spotv2net_amd.train import TrainStep, broadcast_params_
        model = _model(seed=100 + rank).to(dev)   # different init per rank ...
        broadcast_params_(model, 0)               # ... made identical as bench.py does
        data = synthetic_batch(B_LOCAL, S, seed=1234 + rank, device=dev)
        step = TrainStep(model, data, lr=LR, use_graph=True)
        assert step.distributed and step._shapes[0].g_opt is not None
        losses = [float(step().item())]
        m1 = step.opt.m.detach().cpu().clone()  # (1 - beta1) x the all-reduced gradient
        losses += [float(step().item()) for _ in range(STEPS - 1)]
        torch.cuda.synchronize()
        torch.save({"state": {k: v.detach().cpu() for k, v in model.state_dict().items()},
                    "losses": losses, "m1": m1}, os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_two_rank_trainstep_on_hip_equals_concatenated_batch(dev, tmp_path):
    import torch.multiprocessing as mp

    from spotv2net_amd import collate, synthetic_batch
    from spotv2net_amd.data import Data
    from spotv2net_amd.train import TrainStep
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    for k in r0["state"]:   # the replicas stay bit-identical
        assert torch.equal(r0["state"][k], r1["state"][k]), k

    # one process, both shards concatenated (PyG collation of the 2 x 64 graphs)
    E0 = 870
    graphs = []
    for r in range(2):
        b = synthetic_batch(B_LOCAL, S, seed=1234 + r, device=dev)
        for g in range(B_LOCAL):
            nodes = slice(g * 30, (g + 1) * 30)
            graphs.append(Data(x=b.x[nodes], y_x=b.y_x[nodes],
                               edge_index=b.edge_index[:, g * E0:(g + 1) * E0] - g * 30,
                               edge_attr=b.edge_attr[g * E0:(g + 1) * E0]))
    full = collate(graphs)
    model = _model(seed=100).to(dev)
    step = TrainStep(model, full, lr=LR, use_graph=True)
    losses = [float(step().item())]
    m1 = step.opt.m.detach().cpu().clone()
    losses += [float(step().item()) for _ in range(STEPS - 1)]
    assert torch.equal(r0["m1"], r1["m1"])
    # step 1: the all-reduced mean gradient == the full batch's gradient (the
    # first Adam moment is (1 - beta1) g), per parameter by the 1e-5 rule
    off = 0
    for name, p in model.named_parameters():
        k = p.numel()
        assert_close(r0["m1"][off:off + k] / 0.1, m1[off:off + k] / 0.1, what=f"grad {name}")
        off += k
    # the loss each rank reports is its shard's mean; their mean is the full
    # batch's: step 1 within 1e-5, later steps within 1e-4 relative (after an
    # Adam step, rounding-level gradient differences in near-zero entries are
    # lr-sized weight differences: tests/test_gpu_graphed.py)
    for k in range(STEPS):
        tol = 1e-5 if k == 0 else 1e-4
        assert abs(0.5 * (r0["losses"][k] + r1["losses"][k]) - losses[k]) <= tol * max(
            1.0, abs(losses[k])), (k, r0["losses"][k], r1["losses"][k], losses[k])
