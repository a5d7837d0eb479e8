"""Data-parallel path on CPU: world_size-2 ``gloo`` process groups (the GPU
runs use the same code over nccl = RCCL).

* TrainStep's flat-gradient all-reduce (train.allreduce_mean_) over two ranks,
  each holding its own shard of graphs, gives the same Adam step as one
  process on the concatenated batch (mean-reduced MSE, equal shard sizes) —
  SURVEY.md §8e.  The per-rank compute here is the oracle model on the host
  (the HIP path needs a GPU); what is under test is the DP machinery.
* shard_indices partitions like DistributedSampler.
* bench.py's max-over-ranks timing and weight broadcast."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

S, N, HEADS, HIDDEN, B_LOCAL = 2, 30, 2, [6, 4], 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(seed=5154):
    from oracle.pyg_gatconv import OracleGATModel
    torch.manual_seed(seed)
    return OracleGATModel(N * S, 3 * S, HEADS, 1, HIDDEN, concat_heads=True)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from spotv2net_amd import synthetic_batch
        from spotv2net_amd.train import TrainStep
        torch.set_num_threads(1)
        model = _model(seed=100 + rank)        # different init per rank ...
        for p in model.parameters():           # ... made identical like bench.py does
            dist.broadcast(p.data, 0)
        data = synthetic_batch(B_LOCAL, S, n=N, seed=1234 + rank)
        step = TrainStep(model, data, lr=1e-2, use_graph=False, optimizer="torch")
        assert step.distributed
        for _ in range(2):
            step()
        torch.save({k: v.clone() for k, v in model.state_dict().items()},
                   os.path.join(out_dir, f"rank{rank}.pt"))
        t = bench.max_over_ranks(float(rank + 1), torch.device("cpu"))
        assert t == float(world)
    finally:
        dist.destroy_process_group()


def test_two_rank_step_equals_concatenated_batch(tmp_path):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    # single process, both shards concatenated (collate of the two batches)
    from spotv2net_amd import Data, collate, synthetic_batch
    from spotv2net_amd.train import TrainStep
    parts = [synthetic_batch(B_LOCAL, S, n=N, seed=1234 + r) for r in range(2)]
    graphs = []
    for b in parts:
        for g in range(B_LOCAL):
            nodes = slice(g * N, (g + 1) * N)
            E0 = N * (N - 1)
            graphs.append(Data(x=b.x[nodes], edge_index=b.edge_index[:, g * E0:(g + 1) * E0] - g * N,
                               edge_attr=b.edge_attr[g * E0:(g + 1) * E0], y_x=b.y_x[nodes]))
    full = collate(graphs)
    model = _model(seed=100)
    step = TrainStep(model, full, lr=1e-2, use_graph=False, optimizer="torch")
    for _ in range(2):
        step()
    ref = model.state_dict()
    for k in ref:
        torch.testing.assert_close(r0[k], r1[k], rtol=0, atol=0)  # replicas stay identical
        torch.testing.assert_close(r0[k], ref[k], rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("n,world", [(10, 2), (11, 2), (7, 4), (3, 8)])
def test_shard_indices_matches_distributed_sampler(n, world):
    from torch.utils.data.distributed import DistributedSampler

    from spotv2net_amd import shard_indices
    idx = torch.arange(n)
    for r in range(world):
        ds = DistributedSampler(list(range(n)), num_replicas=world, rank=r, shuffle=False)
        assert shard_indices(idx, r, world).tolist() == list(iter(ds))
