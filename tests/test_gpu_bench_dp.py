"""bench.py's N > 1 branch end to end on the GPU (BASELINE config C4):
two ranks run ``bench.main`` with ``--gpus 2`` — the parameter broadcast,
TrainStep's distributed branch (forward+backward graph, one all-reduce of
the flat gradient buffer, Adam graph), ``time_replays``' barriers,
``max_over_ranks``, the replica check, the DDP-wrapped reference loops and
ForwardStep — and rank 0 prints one JSON line.

The box has one MI355X, so both ranks share ``cuda:0`` under ``--backend
gloo`` (RCCL refuses two ranks on one device; gloo moves the buffers through
host copies).  The driver's 8-GPU run takes the same branch with RCCL."""
import contextlib
import json
import os
import socket
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      LOCAL_RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(out_dir, f"out{rank}.txt"), "w") as f, contextlib.redirect_stdout(f):
        bench.main(["--gpus", str(world), "--steps", "3", "--warmup", "2", "--backend", "gloo",
                    "--no-cpu-baseline", "--no-kernel-table"])


def test_bench_two_ranks_one_json_line(tmp_path):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    out0 = (tmp_path / "out0.txt").read_text().strip().splitlines()
    out1 = (tmp_path / "out1.txt").read_text().strip().splitlines()
    assert len(out0) == 1 and out1 == []          # ONE JSON line, from rank 0
    r = json.loads(out0[0])
    assert r["n_gpus"] == 2 and r["config"]["global_batch"] == 1024
    assert r["config"]["parallelism"] == "dp2" and r["backend"] == "gloo"
    assert r["replicas_bit_identical"] is True     # parameters equal after the timed steps
    assert r["value"] > 0 and r["fwd_graphs_per_s"] > 0
    for k in ("ref_loop_graphs_per_s", "ref_loop_fused_adam_graphs_per_s",
              "ref_loop_block_layout_graphs_per_s", "ref_loop_literal_graphs_per_s"):
        assert r[k] > 0, k
    assert r["final_loss"] == r["final_loss"]       # finite
