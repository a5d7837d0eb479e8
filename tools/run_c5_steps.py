"""Runs a few eager C5 training steps (for rocprofv3 counter passes)."""
import sys
import torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from bench import CONFIGS, build_model  # noqa: E402
from spotv2net_amd import synthetic_batch  # noqa: E402
from spotv2net_amd.train import TrainStep  # noqa: E402

cfg = dict(CONFIGS["c5"])
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dev = torch.device("cuda", 0)
model = build_model(dev, cfg)
data = synthetic_batch(B, cfg["S"], n=cfg["n"], seed=1, device=dev)
step = TrainStep(model, data, use_graph=False)
for _ in range(3):
    step()
torch.cuda.synchronize()
print("ok", float(step.loss))
