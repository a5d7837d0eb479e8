"""BASELINE config C3: the reference's full training loop
(5_train_SpotV2Net.py:86-197; yaml model: hidden [500], 6 heads, dropout 0.1,
Adam 1e-3) run by spotv2net_amd.train.fit, its loss curve against the fp32
oracle's curve on the same windows, batch order and dropout masks.

Tolerances (relative, per epoch and phase): fp32 mode 1e-3 (per-step
gradients agree to ~1e-6; Adam's normalisation amplifies that over the
steps), bf16 mode 3e-2 (bf16 operands carry 8 significant bits)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

S, P_DROP, LR, BS = 42, 0.1, 1e-3, 64


def _data(dev):
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    T = 200 + S
    V, W = synthetic_series(T, 30, seed=99)
    return WindowDataset(V, W, S), WindowDataset(V.to(dev), W.to(dev), S)


def _seed(epoch, k):
    torch.cuda.manual_seed(1000 * epoch + k)


def _oracle_curve(ds_cpu, init_state, epochs, dev):
    from oracle.pyg_gatconv import OracleGATModel
    ref = OracleGATModel(30 * S, 3 * S, 6, 1, [500], dropout=P_DROP, concat_heads=True)
    ref.load_state_dict(init_state)
    opt = torch.optim.Adam(ref.parameters(), lr=LR)
    gen = torch.Generator().manual_seed(7)
    n = len(ds_cpu)
    n_train = int(0.8 * n)
    hist = []
    for e in range(epochs):
        perm = torch.randperm(n_train, generator=gen)
        ref.train()
        tot, nb = 0.0, 0
        for k in range(0, n_train, BS):
            idx = perm[k:k + BS]
            b = ds_cpu.batch(idx)
            _seed(e, nb)
            keep = (torch.rand(idx.numel() * 30, 500, device=dev) >= P_DROP).float().cpu()
            ref.post_keep = [keep]
            loss = torch.nn.functional.mse_loss(ref(b), b.y_x)
            opt.zero_grad()
            loss.backward()
            opt.step()
            tot += loss.item()
            nb += 1
        ref.eval()
        tt, nt = 0.0, 0
        with torch.no_grad():
            for k in range(n_train, n, BS):
                b = ds_cpu.batch(torch.arange(k, min(n, k + BS)))
                tt += torch.nn.functional.mse_loss(ref(b), b.y_x).item()
                nt += 1
        hist.append((tot / nb, tt / nt))
    return hist


@pytest.fixture(scope="module")
def curves(dev):
    from spotv2net_amd import GATModel
    from spotv2net_amd.train import fit
    ds_cpu, ds_gpu = _data(dev)
    torch.manual_seed(5154)
    m0 = GATModel(30 * S, 3 * S, 6, 1, [500], dropout=P_DROP, concat_heads=True)
    init = {k: v.clone() for k, v in m0.state_dict().items()}
    out = {"oracle": _oracle_curve(ds_cpu, init, 2, dev)}
    for prec in ("f32", "bf16"):
        m = GATModel(30 * S, 3 * S, 6, 1, [500], dropout=P_DROP, concat_heads=True)
        m.load_state_dict(init)
        m = m.to(dev).set_precision(prec)
        h = fit(m, ds_gpu, num_epochs=2, batch_size=BS, lr=LR,
                generator=torch.Generator().manual_seed(7), step_hook=_seed)
        out[prec] = [(r["train_loss"], r["test_loss"]) for r in h]
    return out


def _rel(a, b):
    return abs(a - b) / abs(b)


def test_fp32_loss_curve_matches_oracle(curves):
    for (tr, te), (rtr, rte) in zip(curves["f32"], curves["oracle"]):
        assert _rel(tr, rtr) < 1e-3, (tr, rtr)
        assert _rel(te, rte) < 1e-3, (te, rte)


def test_bf16_loss_curve_matches_oracle(curves):
    for (tr, te), (rtr, rte) in zip(curves["bf16"], curves["oracle"]):
        assert _rel(tr, rtr) < 3e-2, (tr, rtr)
        assert _rel(te, rte) < 3e-2, (te, rte)


def test_fit_graph_replay_equals_eager(dev):
    """fit with hipGraph replay (window gather + step + ragged tail in graphs)
    == fit with eager steps, no dropout (nothing random on the device)."""
    from spotv2net_amd import GATModel
    from spotv2net_amd.train import fit
    _, ds = _data(dev)
    hs = []
    for use_graph in (True, False):
        torch.manual_seed(11)
        m = GATModel(30 * S, 3 * S, 4, 1, [32, 16], concat_heads=True).to(dev)
        hs.append(fit(m, ds, num_epochs=2, batch_size=48, generator=torch.Generator().manual_seed(3),
                      use_graph=use_graph))
    for a, b in zip(*hs):
        assert abs(a["train_loss"] - b["train_loss"]) <= 1e-6 * abs(b["train_loss"])
        assert abs(a["test_loss"] - b["test_loss"]) <= 1e-6 * abs(b["test_loss"])
