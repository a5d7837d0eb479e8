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


def _oracle_curve(ds_cpu, init_state, epochs, dev, BS=BS, on=None):
    """The oracle's curve; ``on``: the device its (unchanged) PyTorch ops run
    on — the CPU by default, the GPU for the full-size C3 run (minutes of
    unfolded lin_edge GEMMs on the host otherwise; f32 matmuls are exact f32
    on gfx950, which has no reduced-precision f32 MFMA)."""
    from oracle.pyg_gatconv import OracleGATModel
    on = on or torch.device("cpu")
    ref = OracleGATModel(30 * S, 3 * S, 6, 1, [500], dropout=P_DROP, concat_heads=True)
    ref.load_state_dict(init_state)
    ref = ref.to(on)
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
            b = ds_cpu.batch(idx).to(on)
            _seed(e, nb)
            keep = (torch.rand(idx.numel() * 30, 500, device=dev) >= P_DROP).float().to(on)
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
                b = ds_cpu.batch(torch.arange(k, min(n, k + BS))).to(on)
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


# ---- C3 at its stated size: config/GNN_param.yaml:26-39 batch 128, 3 epochs;
#      2,157 windows = what CovarianceLaggedDataset yields from 10,556 matrices
#      after the [8357:] cut (utils/dataset.py:200, :288) ----
BS_FULL, EPOCHS_FULL = 128, 3


@pytest.fixture(scope="module")
def curves_full(dev):
    from spotv2net_amd import GATModel, WindowDataset
    from spotv2net_amd.data import synthetic_series
    from spotv2net_amd.train import fit
    V, W = synthetic_series(10556, 30, seed=1234)
    ds_cpu = WindowDataset(V, W, S, cut=8357)
    ds_gpu = WindowDataset(V.to(dev), W.to(dev), S, cut=8357)
    assert len(ds_cpu) == len(ds_gpu) == 2157
    torch.manual_seed(5154)
    m0 = GATModel(30 * S, 3 * S, 6, 1, [500], dropout=P_DROP, concat_heads=True)
    init = {k: v.clone() for k, v in m0.state_dict().items()}
    out = {"oracle": _oracle_curve(ds_cpu, init, EPOCHS_FULL, dev, BS=BS_FULL, on=dev)}
    for prec in ("f32", "bf16"):
        m = GATModel(30 * S, 3 * S, 6, 1, [500], dropout=P_DROP, concat_heads=True)
        m.load_state_dict(init)
        m = m.to(dev).set_precision(prec)
        h = fit(m, ds_gpu, num_epochs=EPOCHS_FULL, batch_size=BS_FULL, lr=LR,
                generator=torch.Generator().manual_seed(7), step_hook=_seed)
        out[prec] = [(r["train_loss"], r["test_loss"]) for r in h]
    return out


def test_c3_full_size_fp32_curve_matches_oracle(curves_full):
    """3e-3: 42 Adam steps here against 6 in the small run above.  The
    per-step gradients agree to ~1e-6, but Adam's update m/sqrt(v) is close to
    a sign for coordinates whose gradient is small against its history, so
    summation-order differences turn into parameter differences of ~lr per
    step on those coordinates and the curves drift apart slowly.  Measured
    (MI355X): the oracle alone, rerun (its GPU index_add_ sums in atomic
    order), moved its epoch-3 test loss by 1.2e-3 (1.03532 vs 1.03650); the
    HIP path sat within 1.6e-4 / 5.3e-4 (train / test) of it in epoch 1 and
    4.5e-4 / 1.7e-4 in epoch 3."""
    print("C3 full-size curves (train, test) per epoch:", curves_full)
    assert len(curves_full["f32"]) == EPOCHS_FULL
    for (tr, te), (rtr, rte) in zip(curves_full["f32"], curves_full["oracle"]):
        assert _rel(tr, rtr) < 3e-3, (tr, rtr)
        assert _rel(te, rte) < 3e-3, (te, rte)


def test_c3_full_size_bf16_curve_matches_oracle(curves_full):
    for (tr, te), (rtr, rte) in zip(curves_full["bf16"], curves_full["oracle"]):
        assert _rel(tr, rtr) < 3e-2, (tr, rtr)
        assert _rel(te, rte) < 3e-2, (te, rte)


@pytest.mark.parametrize("bs", [16, 12])
def test_test_pass_equals_per_batch_losses(dev, bs):
    """Fit's test pass — one forward over every test window, each batch's MSE
    from its own row slice — gives the reference's per-batch loop
    (5_train_SpotV2Net.py:166-180: model(data) + MSELoss on each sequential
    test batch, averaged over the batches), ragged last batch included."""
    from spotv2net_amd import GATModel
    from spotv2net_amd.train import Fit
    _, ds = _data(dev)
    torch.manual_seed(11)
    m = GATModel(30 * S, 3 * S, 4, 1, [32, 16], concat_heads=True).to(dev)
    f = Fit(m, ds, bs, generator=torch.Generator().manual_seed(3))
    assert f.n_test % bs != 0  # a ragged last batch is part of the check
    rec = f.run_epoch()
    m.eval()
    losses = []
    with torch.no_grad():
        for k in range(f.n_train, len(ds), bs):
            idx = torch.arange(k, min(k + bs, len(ds)), device=dev)
            b = ds.batch(idx)
            losses.append(torch.nn.functional.mse_loss(m(b), b.y_x).item())
    want = sum(losses) / len(losses)
    assert abs(rec["test_loss"] - want) <= 1e-6 * abs(want), (rec["test_loss"], want)


def test_test_pass_chunked_by_memory_budget(dev, monkeypatch):
    """With a device-memory budget below the whole test split the test pass
    runs in chunks of whole batches (Fit.eval_chunk): same per-epoch test
    loss, bit for bit, as one forward over every test window."""
    import copy

    from spotv2net_amd import GATModel, train
    from spotv2net_amd.train import Fit
    _, ds = _data(dev)
    torch.manual_seed(11)
    m0 = GATModel(30 * S, 3 * S, 4, 1, [32, 16], concat_heads=True).to(dev)
    bs = 12
    recs = []
    for budget in (1 << 40, None):
        m = copy.deepcopy(m0)
        f = Fit(m, ds, bs, generator=torch.Generator().manual_seed(3))
        if budget is None:  # two batches per chunk, ragged tail chunk
            budget = 2 * bs * f._window_bytes()
        monkeypatch.setattr(train, "EVAL_BYTES", budget)
        chunk = f.eval_chunk()
        assert chunk == (f.n_test if budget == 1 << 40 else 2 * bs)
        recs.append([f.run_epoch() for _ in range(2)])
    assert f.n_test % (2 * bs) != 0 and f.n_test > 2 * bs
    assert recs[0] == recs[1]


def test_fit_cov_var_only_gather_is_bitwise_full_gather(dev, monkeypatch):
    """Fit gathers only the covariance-layout columns of edge_attr when the
    model reads them through those passes alone (sv2n_window_gather_cv); the
    loss history and the trained parameters are those of the full gather."""
    import copy

    from spotv2net_amd import GATModel, stack
    from spotv2net_amd.train import Fit
    _, ds = _data(dev)
    torch.manual_seed(11)
    m0 = GATModel(30 * S, 3 * S, 4, 1, [32, 16], concat_heads=True, dropout=0.1).to(dev)
    runs = []
    for cv in (True, False):
        if not cv:
            monkeypatch.setattr(stack, "cov_var_edges_only", lambda *a: False)
        m = copy.deepcopy(m0)
        torch.manual_seed(5)
        f = Fit(m, ds, 24, generator=torch.Generator().manual_seed(3))
        assert f._cv_only == cv
        hist = [f.run_epoch() for _ in range(2)]
        runs.append((hist, [p.detach().clone() for p in m.parameters()]))
    (h0, p0), (h1, p1) = runs
    assert h0 == h1
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
