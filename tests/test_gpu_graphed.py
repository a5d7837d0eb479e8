"""GATModel.forward / backward replayed as hipGraphs (graphed.py) — the fast
path of the reference's own loop, 5_train_SpotV2Net.py:142-160, unchanged:
a new batch object per step, model(data), nn.MSELoss, zero_grad, backward,
torch.optim.Adam, loss.item()."""
import copy

import pytest
import torch

from helpers import assert_close

pytestmark = pytest.mark.gpu


def _model(dev, S=4, hidden=(16, 8), heads=4, seed=0, **kw):
    from spotv2net_amd import GATModel
    torch.manual_seed(seed)
    return GATModel(30 * S, 3 * S, heads, 1, list(hidden), concat_heads=True, **kw).to(dev)


def _fresh(data, n=30, canonical=False):
    """A new batch object with a new edge_index each step (what a DataLoader
    yields), graph size known (sv2n collate / PyG slice table); ``canonical``:
    marked as sv2n collate marks a batch of canonical-order graphs."""
    from spotv2net_amd import Batch
    extra = {"canonical_edges": True} if canonical else {}
    return Batch(x=data.x, edge_index=data.edge_index.clone(), edge_attr=data.edge_attr,
                 y_x=data.y_x, batch=data.batch, ptr=data.ptr, nodes_per_graph=n, **extra)


def _ref_loop(model, data, steps, lr=1e-3, canonical=False):
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    crit = torch.nn.MSELoss()
    losses = []
    for _ in range(steps):
        b = _fresh(data, canonical=canonical)
        loss = crit(model(b), b.y_x)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return losses


@pytest.mark.parametrize("canonical", [False, True])
def test_reference_loop_replayed_equals_eager(dev, canonical):
    """The loop with graph replay (captured at step 2, replayed from step 3)
    gives the eager loop's losses and parameters bit for bit: the same
    kernels in the same order (block layout analysed per step, or the
    collate-verified canonical layout)."""
    from spotv2net_amd import synthetic_batch
    data = synthetic_batch(16, 4, seed=2, device=dev)
    m1 = _model(dev, seed=3)
    m2 = copy.deepcopy(m1)
    m2.graph_replay = False
    l1 = _ref_loop(m1, data, 6, canonical=canonical)
    l2 = _ref_loop(m2, data, 6, canonical=canonical)
    assert len(m1._graph_cache.entries) == 1 and m1._graph_cache.entries[
        next(iter(m1._graph_cache.entries))].g_bwd is not None
    assert l1 == l2
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(p, q), n


def _oracle_loop(ref, data, steps, grads_at=None):
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    losses = []
    for k in range(steps):
        loss = torch.nn.functional.mse_loss(ref(data), data.y_x)
        opt.zero_grad()
        loss.backward()
        if grads_at is not None and k == 0:
            grads_at.update({n: p.grad.detach().clone() for n, p in ref.named_parameters()})
        opt.step()
        losses.append(loss.item())
    return losses


def test_reference_loop_matches_oracle_after_3_steps(dev):
    """C2-shaped model (S 42, GAT [100, 50] x 4 heads concat, relu) through
    the reference loop on the replay path vs the PyG-semantics oracle running
    the same loop on the host.

    Step 1 — loss and every gradient — by the parity rule of tests/helpers.py
    (1e-5 of the fp32 oracle, or at least as close to the float64 oracle).
    Steps 2 and 3: losses within 1e-4 relative.  After an update the
    trajectories separate faster than fp32 rounding: a pre-activation within
    rounding of 0 takes ReLU's other branch (that node's whole contribution
    to a layer-0 gradient), and Adam's first steps move every weight by
    ~lr·g/|g|, so a rounding-level difference in a near-zero gradient entry is
    an lr-sized weight difference (MI355X: 1e-6 gradient error at step 1,
    2.8e-5 relative loss difference at step 3; fp32 vs float64 oracle 1e-6)."""
    from helpers import assert_parity, float64_twin, twin_model
    from spotv2net_amd import Data, synthetic_batch
    mine, ref = twin_model(seed=5154, num_node_features=1260, num_edge_features=126,
                           num_heads=4, output_node_channels=1, dim_hidden_layers=[100, 50],
                           concat_heads=True)
    ref64 = float64_twin(ref)
    mine = mine.to(dev)
    data = synthetic_batch(32, 42, seed=1234, device=dev)
    g_mine = {}
    opt = torch.optim.Adam(mine.parameters(), lr=1e-3)
    got = []
    for k in range(3):
        b = _fresh(data, canonical=True)
        loss = torch.nn.functional.mse_loss(mine(b), b.y_x)
        opt.zero_grad()
        loss.backward()
        if k == 0:
            g_mine = {n: p.grad.detach().clone() for n, p in mine.named_parameters()}
        opt.step()
        got.append(loss.item())
    cpu = synthetic_batch(32, 42, seed=1234)
    g32, g64 = {}, {}
    want = _oracle_loop(ref, cpu, 3, g32)
    cpu64 = Data(x=cpu.x.double(), edge_index=cpu.edge_index, edge_attr=cpu.edge_attr.double(),
                 y_x=cpu.y_x.double())
    want64 = _oracle_loop(ref64, cpu64, 3, g64)
    assert_parity(torch.tensor(got[0]), torch.tensor(want[0]), torch.tensor(want64[0]),
                  what="loss of step 1")
    for n in g32:
        assert_parity(g_mine[n], g32[n], g64[n], what=f"step-1 gradient of {n}")
    for k in (1, 2):
        assert abs(got[k] - want[k]) <= 1e-4 * abs(want[k]), (k + 1, got[k], want[k], want64[k])


def test_forward_awaiting_backward_is_not_overwritten(dev):
    """Two forwards before their backwards (gradient accumulation over two
    micro-batches): the second runs eagerly, both backwards are right."""
    from spotv2net_amd import synthetic_batch
    d1 = synthetic_batch(8, 4, seed=5, device=dev)
    d2 = synthetic_batch(8, 4, seed=6, device=dev)
    m1 = _model(dev, seed=7)
    m2 = copy.deepcopy(m1)
    m2.graph_replay = False
    for m in (m1, m2):
        for _ in range(3):  # capture (call 2) and replay (call 3) with d1's signature
            m(_fresh(d1)).sum().backward()
        m.zero_grad()
    for m in (m1, m2):
        a = m(_fresh(d1))
        b = m(_fresh(d1))      # same signature while a awaits its backward
        c = m(_fresh(d2))
        (a ** 2).sum().backward()
        (3 * b).sum().backward()
        (c ** 3).mean().backward()
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(p.grad, q.grad), n


def test_retained_backward_after_overwrite_raises(dev):
    from spotv2net_amd import synthetic_batch
    d = synthetic_batch(8, 4, seed=5, device=dev)
    m = _model(dev, seed=8)
    for _ in range(3):
        m(_fresh(d)).sum().backward()
    out = m(_fresh(d))
    loss = out.sum()
    loss.backward(retain_graph=True)
    m(_fresh(d)).sum().backward()   # replays the same graph: out's saved state is gone
    with pytest.raises(RuntimeError, match="overwritten"):
        loss.backward()


def test_inference_replay_and_autograd_grad(dev):
    """eval + no_grad calls replay a forward-only graph; torch.autograd.grad
    through a replayed training graph returns the eager gradients."""
    from spotv2net_amd import synthetic_batch
    d = synthetic_batch(12, 4, seed=9, device=dev)
    m1 = _model(dev, seed=10)
    m2 = copy.deepcopy(m1)
    m2.graph_replay = False
    m1.eval()
    m2.eval()
    with torch.no_grad():
        outs = [m1(_fresh(d)) for _ in range(3)]
        want = m2(_fresh(d))
    for o in outs:
        assert torch.equal(o, want)
    assert outs[0].data_ptr() != outs[2].data_ptr()  # fresh output per call
    m1.train()
    m2.train()
    for _ in range(3):
        g1 = torch.autograd.grad(m1(_fresh(d)).square().sum(), list(m1.parameters()))
    g2 = torch.autograd.grad(m2(_fresh(d)).square().sum(), list(m2.parameters()))
    for a, b in zip(g1, g2):
        assert torch.equal(a, b)


# ---------------------------------------------------------------------------
# the DataLoader pattern: a different host batch every step, moved with
# .to(device) (5_train_SpotV2Net.py:142-147), so the replayed graphs see new
# contents at allocator-recycled, alternating addresses
# ---------------------------------------------------------------------------
def _host_batches(k, B=12, S=4, seed=40, canonical=False):
    from spotv2net_amd import synthetic_batch
    out = []
    for i in range(k):
        b = synthetic_batch(B, S, seed=seed + i)      # host tensors, distinct contents
        if canonical:
            b.canonical_edges = True
        out.append(b)
    return out


def _loader_loop(model, host, steps, dev, scale_up=None):
    """5_train_SpotV2Net.py:127, :142-160 as written: default torch.optim.Adam,
    ``data = data.to(device)``, the optional scale_up rebinding, MSELoss,
    zero_grad, backward, step, loss.item()."""
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    crit = torch.nn.MSELoss()
    losses, ptrs = [], set()
    for k in range(steps):
        data = host[k % len(host)]
        data = data.to(dev)
        if scale_up:
            data.x = data.x * scale_up
            data.edge_attr = data.edge_attr * scale_up
            data.y_x = data.y_x * scale_up
        ptrs.add((data.x.data_ptr(), data.edge_attr.data_ptr()))
        y_x_hat = model(data)
        loss = crit(y_x_hat, data.y_x)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return losses, ptrs


@pytest.mark.parametrize("scale_up,canonical", [(None, True), (None, False), (2.5, True)])
def test_dataloader_pattern_replay_equals_eager(dev, scale_up, canonical):
    """8 steps over 3 distinct host batches, each moved with .to(device):
    with graph replay on, losses and parameters equal the eager loop's bit for
    bit, and at least one captured entry is replayed at an address a later
    batch reuses (a stale read would show up as a loss difference)."""
    host = _host_batches(3, canonical=canonical)
    m1 = _model(dev, seed=21)
    m2 = copy.deepcopy(m1)
    m2.graph_replay = False
    l1, p1 = _loader_loop(m1, host, 8, dev, scale_up)
    l2, _ = _loader_loop(m2, host, 8, dev, scale_up)
    assert l1 == l2
    assert len(set(l1)) == len(l1)   # every step saw different data
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(p, q), n
    # the allocator recycles addresses: fewer distinct input addresses than steps,
    # so entries were replayed on new contents
    assert len(p1) < 8
    assert any(e.g_bwd is not None for e in m1._graph_cache.entries.values())


def test_inplace_refilled_batch_replay_equals_eager(dev):
    """One device batch whose contents are overwritten in place between steps
    (same addresses every step, e.g. a static prefetch buffer): every replay
    reads the new contents."""
    from spotv2net_amd import synthetic_batch
    host = _host_batches(4, seed=60)
    res = []
    for replay in (True, False):
        m = _model(dev, seed=22)
        m.graph_replay = replay
        buf = synthetic_batch(12, 4, seed=0, device=dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        losses = []
        for k in range(7):
            src = host[k % 4]
            buf.x.copy_(src.x)
            buf.edge_attr.copy_(src.edge_attr)
            buf.y_x.copy_(src.y_x)
            loss = torch.nn.functional.mse_loss(m(_fresh(buf)), buf.y_x)
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.item())
        res.append((losses, [p.detach().clone() for p in m.parameters()]))
    assert res[0][0] == res[1][0]
    assert len(set(res[0][0])) == len(res[0][0])
    for p, q in zip(res[0][1], res[1][1]):
        assert torch.equal(p, q)


def test_replayed_inputs_kept_alive_until_backward(dev):
    """The backward graph reads x / edge_attr in place: a batch dropped
    between forward and backward stays alive (the allocator cannot hand its
    memory to the next batch), so the gradients equal eager ones."""
    host = _host_batches(2, seed=80)
    m1 = _model(dev, seed=23)
    m2 = copy.deepcopy(m1)
    m2.graph_replay = False
    grads = []
    for m in (m1, m2):
        for k in range(3):   # capture + replay this signature
            m(host[0].to(dev)).square().sum().backward()
        m.zero_grad()
        out = m(host[0].to(dev))          # the batch has no other reference
        junk = [host[1].to(dev) for _ in range(3)]   # allocations that could reuse it
        for j in junk:
            j.x.fill_(7.0)
            j.edge_attr.fill_(-3.0)
        out.square().sum().backward()
        grads.append([p.grad.clone() for p in m.parameters()])
        del junk
    for a, b in zip(*grads):
        assert torch.equal(a, b)


def test_inplace_write_between_forward_and_backward_raises(dev):
    """Writing a replayed forward's x in place before its backward raises, as
    the eager node's saved-tensor version check does."""
    from spotv2net_amd import synthetic_batch
    d = synthetic_batch(8, 4, seed=31, device=dev)
    for replay in (True, False):
        m = _model(dev, seed=24)
        m.graph_replay = replay
        for _ in range(3):
            m(_fresh(d)).sum().backward()
        out = m(_fresh(d))
        d.x.add_(1.0)
        with pytest.raises(RuntimeError, match="inplace"):
            out.sum().backward()
        d.x.sub_(1.0)
