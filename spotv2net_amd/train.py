"""Training-step runtime for GATModel on MI355X.

Replaces the per-batch loop body of reference 5_train_SpotV2Net.py:142-160
(forward, MSELoss, zero_grad, backward, Adam step, ``loss.item()``) with a
launch-overhead-free step:

* all parameters and all gradients live in two flat fp32 buffers (``p`` and
  ``p.grad`` are views into them), so data-parallel training needs a single
  RCCL all-reduce per step (2.65 MB for the C2 model, no bucketing) and Adam
  is one kernel launch (``FlatAdam`` -> sv2n_adam_f32);
* the step is captured into a hipGraph (``torch.cuda.CUDAGraph`` on ROCm) —
  forward + loss + backward (+ Adam when single-process) replay as one graph,
  so host launch cost does not bound a ~1 ms step;
* the loss stays on the device: no per-step host synchronisation (the
  reference's ``loss.item()`` at :160); read ``step.loss`` when needed.

Data parallelism: one process per GPU, each with its own
device-resident shard of graphs; gradients are summed with
``all_reduce(SUM)`` over the default (nccl = RCCL) process group and divided
by the world size, which equals the single-process gradient of the
concatenated batch for a mean-reduced loss of equal per-rank batch sizes.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch
import torch.distributed as dist


def flatten_params(params) -> torch.Tensor:
    """Re-home every parameter as a view of ONE flat fp32 buffer (values kept)."""
    params = [p for p in params if p.requires_grad]
    flat = torch.cat([p.detach().reshape(-1) for p in params]).contiguous()
    off = 0
    for p in params:
        k = p.numel()
        p.data = flat[off:off + k].view_as(p)
        off += k
    return flat


def flatten_grads(params) -> torch.Tensor:
    """Allocate one flat buffer and make every ``p.grad`` a view into it."""
    params = [p for p in params if p.requires_grad]
    total = sum(p.numel() for p in params)
    dev = params[0].device
    flat = torch.zeros(total, device=dev, dtype=torch.float32)
    off = 0
    for p in params:
        k = p.numel()
        p.grad = flat[off:off + k].view_as(p)
        off += k
    return flat


class FlatAdam:
    """torch.optim.Adam (amsgrad=False) over flat parameter / gradient buffers:
    one sv2n_adam_f32 launch per step, device-side step counter (capturable)."""

    def __init__(self, flat_params: torch.Tensor, flat_grads: torch.Tensor, lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0):
        from . import library  # noqa: F401  (torch.ops.sv2n.adam_step)
        self.p, self.g = flat_params, flat_grads
        self.m = torch.zeros_like(flat_params)
        self.v = torch.zeros_like(flat_params)
        self.step_t = torch.zeros(1, device=flat_params.device, dtype=torch.float32)
        self.ticket = torch.zeros(288, device=flat_params.device, dtype=torch.int32)  # SV2N_TICKET_WORDS
        self.lr, self.betas, self.eps, self.wd = float(lr), betas, float(eps), float(weight_decay)

    # the kernel advances step_t itself and zeroes the consumed gradient
    zeroes_grads = True

    def step(self) -> None:
        torch.ops.sv2n.adam_step(self.p, self.g, self.m, self.v, self.step_t, self.ticket,
                                 self.lr, float(self.betas[0]), float(self.betas[1]), self.eps,
                                 self.wd)


def _host_staged(t: torch.Tensor, group) -> bool:
    """gloo moves host memory: device tensors go through a host copy."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def allreduce_sum_(flat: torch.Tensor, group=None) -> int:
    """Sum a flat gradient buffer across the data-parallel group in place: ONE
    all-reduce (RCCL over xGMI with the nccl backend; through a host copy with
    gloo).  Returns the world size (1: nothing done)."""
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    ws = dist.get_world_size(group)
    if ws == 1:
        return 1
    if _host_staged(flat, group):
        host = flat.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        flat.copy_(host)
    else:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    return ws


def allreduce_mean_(flat: torch.Tensor, group=None) -> None:
    """Average a flat gradient buffer across the data-parallel group in place."""
    ws = allreduce_sum_(flat, group)
    if ws > 1:
        flat.div_(ws)


def broadcast_params_(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Make every rank's parameters and buffers equal to rank ``src``'s (the
    replicas of data-parallel training start identical)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            if _host_staged(t, group):
                host = t.detach().cpu()
                dist.broadcast(host, src, group=group)
                t.copy_(host)
            else:
                dist.broadcast(t.data, src, group=group)


def make_adam(params, lr: float):
    """Adam(lr) as in 5_train_SpotV2Net.py:127, with the device-side step
    counter needed for graph capture (fused kernel when available)."""
    params = list(params)
    if not params[0].is_cuda:  # host-side replicas (gloo tests): plain Adam
        return torch.optim.Adam(params, lr=lr)
    try:
        return torch.optim.Adam(params, lr=lr, fused=True, capturable=True)
    except (RuntimeError, TypeError):
        return torch.optim.Adam(params, lr=lr, capturable=True, foreach=True)


class _Shape:
    """One captured batch shape of a TrainStep: its static data, the optional
    capturable ``prepare`` (e.g. WindowDataset.fill from an index buffer),
    its graphs and its loss output."""

    def __init__(self, data, prepare: Optional[Callable[[], None]]):
        self.data, self.prepare = data, prepare
        self.g_fb = self.g_opt = None
        self.loss: Optional[torch.Tensor] = None


class TrainStep:
    """One optimisation step over a static device-resident batch.

    ``data`` is read through ``data.x / edge_index / edge_attr / y_x``; for
    graph replay the same tensors must stay alive (refresh them in place, or
    pass ``prepare``: a capturable callable run at the start of every step that
    refills them, e.g. ``lambda: dataset.fill(data, idx_buffer)``).
    ``add_shape`` captures further batch shapes (a ragged last batch) that
    share the parameters, gradients and optimizer state.

    Constructing it applies no update: the warm-up steps before capture are
    undone (parameters, buffers, optimizer state, RNG).

    ``loss_sum``: a device scalar every step adds its loss to inside the
    captured step (the reference's per-epoch running loss,
    5_train_SpotV2Net.py:160-163, without an eager launch per step)."""

    def __init__(self, model: torch.nn.Module, data, lr: float = 1e-3,
                 loss_fn: Callable = torch.nn.functional.mse_loss, use_graph: bool = True,
                 group=None, warmup: int = 3, optimizer: str = "sv2n",
                 prepare: Optional[Callable[[], None]] = None,
                 loss_sum: Optional[torch.Tensor] = None, device_rng: bool = True,
                 dropout_seed: Optional[int] = None):
        self.model = model
        self.loss_sum = loss_sum
        self.loss_fn = loss_fn
        self.group = group
        self.warmup = warmup
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.flat_params = flatten_params(self.params)
        self.flat = flatten_grads(self.params)
        self.opt = FlatAdam(self.flat_params, self.flat, lr) if optimizer == "sv2n" \
            else make_adam(self.params, lr)
        # post-layer dropout uniforms keyed by (seed, Adam's device step
        # count, layer) (stack.device_dropout): no torch random op in the
        # captured step; device_rng=False keeps torch's generator
        self.device_rng = device_rng and isinstance(self.opt, FlatAdam)
        self.dropout_seed = int(torch.initial_seed() if dropout_seed is None else dropout_seed)
        self.distributed = dist.is_available() and dist.is_initialized() and \
            dist.get_world_size(group) > 1
        self.use_graph = use_graph
        self.loss = torch.zeros((), device=self.flat.device)
        self._one = torch.ones((), device=self.flat.device)
        # fused head + MSE (one launch, forward and backward) when the model offers it
        self._fused_mse = loss_fn is torch.nn.functional.mse_loss and hasattr(model, "mse_loss") \
            and hasattr(model, "_hidden") and hasattr(model, "linear")
        self._shapes = []
        self.add_shape(data, prepare)

    @property
    def data(self):
        return self._shapes[0].data

    def add_shape(self, data, prepare: Optional[Callable[[], None]] = None) -> int:
        """Capture the step for another static batch; returns its index for
        ``__call__(shape)``."""
        sh = _Shape(data, prepare)
        self._shapes.append(sh)
        if self.use_graph:
            self._capture(sh, self.warmup)
        return len(self._shapes) - 1

    # -- eager pieces -------------------------------------------------------
    def _fwd_bwd(self, sh: _Shape) -> None:
        from .stack import device_dropout
        if not self.device_rng:
            return self._fwd_bwd_inner(sh)
        with device_dropout(self.dropout_seed, self.opt.step_t):
            return self._fwd_bwd_inner(sh)

    def _fwd_bwd_inner(self, sh: _Shape) -> None:
        from .stack import direct_grad_accumulation, head_mse_train, head_mse_train_split
        if sh.prepare is not None:
            sh.prepare()
        if not getattr(self.opt, "zeroes_grads", False):
            self.flat.zero_()
        # every p.grad is a view of self.flat: the fused nodes accumulate into
        # it directly (no per-parameter AccumulateGrad launches)
        with direct_grad_accumulation():
            if self._fused_mse:
                # the output head and the loss inside the last GAT layer's
                # attention forward (stack.gat_train_head_mse) ...
                # (both add the loss to loss_sum in their own launch)
                loss = self.model._train_head_mse(sh.data, sh.data.y_x, self.loss_sum)
                if loss is not None:
                    sh.loss = loss.detach()
                    return
                # ... or head + loss forward AND backward (the upstream
                # gradient of the loss is 1), then the stack's backward: dx
                # first, the loss and head-gradient reduction after the backward
                h = self.model._hidden(sh.data)
                res = head_mse_train_split(h, self.model.linear, sh.data.y_x, self.loss_sum)
                if res is not None:
                    loss, dh, finish = res
                    torch.autograd.backward(h, dh)
                    finish()
                    sh.loss = loss.detach()
                    return
                res = head_mse_train(h, self.model.linear, sh.data.y_x, self.loss_sum)
                if res is not None:
                    loss, dh = res
                    torch.autograd.backward(h, dh)
                    sh.loss = loss.detach()
                    return
                loss = self.model.mse_loss(sh.data)
            else:
                loss = self.loss_fn(self.model(sh.data), sh.data.y_x)
            torch.autograd.backward(loss, self._one)
        sh.loss = loss.detach()
        self._accumulate(sh)

    def _accumulate(self, sh: _Shape) -> None:
        if self.loss_sum is not None:
            self.loss_sum.add_(sh.loss)

    def _opt_step(self) -> None:
        self.opt.step()

    def eager_step(self, sh: Optional[_Shape] = None) -> None:
        sh = sh or self._shapes[0]
        self._fwd_bwd(sh)
        if self.distributed:
            allreduce_mean_(self.flat, self.group)
        self._opt_step()
        self.loss = sh.loss

    # -- graph capture ------------------------------------------------------
    def _snapshot(self) -> dict:
        """Everything the warm-up steps before capture advance: parameters,
        module buffers (BatchNorm running statistics with ``standardize``),
        optimizer state, RNG streams."""
        snap = {"params": self.flat_params.clone(), "opt": None,
                "loss_sum": None if self.loss_sum is None else self.loss_sum.clone(),
                "buffers": [b.detach().clone() for b in self.model.buffers()],
                "cpu_rng": torch.get_rng_state(),
                "cuda_rng": torch.cuda.get_rng_state(self.flat.device)}
        if isinstance(self.opt, FlatAdam):
            snap["opt"] = (self.opt.m.clone(), self.opt.v.clone(), self.opt.step_t.clone())
        else:
            snap["opt"] = {id(p): {k: (v.clone() if torch.is_tensor(v) else v)
                                   for k, v in st.items()}
                           for p, st in self.opt.state.items()}
        return snap

    def _restore(self, snap: dict) -> None:
        """Undo the warm-up (in place: the captured graphs keep pointing at the
        same buffers), so that construction does not train the model."""
        with torch.no_grad():
            self.flat_params.copy_(snap["params"])
            if snap["loss_sum"] is not None:
                self.loss_sum.copy_(snap["loss_sum"])
            for b, old in zip(self.model.buffers(), snap["buffers"]):
                b.copy_(old)
            self.flat.zero_()
            if isinstance(self.opt, FlatAdam):
                m, v, t = snap["opt"]
                self.opt.m.copy_(m)
                self.opt.v.copy_(v)
                self.opt.step_t.copy_(t)
            else:  # torch.optim.Adam: state tensors back to their pre-warm-up values
                for p, st in self.opt.state.items():
                    old = snap["opt"].get(id(p))
                    for k, val in st.items():
                        if torch.is_tensor(val):
                            if old is not None and k in old:
                                val.copy_(old[k])
                            else:
                                val.zero_()
        torch.set_rng_state(snap["cpu_rng"])
        try:
            torch.cuda.set_rng_state(snap["cuda_rng"], self.flat.device)
        except RuntimeError:  # generator registered with a live capture
            pass

    def _capture(self, sh: _Shape, warmup: int) -> None:
        """Warm up (allocator, lazy optimizer state), capture, then restore the
        pre-warm-up parameters / buffers / optimizer state / RNG: constructing a
        TrainStep applies no update (k calls == k eager reference steps)."""
        snap = self._snapshot()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(max(1, warmup)):
                self.eager_step(sh)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if self.distributed:
            sh.g_fb = torch.cuda.CUDAGraph()
            with torch.cuda.graph(sh.g_fb):
                self._fwd_bwd(sh)
            # the ÷ world size of the all-reduced sum rides in the optimizer
            # graph (no eager launch between the collective and the replay)
            ws = dist.get_world_size(self.group)
            sh.g_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(sh.g_opt):
                self.flat.div_(ws)
                self._opt_step()
        else:
            sh.g_fb = torch.cuda.CUDAGraph()
            with torch.cuda.graph(sh.g_fb):
                self._fwd_bwd(sh)
                self._opt_step()
        torch.cuda.synchronize()
        self._restore(snap)
        torch.cuda.synchronize()

    def __call__(self, shape: int = 0) -> torch.Tensor:
        sh = self._shapes[shape]
        if not self.use_graph:
            self.eager_step(sh)
            return self.loss
        sh.g_fb.replay()
        if self.distributed:
            allreduce_sum_(self.flat, self.group)  # the mean's ÷ is inside g_opt
            sh.g_opt.replay()
        self.loss = sh.loss
        return self.loss


class ForwardStep:
    """Inference forward (eval mode, no grad) captured into a hipGraph.
    ``fn(model, data)`` is what runs (default ``model(data)``; e.g.
    ``lambda m, d: m.mse_loss(d)`` for the evaluation loss); ``prepare`` as in
    TrainStep."""

    def __init__(self, model: torch.nn.Module, data, use_graph: bool = True, warmup: int = 2,
                 fn: Optional[Callable] = None, prepare: Optional[Callable[[], None]] = None,
                 out_sum: Optional[torch.Tensor] = None):
        self.model, self.data = model, data
        self.out_sum = out_sum  # device scalar each call adds fn's (scalar) output to
        self.fn = fn or (lambda m, d: m(d))
        self.prepare = prepare
        self.out: Optional[torch.Tensor] = None
        self.graph = None
        saved = None if out_sum is None else out_sum.clone()
        with torch.no_grad():
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(max(1, warmup)):
                    self._run()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            if use_graph:
                self.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph):
                    self._run()
                torch.cuda.synchronize()
            if self.out_sum is not None:
                self.out_sum.copy_(saved)  # undo the warm-up and capture calls

    def _run(self) -> None:
        if self.prepare is not None:
            self.prepare()
        self.out = self.fn(self.model, self.data)
        if self.out_sum is not None:
            self.out_sum.add_(self.out)

    def __call__(self) -> torch.Tensor:
        if self.graph is None:
            with torch.no_grad():
                self._run()
        else:
            self.graph.replay()
        return self.out


# ---------------------------------------------------------------------------
# the reference's training loop (5_train_SpotV2Net.py:86-197) on the device
# ---------------------------------------------------------------------------
# device-memory budget of one captured test forward (Fit.eval_chunk): C3's
# 432 test windows (~2 MB each) stay one forward
EVAL_BYTES = int(os.environ.get("SV2N_EVAL_BYTES", 1 << 30))
# "off": Fit's bf16 batches keep x written beside its bf16 twin (A/B switch)
TWIN_ONLY = os.environ.get("SV2N_TWIN_ONLY", "on")


class Fit:
    """5_train_SpotV2Net.py's loop over a device-resident WindowDataset:
    train/test split ``int(split * len)`` (:86-88), DataLoader(shuffle=True)
    order for training and sequential order for testing (:90-91), per batch
    MSE + zero_grad + backward + Adam (:150-159), per epoch the mean batch
    loss of each phase (:163, :180), and the checkpoint rule (:186-191).

    The steps are hipGraph replays: the window gather (WindowDataset.fill from
    a device index buffer), forward, fused head + MSE, backward and Adam of
    one batch are ONE graph; the ragged last batch has its own graph; batch
    losses are summed on the device, so the host synchronises once per epoch
    (the reference calls loss.item() per batch, :160)."""

    def __init__(self, model: torch.nn.Module, dataset, batch_size: int, lr: float = 1e-3,
                 split: float = 0.8, generator: Optional[torch.Generator] = None,
                 use_graph: bool = True, optimizer: str = "sv2n",
                 step_hook: Optional[Callable[[int, int], None]] = None):
        self.model, self.ds, self.bs = model, dataset, int(batch_size)
        n = len(dataset)
        self.n_train = int(split * n)
        self.n_test = n - self.n_train
        dev = dataset.vol.device
        self.dev = dev
        self.gen = generator if generator is not None else torch.Generator()
        self.step_hook = step_hook
        self.use_graph = use_graph and step_hook is None
        self.epoch = 0
        self._idx = {}     # batch size -> static index buffer
        self._batch = {}   # batch size -> static Batch
        # the edge features are read only by the covariance-layout edge passes:
        # the gather writes just their columns (sv2n_window_gather_cv)
        from .stack import cov_var_edges_only
        self._cv_only = bool(not getattr(model, "standardize", False) and
                             cov_var_edges_only(list(model.gat_layers), dataset.n, dataset.S))
        self._bf16 = getattr(model, "precision", None) == "bf16"
        sizes = [self.bs] if self.n_train >= self.bs else []
        if self.n_train % self.bs:
            sizes.append(self.n_train % self.bs)
        self._train_shape = {}
        self.step = None
        # per-epoch loss sums, accumulated inside the captured steps
        self._tot_train = torch.zeros((), device=dev)
        self._tot_test = torch.zeros((), device=dev)
        model.train()  # the training graphs are captured in train mode (dropout on)
        for b in sizes:
            data, prep = self._static(b)
            if self.step is None:
                # a step_hook seeds torch's generator per step: its draws stay torch's
                self.step = TrainStep(model, data, lr=lr, use_graph=self.use_graph,
                                      optimizer=optimizer, prepare=prep,
                                      loss_sum=self._tot_train, device_rng=step_hook is None)
                self._train_shape[b] = 0
            else:
                self._train_shape[b] = self.step.add_shape(data, prep)
        self._eval = {}
        self.history: list = []
        self.best_test = float("inf")

    def _static(self, b: int):
        if b not in self._batch:
            self._idx[b] = torch.zeros(b, dtype=torch.long, device=self.dev)
            # the bf16 mode's layer-0 GEMMs read bf16(x) from the gather
            self._batch[b] = self.ds.empty_batch(
                b, bf16_x=self._bf16, cov_var_only=self._cv_only, twin_only=self._twin_only(b))
            self.ds.fill(self._batch[b], self._idx[b])
        data, idx = self._batch[b], self._idx[b]
        return data, (lambda: self.ds.fill(data, idx))

    def _twin_only(self, b: int) -> bool:
        """Whether a ``b``-window batch's x is gathered as its bf16 twin alone
        (data.WindowDataset.empty_batch(twin_only=True)): the bf16 mode, the
        covariance-layout edge passes (a canonical batch on the unfused
        attention) and a layer 0 that reads x only through the twin
        (stack.twin_only_ok); SV2N_TWIN_ONLY=off keeps x written."""
        from .stack import twin_only_ok
        return bool(TWIN_ONLY == "on" and self._bf16 and self._cv_only and
                    twin_only_ok(list(self.model.gat_layers), b * self.ds.n))

    def _window_bytes(self) -> int:
        """Device bytes one test window costs in the captured test forward:
        x (and its bf16 twin), edge_attr, and per layer xs, y and the layer
        output (an upper bound: the gather may write fewer edge columns)."""
        n, S = self.ds.n, self.ds.S
        b = 6 * n * n * S + 4 * n * (n - 1) * 3 * S
        for c in self.model.gat_layers:
            b += 3 * 4 * n * (c.heads * c.out_channels + 2 * c.heads)
        return b

    def eval_chunk(self) -> int:
        """Test windows per captured test forward: every test window in one
        forward while that fits EVAL_BYTES, else the largest multiple of the
        batch size that does (at least one batch), so the test pass's memory
        is bounded by the budget, not by the test split."""
        nb = -(-self.n_test // self.bs)
        k = max(1, min(nb, EVAL_BYTES // max(1, self._window_bytes() * self.bs)))
        return min(self.n_test, k * self.bs)

    def _eval_pass(self):
        """The test pass (5_train_SpotV2Net.py:166-180: sequential batches of
        ``bs``, each batch's MSE added up) as captured forwards over chunks of
        ``eval_chunk()`` test windows (normally one chunk: all of them): the
        graphs are independent and eval mode draws no dropout, so each window's
        output is the one its batch would give, and each batch's loss is its
        own row slice's mean (one fused head + MSE launch per batch, added to
        the epoch's test sum in batch order; chunks are multiples of the batch
        size, so batch boundaries never straddle a chunk).  Returns
        ({chunk size: (ForwardStep, index buffer)}, chunk, test indices)."""
        if "all" not in self._eval:
            n_test, bs = self.n_test, self.bs
            chunk = self.eval_chunk()
            all_idx = torch.arange(self.n_train, self.n_train + n_test, device=self.dev)
            steps = {}
            for size in dict.fromkeys([chunk] + ([n_test % chunk] if n_test % chunk else [])):
                # buffers of its own (a training shape of the same size refills
                # its index buffer every step)
                idx = all_idx[:size].clone()
                data = self.ds.empty_batch(
                    size, bf16_x=self._bf16, cov_var_only=self._cv_only,
                    twin_only=self._twin_only(size))
                self.ds.fill(data, idx)
                rows = data.x.shape[0] // size  # nodes per window
                tot = self._tot_test

                def fn(m, d, size=size, rows=rows, tot=tot):
                    from .stack import head_mse_loss
                    h = m._hidden(d)
                    y = d.y_x.view(size * rows, -1)
                    for k in range(0, size, bs):
                        b = min(bs, size - k)
                        head_mse_loss(h[k * rows:(k + b) * rows], m.linear,
                                      y[k * rows:(k + b) * rows].reshape(-1), tot)
                    return tot

                was = self.model.training
                self.model.eval()
                saved = self._tot_test.clone()
                steps[size] = (ForwardStep(self.model, data, use_graph=self.use_graph, fn=fn,
                                           prepare=(lambda data=data, idx=idx:
                                                    self.ds.fill(data, idx))), idx)
                self._tot_test.copy_(saved)  # undo the warm-up and capture calls
                self.model.train(was)
            self._eval["all"] = (steps, chunk, all_idx)
        return self._eval["all"]

    def _test_pass(self) -> None:
        """Adds every test batch's loss to _tot_test, chunk by chunk in order."""
        steps, chunk, all_idx = self._eval_pass()
        for k0 in range(0, self.n_test, chunk):
            size = min(chunk, self.n_test - k0)
            step, idx = steps[size]
            if chunk < self.n_test:  # one chunk: its index buffer never changes
                idx.copy_(all_idx[k0:k0 + size])
            step()

    def run_epoch(self, checkpoint_path: Optional[str] = None, tolerance: float = 1e-9) -> dict:
        """One epoch: training pass, test pass, history entry (and checkpoint)."""
        dev = self.dev
        perm = torch.randperm(self.n_train, generator=self.gen).to(dev, non_blocking=True)
        self._tot_train.zero_()
        self.model.train()
        nb = 0
        for k in range(0, self.n_train, self.bs):
            b = min(self.bs, self.n_train - k)
            self._idx[b].copy_(perm[k:k + b])
            if self.step_hook is not None:
                self.step_hook(self.epoch, nb)
            self.step(self._train_shape[b])   # adds its loss to _tot_train
            nb += 1
        nt = -(-self.n_test // self.bs)   # test batches
        self._tot_test.zero_()   # an empty test split reports 0, not the last epoch's sum
        self.model.eval()
        if self.n_test > 0:
            self._test_pass()   # adds every test batch's loss to _tot_test
        self.model.train()
        train_loss = float(self._tot_train) / max(nb, 1)   # one host sync per epoch
        test_loss = float(self._tot_test) / max(nt, 1)
        rec = {"epoch": self.epoch + 1, "train_loss": train_loss, "test_loss": test_loss,
               "train_rmse": train_loss ** 0.5, "test_rmse": test_loss ** 0.5}
        if checkpoint_path is not None and (self.epoch == 0 or
                                            test_loss + tolerance < self.best_test):
            torch.save({k: v.detach().clone() for k, v in self.model.state_dict().items()},
                       checkpoint_path)
        if self.epoch == 0 or test_loss + tolerance < self.best_test:
            self.best_test = test_loss
        self.history.append(rec)
        self.epoch += 1
        return rec


def fit(model: torch.nn.Module, dataset, num_epochs: int, batch_size: int, lr: float = 1e-3,
        split: float = 0.8, generator: Optional[torch.Generator] = None, use_graph: bool = True,
        checkpoint_path: Optional[str] = None, tolerance: float = 1e-9,
        step_hook: Optional[Callable[[int, int], None]] = None) -> list:
    """Train like 5_train_SpotV2Net.py:139-197 and return the per-epoch history
    (train/test loss and RMSE).  See ``Fit``."""
    f = Fit(model, dataset, batch_size, lr, split, generator, use_graph, step_hook=step_hook)
    for _ in range(num_epochs):
        f.run_epoch(checkpoint_path, tolerance)
    return f.history
