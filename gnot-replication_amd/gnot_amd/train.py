"""The training step around the GNOT path on the GPU.

* `RelL2Loss` -- reference loss.py:14-23 (`RelL2Loss()(g, pred, tgt)`, dgl SumPooling over the
  batched graph) restated over packed offsets: `RelL2Loss()(x_off, pred, tgt)`.  One native pass
  (libgnot_hip.so gnot_rel_l2_loss) computes the per-sample segment sums, the loss and d loss/d pred.
* `OneCycle` -- torch's OneCycleLR (main.py:52: max_lr=1e-3, steps_per_epoch, epochs; cosine,
  two phases, cycle_momentum -> AdamW's beta1) as host arithmetic.  Calling `step()` once per
  EPOCH reproduces the reference's call pattern (main.py:106) although the schedule is sized per
  batch, so the LR stays near max_lr / 25; calling it per batch is the intended OneCycle.
* `FlatAdamW` -- torch.optim.AdamW (main.py:51, default betas/eps/weight_decay) over ONE flat fp32
  arena: the model's parameters are re-homed into a single buffer laid out exactly like the engine's
  gradient arena, so the whole update is one kernel (gnot_adamw_step) reading the step's flat
  gradient buffer directly.  The hyper-parameters live in a small device array that `prepare()`
  refreshes from the host schedule, so `launch()` can be captured in a hipGraph.
"""
import ctypes
import math

import torch

from . import _lib


# ------------------------------------------------------------------ loss (loss.py:14-23)
class _RelL2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, tgt, off_dev, off_host, work):
        lib = _lib.load()
        B = len(off_host) - 1
        C = pred.shape[1]
        loss = torch.empty((), device=pred.device, dtype=torch.float32)
        dpred = torch.empty_like(pred) if pred.requires_grad else None
        oh = (ctypes.c_int64 * (B + 1))(*off_host)
        s = ctypes.c_void_p(torch.cuda.current_stream(pred.device).cuda_stream)
        _lib.check(lib.gnot_rel_l2_loss(pred.data_ptr(), tgt.data_ptr(), off_dev.data_ptr(), oh, B, C,
                                        work.data_ptr(), loss.data_ptr(),
                                        dpred.data_ptr() if dpred is not None else None, s))
        ctx.save_for_backward(dpred) if dpred is not None else None
        return loss

    @staticmethod
    def backward(ctx, g):
        (dpred,) = ctx.saved_tensors
        return dpred * g, None, None, None, None


class RelL2Loss(torch.nn.Module):
    """mean over (sample, channel) of sqrt(sum_n (p - t)^2 / sum_n t^2) (reference loss.py:14-23).
    The dgl graph argument of the reference becomes the packed offsets x_off [B+1] (host list)."""

    def __init__(self):
        super().__init__()
        self._cache = {}

    def forward(self, x_off, predictions, targets):
        if not predictions.is_cuda:
            raise RuntimeError("gnot_amd.RelL2Loss runs on a ROCm GPU only (libgnot_hip.so)")
        key = (tuple(int(v) for v in x_off), predictions.shape[1], predictions.device)
        if key not in self._cache:
            B = len(key[0]) - 1
            oh = (ctypes.c_int64 * (B + 1))(*key[0])
            n = _lib.load().gnot_rel_l2_work_floats(oh, B, key[1])
            # pinned source + non_blocking: a new geometry must not stall the host on the stream
            # (a pageable copy would); the pinned tensor lives in the cache entry past the copy
            pinned = torch.tensor(key[0], dtype=torch.int64).pin_memory()
            self._cache = {key: (pinned.to(predictions.device, non_blocking=True),
                                 torch.empty(n, dtype=torch.float32, device=predictions.device), pinned)}
        off_dev, work, _ = self._cache[key]
        return _RelL2.apply(predictions.contiguous().float(), targets.contiguous().float(), off_dev, key[0], work)


# ------------------------------------------------------------------ OneCycleLR (main.py:52)
class OneCycle:
    """torch.optim.lr_scheduler.OneCycleLR(max_lr, total_steps = epochs * steps_per_epoch) defaults:
    pct_start 0.3, cosine annealing, div_factor 25, final_div_factor 1e4, cycle_momentum with
    base/max momentum 0.85/0.95 applied to AdamW's beta1."""

    def __init__(self, max_lr, epochs, steps_per_epoch, pct_start=0.3, div_factor=25.0, final_div_factor=1e4,
                 base_momentum=0.85, max_momentum=0.95):
        self.total = epochs * steps_per_epoch
        self.max_lr = max_lr
        self.initial_lr = max_lr / div_factor
        self.min_lr = self.initial_lr / final_div_factor
        self.phases = [(float(pct_start * self.total) - 1, self.initial_lr, max_lr, max_momentum, base_momentum),
                       (self.total - 1, max_lr, self.min_lr, base_momentum, max_momentum)]
        self.last = 0          # OneCycleLR.__init__ performs the first step(): last_epoch = 0

    @staticmethod
    def _cos(start, end, pct):
        return end + (start - end) / 2.0 * (math.cos(math.pi * pct) + 1)

    def values(self, step=None):
        """(lr, beta1) at scheduler step `step` (default: the current one)."""
        s = self.last if step is None else step
        start = 0.0
        for i, (end, lr0, lr1, m0, m1) in enumerate(self.phases):
            if s <= end or i == len(self.phases) - 1:
                pct = (s - start) / (end - start)
                return self._cos(lr0, lr1, pct), self._cos(m0, m1, pct)
            start = end
        raise AssertionError

    def step(self):
        self.last += 1


# ------------------------------------------------------------------ AdamW (main.py:51)
def flatten_parameters(model):
    """Re-home every Linear's weight/bias into ONE device buffer laid out like the engine's gradient
    arena (W0, b0, W1, b1, ... in canonical order).  Parameters keep their identity (only .data
    moves), so existing optimizers and state_dict() are unaffected.  Returns the flat buffer."""
    lins = model.linears()
    dev = lins[0].weight.device
    total = sum(l.weight.numel() + l.bias.numel() for l in lins)
    flat = torch.empty(total, dtype=torch.float32, device=dev)
    o = 0
    with torch.no_grad():
        for l in lins:
            for p in (l.weight, l.bias):
                n = p.numel()
                flat[o:o + n].copy_(p.reshape(-1))
                p.data = flat[o:o + n].view(p.shape)
                o += n
    model._engine = None        # parameter pointers moved: rebind
    return flat


class FlatAdamW:
    """torch.optim.AdamW(params, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2) on a flat arena.
    grad: the flat gradient buffer of the step (Engine.grad_flat, same layout as `flat`)."""

    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, schedule=None):
        self.flat = flat
        self.m = torch.zeros_like(flat)
        self.v = torch.zeros_like(flat)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.schedule = schedule
        self.t = 0
        self.hyper = torch.zeros(8, dtype=torch.float32, device=flat.device)
        # pinned staging ring: the host may run steps ahead of the GPU; a slot is rewritten only
        # after the copy that last read it has executed (its event)
        self._ring = [torch.zeros(8, dtype=torch.float32).pin_memory() for _ in range(4)]
        self._ev = [None] * 4

    def prepare(self):
        """Advance the step count and write this step's hyper-parameters to the device array."""
        self.t += 1
        lr, b1 = (self.lr, self.betas[0]) if self.schedule is None else self.schedule.values()
        b2 = self.betas[1]
        k = self.t % len(self._ring)
        if self._ev[k] is not None:
            self._ev[k].synchronize()
        h = self._ring[k]
        for i, val in enumerate((lr, b1, b2, self.eps, self.wd, 1 - b1 ** self.t, 1 - b2 ** self.t, 1.0)):
            h[i] = val
        self.hyper.copy_(h, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ev[k] = ev

    def launch(self, grad):
        """The update kernel only (graph-capturable)."""
        if grad.numel() != self.flat.numel():
            raise ValueError("gradient buffer does not match the parameter arena")
        s = ctypes.c_void_p(torch.cuda.current_stream(self.flat.device).cuda_stream)
        _lib.check(_lib.load().gnot_adamw_step(self.flat.data_ptr(), grad.data_ptr(), self.m.data_ptr(),
                                               self.v.data_ptr(), self.flat.numel(), self.hyper.data_ptr(), s))

    def step(self, grad):
        self.prepare()
        self.launch(grad)


# ------------------------------------------------------------------ driver (main.py:55-153)
def save_checkpoint(model, path):
    """torch.save(model.state_dict()) exactly as main.py:151 (reference-compatible keys/shapes)."""
    torch.save(model.state_dict(), path)


def load_checkpoint(model, path):
    """Load a reference (or gnot_amd) state_dict checkpoint; tensors only (weights_only=True)."""
    model.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
    return model


def _to(batch, dev):
    return (batch["x"].to(dev), batch["x_off"], batch["theta"].to(dev), [f.to(dev) for f in batch["fns"]],
            batch["fn_offs"], batch["y"].to(dev))


def _forward_batch(model, batch, dev):
    """(prediction [sum N, out], packed offsets, target) of one batch.  Packed batches (collate_packed)
    go through forward_packed; padded batches (collate_padded) through the reference calling
    convention `model(x, theta, input_functions)` (main.py:84) and are un-padded with the real point
    counts (main.py:87-89) -- the pad rows still enter the attention sums, exactly as in main.py."""
    if "counts" in batch:
        x = batch["x"].to(dev)
        fns = batch["fns"].to(dev) if batch["fns"] is not None else None
        out = model(x, batch["theta"].to(dev), fns)
        counts = batch["counts"]
        pred = torch.cat([out[b, :n] for b, n in enumerate(counts)])
        off = [0]
        for n in counts:
            off.append(off[-1] + n)
        return pred, off, batch["y"].to(dev)
    x, x_off, theta, fns, fn_offs, y = _to(batch, dev)
    return model.forward_packed(x, x_off, theta, fns, fn_offs), x_off, y


def evaluate(model, loader, loss_fn=None):
    """main.py:108-147: mean RelL2 over the test batches, no_grad (no activations kept).  Batches from
    collate_padded reproduce main.py's padded evaluation; collate_packed batches the unpadded one."""
    loss_fn = loss_fn or RelL2Loss()
    dev = next(model.parameters()).device
    vals = []
    with torch.no_grad():
        for batch in loader:
            pred, off, y = _forward_batch(model, batch, dev)
            vals.append(float(loss_fn(off, pred, y)))
    return sum(vals) / max(len(vals), 1)


def fit(model, train_loader, test_loader=None, epochs=100, lr=1e-3, per_epoch_schedule=True, checkpoint=None,
        log=print):
    """The reference training loop (main.py:50-153): AdamW(lr) + OneCycleLR(max_lr=lr, steps_per_epoch,
    epochs), RelL2 loss, per-epoch test metric and best checkpoint.  With per_epoch_schedule=True the
    schedule is stepped once per epoch, as main.py:106 does.  The loaders decide the batch form:
    collate_padded batches run main.py's zero-padded semantics (pad rows in the attention sums),
    collate_packed batches the packed (per-sample exact) one.
    Returns (train losses per epoch, test metrics per epoch)."""
    flat = flatten_parameters(model)
    sched = OneCycle(lr, epochs, len(train_loader))
    opt = FlatAdamW(flat, lr=lr, schedule=sched)
    dev = flat.device
    eng = model.engine()
    prev = eng.param_grads
    eng.param_grads = False          # FlatAdamW reads the gradient arena; no .grad copies
    loss_fn = RelL2Loss()
    best, hist_train, hist_test = float("inf"), [], []
    try:
        for epoch in range(epochs):
            losses = []
            for batch in train_loader:
                pred, off, y = _forward_batch(model, batch, dev)
                loss = loss_fn(off, pred, y)
                loss.backward()
                opt.step(eng.grad_flat)
                if not per_epoch_schedule:
                    sched.step()
                losses.append(float(loss))
            if per_epoch_schedule:
                sched.step()
            hist_train.append(sum(losses) / max(len(losses), 1))
            log(f"Epoch {epoch}, Loss: {hist_train[-1]}")
            if test_loader is not None:
                res = evaluate(model, test_loader, loss_fn)
                hist_test.append(res)
                log(f"Epoch {epoch}, Test Metric: {res}")
                if res < best and checkpoint:
                    best = res
                    save_checkpoint(model, checkpoint)
    finally:
        eng.param_grads = prev       # ordinary autograd use after fit() gets .grad again
    return hist_train, hist_test
