"""Fused gradient clipping + Adam for the training step (train_visual.py:533, :575-577;
train_audio.py:21, :40-44): ``clip_grad_norm_(params, max_norm)`` followed by
``torch.optim.Adam(params, lr, betas, eps, weight_decay)`` in two HIP launches over a chunk
table of every parameter (csrc/optim.hip), with the clip coefficient kept on the device.

A ``torch.optim.Optimizer``: ``param_groups`` (so ReduceLROnPlateau / OneCycleLR adjust
``lr``), per-parameter ``state`` with torch Adam's keys (``step``, ``exp_avg``,
``exp_avg_sq``; checkpoints interchange with torch.optim.Adam), ``zero_grad``,
``state_dict`` / ``load_state_dict``, and ``GradScaler.step`` (which unscales the grads
of ``param_groups`` before calling ``step``).  As torch Adam, parameters whose ``grad`` is
None are skipped, so a backbone that is frozen when the optimiser is built (the
reference's first three epochs, train_visual.py:547-553) starts training when it is
unfrozen.

Same update as torch's Adam (L2 weight decay, bias correction from each parameter's own
step count, no amsgrad / maximize).  With ``max_norm`` the gradients are clipped to that
total norm inside the update; ``param.grad`` keeps the unclipped gradient and ``step()``
returns the pre-clip total norm as a fresh 0-d device tensor (clip_grad_norm_'s return).
Without ``max_norm`` the script's own clip_grad_norm_ call does the clipping (as the
reference scripts do) and ``step()`` returns None.

``capturable=True`` (torch Adam's flag of that name): the step counts live on the device,
incremented and turned into the bias corrections there (xcp_opt_adam_dev), so the step can be
captured in a HIP graph and replayed -- no host arithmetic, no host sync.  Parameters whose counts
are equal share one 0-d device counter (``state["step"]`` is that tensor), so a group normally costs
one Adam launch.  Which parameters share a counter is decided on the host, without a device read,
so that torch Adam's per-parameter semantics hold: a parameter whose state is created after its group has stepped (a backbone
unfrozen after epoch 3, train_visual.py:547-556), a parameter whose grad is None on a step while its
counter-mates step, and a loaded state whose count differs from the others each get a counter of
their own (one more launch), never the group's count.
"""
import math

import torch
from torch.autograd.graph import increment_version

from . import _lib, ops

CHUNK = 16384


class FusedAdamClip(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_norm=None,
                 capturable=False):
        if lr < 0.0 or eps < 0.0 or weight_decay < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("FusedAdamClip: invalid hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        for grp in self.param_groups:
            for p in grp["params"]:
                if p.dtype != torch.float32 or not p.is_contiguous():
                    raise ValueError("FusedAdamClip: fp32 contiguous parameters only")
                ops.check_gpu(p)
        self.max_norm = max_norm
        self.capturable = capturable
        self._counters = {}   # capturable: id(device step counter) -> the counter
        self._tables = {}
        self._out = None

    def _state(self, p, counter=None):
        st = self.state[p]
        if not st:
            st["step"] = counter if self.capturable else torch.tensor(0.0)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    @staticmethod
    def _key(kind, rows):
        """cache key of a chunk table: every pointer a row of it holds (param, grad and both
        moment buffers), so a replaced state tensor (load_state_dict, a re-zeroed moment) or a
        re-attached gradient can never reuse a table that points at the old storage"""
        return (kind,) + tuple((p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel())
                               for p, g, m, v in rows)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._tables.clear()   # the moment buffers were replaced

    def _table(self, key, rows, dev):
        """device chunk table for a list of (param, grad, exp_avg, exp_avg_sq), cached by pointers"""
        tab = self._tables.get(key)
        if tab is None:
            r = []
            for p, g, m, v in rows:
                if g.dtype != torch.float32 or not g.is_contiguous():
                    raise ValueError("FusedAdamClip: fp32 contiguous gradients only")
                n = p.numel()
                for s in range(0, n, CHUNK):
                    r.append([p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), s, min(CHUNK, n - s)])
            tab = torch.tensor(r, dtype=torch.int64).to(dev)
            if len(self._tables) > 64:
                self._tables.clear()
            self._tables[key] = tab
        return tab

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self.capturable:
            return self._step_capturable(loss)
        # parameters with a gradient, grouped by (param group, step count) for the bias corrections
        launches, every = [], []
        for gi, grp in enumerate(self.param_groups):
            by_step = {}
            for p in grp["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdamClip does not support sparse gradients")
                st = self._state(p)
                st["step"] += 1
                row = (p, p.grad, st["exp_avg"], st["exp_avg_sq"])
                by_step.setdefault(int(st["step"].item()), []).append(row)
                every.append(row)
            for t, rows in by_step.items():
                launches.append((grp, t, rows))
        if not every:
            return loss
        dev = every[0][0].device
        with ops.device_guard(every[0][0]):
            s = ops.stream()
            coef = 0
            if self.max_norm is not None:
                tab = self._table(self._key("all", every), every, dev)
                part = torch.empty(tab.shape[0], device=dev, dtype=torch.float32)
                self._out = torch.empty(2, device=dev, dtype=torch.float32)
                _lib.call("xcp_opt_sumsq", tab.data_ptr(), tab.shape[0], part.data_ptr(), float(self.max_norm),
                          self._out.data_ptr(), s)
                coef = self._out.data_ptr()
            for grp, t, rows in launches:
                tab = self._table(self._key("grp", rows), rows, dev)
                b1, b2 = grp["betas"]
                _lib.call("xcp_opt_adam", tab.data_ptr(), tab.shape[0], coef, float(grp["lr"]), float(b1), float(b2),
                          float(grp["eps"]), float(grp["weight_decay"]), float(1.0 - b1 ** t),
                          float(math.sqrt(1.0 - b2 ** t)), s)
        # the kernels wrote the parameters through raw pointers: bump their autograd version
        # counters as an in-place torch op would, so that consumers keyed on them (the xcp
        # engine's packed-weight cache, engine.pack) see the update
        increment_version([row[0] for row in every])
        if loss is not None:
            return loss
        return self._out[1].clone() if self.max_norm is not None else None

    def _counter(self, value, device=None):
        """a new device step counter: a fresh one holding the host number `value`, or a copy of the
        device counter `value`.  Never inside a graph capture: the replay would re-run the fill /
        copy, so the count would restart on every replay"""
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("FusedAdamClip(capturable=True): the set of parameters with gradients changed "
                               "inside a graph capture; run one eager step with the captured structure first")
        if torch.is_tensor(value):
            t = value.clone()
        else:
            t = torch.full((), float(value), device=device, dtype=torch.float32)
        self._counters[id(t)] = t
        return t

    def _step_capturable(self, loss):
        """step() with the step counts on the device: per distinct counter, t += 1 on the device,
        then one Adam launch reading t (no .item(), no host-side bias corrections).  Counters are
        regrouped on the host by which parameters hold them (never by reading a count), so that every
        parameter's count is its own number of steps, as in torch Adam: a fresh state starts a fresh
        counter at 0, a loaded state joins a counter of its own count, and a counter whose parameters
        do not all step this time is split (a device copy) before the stepping ones advance it."""
        launches, every = [], []
        for gi, grp in enumerate(self.param_groups):
            stepping = []
            fresh = None
            for p in grp["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdamClip does not support sparse gradients")
                if not self.state[p]:
                    if fresh is None:
                        fresh = self._counter(0, p.device)
                    self._state(p, fresh)
                stepping.append(p)
            # adopt loaded (host / foreign) step tensors: one shared counter per distinct count
            adopted = {}
            for p in grp["params"]:
                st = self.state.get(p)
                if not st or id(st["step"]) in self._counters:
                    continue
                v = int(float(st["step"]))
                if v not in adopted:
                    adopted[v] = self._counter(v, p.device)
                st["step"] = adopted[v]
            # group the stepping parameters by counter; split counters whose other members skip
            members = {}
            for p in grp["params"]:
                if p in self.state and self.state[p]:
                    members.setdefault(id(self.state[p]["step"]), set()).add(p)
            by_counter = {}
            for p in stepping:
                by_counter.setdefault(id(self.state[p]["step"]), []).append(p)
            for cid, ps in by_counter.items():
                t = self._counters[cid]
                if len(ps) != len(members[cid]):
                    t = self._counter(t)
                    for p in ps:
                        self.state[p]["step"] = t
                rows = [(p, p.grad, self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"]) for p in ps]
                launches.append((grp, t, rows))
                every.extend(rows)
        # forget counters no parameter holds any more
        live = {id(st["step"]) for st in self.state.values() if st and "step" in st}
        for cid in [c for c in self._counters if c not in live]:
            del self._counters[cid]
        if not every:
            return loss
        dev = every[0][0].device
        with ops.device_guard(every[0][0]):
            s = ops.stream()
            coef = 0
            if self.max_norm is not None:
                tab = self._table(self._key("all", every), every, dev)
                part = torch.empty(tab.shape[0], device=dev, dtype=torch.float32)
                self._out = torch.empty(2, device=dev, dtype=torch.float32)
                _lib.call("xcp_opt_sumsq", tab.data_ptr(), tab.shape[0], part.data_ptr(), float(self.max_norm),
                          self._out.data_ptr(), s)
                coef = self._out.data_ptr()
            for grp, t, rows in launches:
                t.add_(1.0)
                tab = self._table(self._key("grp", rows), rows, dev)
                b1, b2 = grp["betas"]
                _lib.call("xcp_opt_adam_dev", tab.data_ptr(), tab.shape[0], coef, float(grp["lr"]), float(b1), float(b2),
                          float(grp["eps"]), float(grp["weight_decay"]), t.data_ptr(), s)
        increment_version([row[0] for row in every])
        if loss is not None:
            return loss
        return self._out[1].clone() if self.max_norm is not None else None
