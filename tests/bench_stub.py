"""CPU stand-ins for StyleEngine and LbfgsLoop, for the CPU tests of bench.py's and the batch
CLI's launcher and rank logic (tests/test_distributed.py, tests/test_batch.py).  StubEngine
implements the engine surface bench.py, AdamLoop, GatysNet and the batch mode call (embeds /
set_targets / set_gamma / loss_grad / adam_step_dev / range flags / timing) with a small
deterministic per-clip problem, so a clip's result depends only on its own inputs: the
multi-rank result can be compared clip by clip with a single-process one.  LbfgsLoop drives
scipy's L-BFGS-B per active clip through the same interface as engine.LbfgsLoop (minimize /
state / parts / history; begin(x0) restarts every clip of the loop, as ast_lbfgs_begin does).
IllCondStubEngine: a problem that keeps clips running over epochs, and scheduled range flags
for the batch CLI's fp32 fallback."""
from __future__ import annotations

import os

import numpy as np
import torch


class StubEngine:
    def __init__(self, batch, T, cont_ids, style_ids, precision='split', device=None,
                 lambd=100.0, gatys=False, **kw):
        if device is None or torch.device(device).type != 'cpu':
            raise RuntimeError('StubEngine is the CPU stand-in (device cpu)')
        self.batch, self.T, self.device = int(batch), int(T), torch.device(device)
        self.lambd = float(lambd)
        self.precision = precision
        self.gamma = 0.0
        self.style_shape = (1, 4, 4)
        self._t = None
        self.calls = 0

    def embeds(self, x, content=True, style=True):
        B = x.shape[0]
        emb_c = (x / 128.0)[..., None].repeat(1, 1, 4) if content else None
        s = torch.stack([x.mean(1), x.std(1), x.abs().mean(1), x.max(1).values], 1)
        emb_s = (s[:, :, None] * s[:, None, :])[:, None] if style else None
        return emb_c, emb_s.reshape(B, 1, 4, 4) if style else None

    def set_targets(self, phi_c, phi_s):
        phi_c = torch.as_tensor(phi_c, dtype=torch.float32)
        if phi_c.dim() == 2:
            phi_c = phi_c[None].expand(self.batch, -1, -1)
        self._t = (phi_c[..., 0] * 128.0, phi_s)

    def set_gamma(self, gamma):
        self.gamma = float(gamma)

    def loss_grad(self, x, grad=None, parts=None):
        d = x - self._t[0]
        if grad is None:
            grad = torch.empty_like(x)
        if parts is None:
            parts = torch.empty(self.batch, 4)
        grad.copy_(2.0 * d / self.T)
        c = (d * d).mean(1)
        parts[:, 0] = c
        parts[:, 1] = c
        parts[:, 2] = 0.0
        parts[:, 3] = 0.0
        self.calls += 1
        return parts, grad

    def adam_step_dev(self, x, m, v, grad, step_dev, lr=1.0, beta1=0.9, beta2=0.999, eps=1e-8):
        step_dev += 1
        k = int(step_dev.item())
        m.mul_(beta1).add_((1 - beta1) * grad)
        v.mul_(beta2).add_((1 - beta2) * grad * grad)
        x.sub_(lr * (m / (1 - beta1 ** k)) / ((v / (1 - beta2 ** k)).sqrt() + eps))

    def reset_range_flags(self):
        self._flags = torch.zeros(self.batch, dtype=torch.int32)

    def range_flags(self, reset=False):
        f = getattr(self, '_flags', torch.zeros(self.batch, dtype=torch.int32)).clone()
        if reset:
            self.reset_range_flags()
        return f

    def timing(self, enable):
        if enable:
            self.calls = 0

    def timing_read(self):
        c = float(max(self.calls, 1))
        return {'block_fwd_ms': 30 * c, 'block_bwd_ms': 30 * c, 'gram_fwd_ms': c,
                'gram_bwd_ms': c, 'other_ms': c, 'calls': c, 'blocks': 30.0}

    def close(self):
        pass


class IllCondStubEngine(StubEngine):
    """StubEngine with an ill-conditioned per-clip problem, mean(w (x - target)^2) with w spread
    over five decades, so an L-BFGS-B epoch (maxiter 100) uses more than 50 evaluations and a
    clip keeps going from epoch to epoch (methods.py:180-181); and range flags on a schedule:
    STUB_RANGE_FLAGS="b:k,..." raises RANGE_ACT for local clip b in the k-th minimize call
    (0-based) of a split-precision engine, as a real split context would after an out-of-range
    evaluation.  Its results do not depend on the precision."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self._w = torch.logspace(-5, 0, self.T)
        self.minimize_calls = 0
        spec = os.environ.get('STUB_RANGE_FLAGS', '')
        self._sched = [tuple(int(v) for v in item.split(':')) for item in spec.split(',') if item]

    def loss_grad(self, x, grad=None, parts=None):
        d = x - self._t[0]
        if grad is None:
            grad = torch.empty_like(x)
        if parts is None:
            parts = torch.empty(self.batch, 4)
        grad.copy_(2.0 * self._w * d / self.T)
        c = (self._w * d * d).mean(1)
        parts[:, 0] = c
        parts[:, 1] = c
        parts[:, 2] = 0.0
        parts[:, 3] = 0.0
        self.calls += 1
        return parts, grad

    def end_minimize(self, active):
        if self.precision == 'split':
            for b, k in self._sched:
                if k == self.minimize_calls and active[b]:
                    self._flags = self.range_flags()
                    self._flags[b] |= 2                      # RANGE_ACT
        self.minimize_calls += 1


class LbfgsLoop:
    """engine.LbfgsLoop's interface (minimize / state / parts) over StubEngine: scipy L-BFGS-B
    (maxiter, default options) per active clip, the other clips' points held fixed."""

    def __init__(self, eng, m=10, maxiter=100, **kw):
        self.eng, self.maxiter = eng, int(maxiter)
        self.x64 = torch.zeros(eng.batch, eng.T, dtype=torch.float64)
        self.parts = torch.zeros(eng.batch, 4)
        self.info = np.zeros((eng.batch, 4), np.int32)
        self.hist = [np.zeros((0, 4))] * eng.batch

    def minimize(self, x0=None, active=None, **kw):
        from scipy.optimize import minimize
        eng = self.eng
        if x0 is not None:
            self.x64 = torch.as_tensor(x0, dtype=torch.float64).clone()
        act = np.ones(eng.batch, bool) if active is None else np.asarray(active).astype(bool)
        self.info[:] = 0
        self.hist = [np.zeros((0, 4))] * eng.batch
        if hasattr(eng, 'reset_range_flags'):
            eng.reset_range_flags()                 # begin() starts a new epoch's flags
        for b in np.flatnonzero(act):
            base = self.x64.float()
            h = []

            def fg(v, b=b, h=h):
                x = base.clone()
                x[b] = torch.from_numpy(v.astype(np.float32))
                parts, grad = eng.loss_grad(x)
                self.parts[b] = parts[b]
                h.append(parts[b].double().numpy())
                return float(parts[b, 0]), grad[b].double().numpy()

            res = minimize(fg, self.x64[b].float().double().numpy(), jac=True, method='L-BFGS-B',
                           options={'maxiter': self.maxiter})
            self.x64[b] = torch.from_numpy(res.x)
            self.info[b] = (0, res.nit, res.nfev, 1)
            self.hist[b] = np.array(h).reshape(-1, 4)
        if hasattr(eng, 'end_minimize'):
            eng.end_minimize(act)
        return self.info.copy()

    def history(self, info=None):
        return [h.copy() for h in self.hist]

    def state(self, with_x=False):
        return self.info.copy(), (self.x64.clone() if with_x else None)
