"""CPU stand-in for StyleEngine, for the CPU tests of bench.py's launcher and rank logic
(tests/test_distributed.py).  It implements the engine surface bench.py and AdamLoop call
(embeds / set_targets / loss_grad / adam_step_dev / range flags / timing) with a small deterministic
per-clip problem, so a clip's result depends only on its own inputs: the multi-rank result can
be compared clip by clip with a single-process one."""
from __future__ import annotations

import torch


class StubEngine:
    def __init__(self, batch, T, cont_ids, style_ids, precision='split', device=None,
                 lambd=100.0, gatys=False, **kw):
        if device is None or torch.device(device).type != 'cpu':
            raise RuntimeError('StubEngine is the CPU stand-in (device cpu)')
        self.batch, self.T, self.device = int(batch), int(T), torch.device(device)
        self.lambd = float(lambd)
        self._t = None
        self.calls = 0

    def embeds(self, x, content=True, style=True):
        B = x.shape[0]
        emb_c = (x / 128.0)[..., None].repeat(1, 1, 4) if content else None
        s = torch.stack([x.mean(1), x.std(1), x.abs().mean(1), x.max(1).values], 1)
        emb_s = (s[:, :, None] * s[:, None, :])[:, None] if style else None
        return emb_c, emb_s.reshape(B, 1, 4, 4) if style else None

    def set_targets(self, phi_c, phi_s):
        self._t = (phi_c[..., 0] * 128.0, phi_s)

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
