"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.  Independent torch-autograd restatement of the
reference loss: imported by tests/ (it pins astyle_oracle.py's hand-derived gradient) and timed
by bench.py's cpu_baseline leg (the reference's TF-CPU path is not runnable here: no TF).

Written separately from ``oracle/astyle_oracle.py`` (channels-first ``F.conv1d`` with
symmetric ``padding=dilation``, autograd instead of hand-written backward, ``torch.stft``)
so that agreement between the two pins the oracle's hand-derived gradient.
Follows model.py:80-127, methods.py:58-76 and 113-125, utils.py:92-104.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def _w(W, name, dtype):
    return torch.as_tensor(np.asarray(W[name]), dtype=dtype)


def _conv(x, Whwio, b, d):
    # x [1, Cin, T]; HWIO [1, K, Cin, Cout] -> OIK [Cout, Cin, K]
    w = Whwio[0].permute(2, 1, 0).contiguous()
    k = w.shape[2]
    return F.conv1d(x, w, b, padding=((k - 1) // 2) * d, dilation=d)


def _abs_tf(v):
    return torch.clamp(v, min=1e-12) + torch.clamp(-v, min=0.0)


def _inv_mu_law_tf(x, mu=255):
    o = (x + 0.5) * 2.0 / (mu + 1)
    sgn = torch.where(o.abs() <= 1e-12, torch.zeros_like(o), o) / _abs_tf(o)
    out = sgn / mu * ((1 + mu) ** _abs_tf(o) - 1)
    return torch.where(x == 0, x, out)


def loss_fn(x, W, *, cont_ids, style_ids, phi_c, phi_s, lambd=100.0, gamma=0.0, gatys=False,
            nb_channels=128, cnt_channels=128, n_blocks=30, dtype=torch.float64):
    """x: torch [T] (requires_grad).  Returns (total, content, style, reg)."""
    h = (x / 128.0)[None, None, :].to(dtype)
    e = _conv(h, _w(W, 'ae_startconv/W', dtype), _w(W, 'ae_startconv/biases', dtype), 1)
    ext = []                                              # extracts as [C, T] (conv1d layout)
    for l in range(n_blocks):
        d = 2 ** (l % 10)
        u = _conv(torch.relu(e), _w(W, 'ae_dilatedconv_%d/W' % (l + 1), dtype),
                  _w(W, 'ae_dilatedconv_%d/biases' % (l + 1), dtype), d)
        e = e + _conv(torch.relu(u), _w(W, 'ae_res_%d/W' % (l + 1), dtype),
                      _w(W, 'ae_res_%d/biases' % (l + 1), dtype), 1)
        ext.append(e[0])                                  # [C, T]
    if n_blocks == 30:
        ext.append(ext[-1])
        bott = _conv(e, _w(W, 'ae_bottleneck/W', dtype), _w(W, 'ae_bottleneck/biases', dtype), 1)
        ext.append(bott[0])
    # methods.py:58: content taps [T, n cnt] (kept transposed: [n cnt, T])
    emb = torch.cat([ext[i][:cnt_channels] for i in cont_ids], dim=0)
    content = 10.0 * torch.mean((emb - torch.as_tensor(phi_c, dtype=dtype).T) ** 2)
    # methods.py:60-73: ours G_c = E_c E_c^T over [C, L, T]; Gatys G_l = F_l F_l^T over [L, C, T]
    stl = torch.stack([ext[i] for i in style_ids], 0)     # [L, C, T]
    s = stl.permute(1, 0, 2).contiguous() if not gatys else stl
    G = s @ s.transpose(1, 2)
    ss = (G * G).sum(dim=(1, 2), keepdim=True)
    Gn = G * torch.rsqrt(torch.clamp(ss, min=1e-12))
    if nb_channels < 128 and not gatys:
        Gn = Gn[:nb_channels]
    style = 1e3 * torch.mean((Gn - torch.as_tensor(phi_s, dtype=dtype)) ** 2)
    a = _inv_mu_law_tf(x.to(dtype))
    S = torch.stft(a, n_fft=1024, hop_length=512, win_length=1024,
                   window=torch.hann_window(1024, periodic=True, dtype=dtype),
                   center=False, return_complex=True)     # [513, frames]
    reg = torch.mean(_abs_tf(S.real) + _abs_tf(S.imag))
    total = content + lambd * style + gamma * reg
    return total, content, style, reg


def cpu_step(x, W, *, cont_ids, style_ids, phi_c, phi_s, lambd=100.0, gatys=False,
             dtype=torch.float32):
    """One loss+grad evaluation of one clip (the reference's CPU path restated: fp32 conv1d
    forward, autograd backward to x).  Returns (total, grad [T])."""
    xt = torch.as_tensor(x, dtype=dtype).detach().clone().requires_grad_(True)
    total, _, _, _ = loss_fn(xt, W, cont_ids=cont_ids, style_ids=style_ids, phi_c=phi_c,
                             phi_s=phi_s, lambd=lambd, gatys=gatys, dtype=dtype)
    g, = torch.autograd.grad(total, xt)
    return float(total.detach()), g


def stft_reg(x):
    """The regulariser alone (methods.py:121-123) for x [B, T] -> (value [B], d value / d x)
    by torch.stft + autograd."""
    x = torch.as_tensor(x).detach().clone().requires_grad_(True)
    S = torch.stft(_inv_mu_law_tf(x), n_fft=1024, hop_length=512, win_length=1024,
                   window=torch.hann_window(1024, periodic=True, dtype=x.dtype),
                   center=False, return_complex=True)
    reg = (_abs_tf(S.real) + _abs_tf(S.imag)).mean(dim=(-2, -1))
    g, = torch.autograd.grad(reg.sum(), x)
    return reg.detach(), g
