"""Drop-in for the reference's ``optimal_transport.py`` (ADMM optimal transport between NMF
palettes, optimal_transport.py:22-162): the same function names, arguments and float64 results,
computed on the GPU by ``ast_ot_admm`` (csrc/ot_admm.hip: one workgroup per problem runs the
whole ADMM loop).  ``ot_admm_batched`` solves many palette pairs of one shape in one launch.

numpy in, numpy out, as the reference (device tensors are accepted too and stay on the device).
The reference's only caller is ``utils.transform`` (utils.py:132-145, NMF + compute_permutation),
which nothing calls."""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def _dev(device=None):
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise _lib.AstError('optimal_transport runs on the GPU (ast_ot_admm); no device visible')
    return torch.device('cuda', torch.cuda.current_device())


def _as_dev(a, device):
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=torch.float64).contiguous()
    return torch.as_tensor(np.asarray(a, dtype=np.float64), device=device).contiguous()


MAX_CELLS = 1 << 16    # n1 * n2 per problem (ast_ot_admm)


def ot_admm_batched(p_mod, p_ref, eps=1e-4, miter=1e5, palette=True, device=None):
    """p_mod [B, n1, d], p_ref [B, n2, d] -> (plans [B, n1, n2], palettes [B, n1, d] or None,
    iterations [B]) as device tensors; one OT_ADMM + transform_palette per pair.

    Size limit: n1 * n2 <= 2^16 cells (MAX_CELLS; e.g. 256 x 256) and n1 + n2 <= 20000.  The
    reference's OT_ADMM has no limit, but one problem runs on one workgroup whose ADMM iteration
    streams ~80 B per cell, so 2^16 cells already take seconds per solve and 2^26 (the round-3
    limit) would take hours; larger palettes raise ValueError here (the C ABI: AST_E_ARG)."""
    n1, n2 = int(p_mod.shape[-2]), int(p_ref.shape[-2])
    if n1 * n2 > MAX_CELLS or n1 + n2 > 20000:
        raise ValueError('ot_admm_batched: %d x %d palettes exceed the solver limit n1 * n2 <= %d '
                         '(and n1 + n2 <= 20000)' % (n1, n2, MAX_CELLS))
    lib = _lib.load()
    dev = p_mod.device if isinstance(p_mod, torch.Tensor) and p_mod.is_cuda else _dev(device)
    a = _as_dev(p_mod, dev)
    b = _as_dev(p_ref, dev)
    if a.dim() != 3 or b.dim() != 3 or a.shape[0] != b.shape[0] or a.shape[2] != b.shape[2]:
        raise ValueError('need p_mod [B, n1, d] and p_ref [B, n2, d], got %s and %s'
                         % (tuple(a.shape), tuple(b.shape)))
    B, n1, d = a.shape
    n2 = b.shape[1]
    plan = torch.empty(B, n1, n2, dtype=torch.float64, device=dev)
    pal = torch.empty(B, n1, d, dtype=torch.float64, device=dev) if palette else None
    its = torch.empty(B, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream().cuda_stream
        _lib.check(lib.ast_ot_admm(a.data_ptr(), b.data_ptr(), B, n1, n2, d, float(eps),
                                   float(miter), plan.data_ptr(),
                                   pal.data_ptr() if palette else None, its.data_ptr(), stream))
    return plan, pal, its


def _host(t, like):
    return t if isinstance(like, torch.Tensor) else t.cpu().numpy()


def OT_ADMM(palette2Mod, paletteRef, eps=1e-4, miter=1e5, verbose=False):
    """optimal_transport.py:77-137: the transport plan [n1, n2].  (``verbose``: the reference
    prints residuals every 100 iterations; here the iteration count is printed at the end.)"""
    plan, _, its = ot_admm_batched(_as_batch(palette2Mod), _as_batch(paletteRef), eps, miter,
                                   palette=False)
    if verbose:
        print('OT_ADMM: %d iterations' % int(its[0]))
    return _host(plan[0], palette2Mod)


def compute_permutation(W1, W2):
    """optimal_transport.py:151-162: W2's palette transported onto W1's, [n1, d]."""
    _, pal, _ = ot_admm_batched(_as_batch(W1), _as_batch(W2))
    return _host(pal[0], W1)


def transform_palette(palette_orig, palette_target, Transport):
    """optimal_transport.py:140-148: Transport palette_target / (row sums + 1e-10), on the
    device (one matmul and one division; palette_orig is unused, as in the reference)."""
    dev = _dev()
    t = _as_dev(Transport, dev)
    p = _as_dev(palette_target, dev)
    out = (t @ p) / (t.sum(1) + 1e-10)[:, None]
    return _host(out, Transport)


def build_moving_cost_matrix(palette1, palette2):
    """optimal_transport.py:22-37: Euclidean distances between the palettes' rows, squared
    feature differences accumulated in feature order (on the device)."""
    dev = _dev()
    a = _as_dev(palette1, dev)
    b = _as_dev(palette2, dev)
    c = torch.zeros(a.shape[0], b.shape[0], dtype=torch.float64, device=dev)
    for k in range(a.shape[1]):
        c += (a[:, k, None] - b[None, :, k]) ** 2
    return _host(torch.sqrt(c), palette1)


def projection_sum_equal(X0, target_value):
    """optimal_transport.py:40-47."""
    x = _as_dev(X0, _dev())
    return _host(x + (target_value - x.sum()) / x.numel(), X0)


def projection_column_sum_in_range(X0, bounds):
    """optimal_transport.py:50-74: rows whose sum leaves [min(bounds_i), max(bounds_i)] are
    shifted onto the nearest bound."""
    dev = _dev()
    x = _as_dev(X0, dev)
    bd = _as_dev(bounds, dev)
    lo, hi = bd.min(1).values, bd.max(1).values
    s = x.sum(1)
    corr = torch.where(s < lo, (lo - s) / x.shape[1], torch.zeros_like(s))
    corr = torch.where(s > hi, (hi - s) / x.shape[1], corr)
    return _host(x + corr[:, None], X0)


def _as_batch(a):
    if isinstance(a, torch.Tensor):
        return a[None]
    return np.asarray(a, dtype=np.float64)[None]
