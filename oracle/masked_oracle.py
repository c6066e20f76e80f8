"""CPU ORACLE — TEST INFRASTRUCTURE ONLY: the fp64 oracle evaluated on a given relu pattern.

Imported by tests/ and tools/diag only (never by the product path).  Restates
astyle_oracle.encoder_forward / encoder_backward (model.py:80-127) with the relu decisions
optionally forced.

The encoder is piecewise linear in its relu decisions (model.py:96-116: relu(e_l) before the
dilated conv, relu(u_l) before the 1x1).  A run in finite precision picks one side of every
near-zero decision; where it picks the other side than the fp64 oracle, the gradient jumps by
that decision's whole contribution, whatever the arithmetic precision.  Forcing the fp64 oracle
onto a run's relu pattern separates the two error sources of a gradient:

    |g_run - g_fp64|  <=  |g_run - g_fp64[run masks]|  (arithmetic on the run's linear piece)
                        + |g_fp64[run masks] - g_fp64|  (the relu-decision lottery)

Masks are lists me[l] = (e_l > 0), mu[l] = (u_l > 0) of [T, C] booleans, l = 0..n_blocks-1.
"""
from __future__ import annotations

import numpy as np

from . import astyle_oracle as O


def forward(x, W, n_blocks=30, me=None, mu=None, dtype=np.float64):
    """encoder_forward with optional forced relu masks; returns extracts, cache, (me, mu)."""
    x = np.asarray(x, dtype=dtype)
    e = O.conv1d_same((x / 128.0)[:, None], W['ae_startconv/W'].astype(dtype),
                      W['ae_startconv/biases'].astype(dtype), 1)
    es, us, ext, me_out, mu_out = [e], [], [], [], []
    for l in range(n_blocks):
        d = O.dilation_of(l)
        m_e = (e > 0) if me is None else me[l]
        u = O.conv1d_same(e * m_e, W['ae_dilatedconv_%d/W' % (l + 1)].astype(dtype),
                          W['ae_dilatedconv_%d/biases' % (l + 1)].astype(dtype), d)
        m_u = (u > 0) if mu is None else mu[l]
        y = O.conv1d_same(u * m_u, W['ae_res_%d/W' % (l + 1)].astype(dtype),
                          W['ae_res_%d/biases' % (l + 1)].astype(dtype), 1)
        e = e + y
        es.append(e)
        us.append(u)
        ext.append(e)
        me_out.append(m_e)
        mu_out.append(m_u)
    if n_blocks == O.N_BLOCKS:
        ext.append(e)
    return ext, {'es': es, 'us': us, 'n_blocks': n_blocks}, (me_out, mu_out)


def backward(cache, masks, W, ext_grads, dtype=np.float64):
    es, n_blocks = cache['es'], cache['n_blocks']
    me, mu = masks
    T = es[0].shape[0]
    g = np.zeros((T, O.C), dtype=dtype)
    if 30 in ext_grads:
        g += ext_grads[30]
    for l in reversed(range(n_blocks)):
        if l in ext_grads:
            g = g + ext_grads[l]
        gv = O.conv1d_same_bwd(g, W['ae_res_%d/W' % (l + 1)].astype(dtype), 1)
        gh = O.conv1d_same_bwd(gv * mu[l], W['ae_dilatedconv_%d/W' % (l + 1)].astype(dtype),
                               O.dilation_of(l))
        g = g + gh * me[l]
    gxs = O.conv1d_same_bwd(g, W['ae_startconv/W'].astype(dtype), 1)
    return gxs[:, 0] / 128.0


def loss_and_grad(x, W, *, cont_ids, style_ids, phi_c, phi_s, lambd=100.0, me=None, mu=None,
                  nb_channels=128, cnt_channels=128, dtype=np.float64):
    """O.loss_and_grad (ours Gram, gamma = 0, no bottleneck tap) on forced masks."""
    nb = O.needed_blocks(cont_ids, style_ids)
    ext, cache, masks = forward(x, W, nb, me, mu, dtype)
    content, style, grads = O.tap_terms(ext, cont_ids=cont_ids, style_ids=style_ids,
                                        phi_c=phi_c, phi_s=phi_s, lambd=lambd,
                                        nb_channels=nb_channels, cnt_channels=cnt_channels)
    g = backward(cache, masks, W, grads, dtype)
    return np.array([content + lambd * style, content, style, 0.0]), g, ext, masks


def masks_from_extracts(x, W, ext_run, n_blocks=30, e0_mode='fma'):
    """The relu pattern a run used, reconstructed from its extracts (e_1 .. e_n, fp32):
    me[l] = e_l > 0 from the run's own e_l (l >= 1); me[0] from e_0 formed in fp32 as the
    kernels form it (e0_val, common.h: fma(w2, xp/128, fma(w1, x0/128, w0 * xm/128)) + b);
    mu[l] = u_l > 0 for u_l formed in fp64 from the run's e_l (the run's own u differs from that
    by one GEMM's rounding, ~2^-22 relative, so the few decisions inside that band are the
    approximation of this reconstruction)."""
    x = np.asarray(x, np.float64)
    T = x.shape[0]
    w0 = W['ae_startconv/W'][0].astype(np.float32)          # [3, 1, C]
    b0 = W['ae_startconv/biases'].astype(np.float32)
    xs = (x.astype(np.float32) * np.float32(0.0078125)).astype(np.float32)
    xm = np.concatenate([[0], xs[:-1]]).astype(np.float32)[:, None]
    xp = np.concatenate([xs[1:], [0]]).astype(np.float32)[:, None]
    x0 = xs[:, None]

    def fma32(a, b, c):
        # fp32 fma: the product of two fp32 values is exact in fp64 (48 bits); the fp64 sum
        # then rounds twice (to fp64, to fp32), which differs from one rounding only at ties
        return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)
    if e0_mode == 'fma':
        e0 = fma32(w0[2, 0][None], xp, fma32(w0[1, 0][None], x0, (w0[0, 0][None] * xm).astype(np.float32)))
        e0 = (e0 + b0[None]).astype(np.float32)
    else:
        e0 = (O.conv1d_same(x[:, None] / 128.0, W['ae_startconv/W'], W['ae_startconv/biases'], 1))
    es = [e0.astype(np.float64)] + [np.asarray(ext_run[l], np.float64) for l in range(n_blocks - 1)]
    me, mu = [], []
    for l in range(n_blocks):
        m_e = es[l] > 0
        u = O.conv1d_same(es[l] * m_e, W['ae_dilatedconv_%d/W' % (l + 1)],
                          W['ae_dilatedconv_%d/biases' % (l + 1)], O.dilation_of(l))
        me.append(m_e)
        mu.append(u > 0)
    return me, mu


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(np.asarray(b)))


def flips(masks_a, masks_b):
    """Per-layer counts of relu decisions that differ: (e flips, u flips)."""
    return ([int(np.count_nonzero(a != b)) for a, b in zip(masks_a[0], masks_b[0])],
            [int(np.count_nonzero(a != b)) for a, b in zip(masks_a[1], masks_b[1])])
