"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

This module is a plain-numpy restatement of the reference's style-transfer hot path
(winlp4ever/audio_style_transfer).  It is the checker, never the product: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``audio_style_transfer_amd``) never routes through it.

Parity status
-------------
* mu-law codecs (``mu_law_numpy`` / ``inv_mu_law_numpy``) and the output-path naming are
  PINNED: ``tests/golden/make_golden.py`` executes the reference's own pure-numpy functions
  (utils.py:18-90) in the build container and commits their outputs as fixtures.
* encoder / Gram / loss / gradient: **parity unpinned** against the reference itself.
  The reference computes them with TensorFlow 1.x (absent in this image; no network) and
  ships no tests, golden vectors or checkpoint.  They are pinned instead by
  (i) fp64 central finite differences of this oracle's own loss, and (ii) agreement with an
  independent torch-autograd restatement (tests/test_oracle.py).

Every function cites the reference file:line it restates.  Arrays are channels-last
``[T, C]`` per clip (the reference's ``[1, T, C]`` with the batch-of-one dropped).
"""
from __future__ import annotations

import numpy as np

MU = 255
C = 128                  # ae_width, model.py:77
N_BLOCKS = 30            # ae_num_layers, model.py:75
N_STAGES = 10            # ae_num_stages, model.py:74
K = 3                    # ae_filter_length, model.py:76
BOTTLENECK = 16          # ae_bottleneck_width, model.py:23


# ----------------------------------------------------------------------------------------
# mu-law codecs (utils.py:79-104)
# ----------------------------------------------------------------------------------------
def mu_law_numpy(x, mu=MU):
    """utils.py:79-82 — floor(128*sign(x)*ln(1+mu|x|)/ln(1+mu))."""
    out = np.sign(x) * np.log(1 + mu * np.abs(x)) / np.log(1 + mu)
    return np.floor(out * 128)


def inv_mu_law_numpy(x, mu=float(MU)):
    """utils.py:85-90 — note the +0.5 offset and the x==0 -> 0 passthrough."""
    x = np.array(x).astype(np.float32)
    out = (x + 0.5) * 2. / (mu + 1)
    out = np.sign(out) / mu * ((1 + mu) ** np.abs(out) - 1)
    return np.where(np.equal(x, 0), x, out)


def _abs_tf(v):
    """utils.py:92-93 — abs(v) = max(v, 1e-12) + max(0, -v)."""
    return np.maximum(v, 1e-12) + np.maximum(0.0, -v)


def _abs_tf_grad(v):
    # TF Maximum routes the gradient to its first input where x >= y.
    return (v >= 1e-12).astype(v.dtype) - (v < 0).astype(v.dtype)


def inv_mu_law_tf(x, mu=MU):
    """utils.py:95-104 (TF version used by the regulariser) -> (value, d value / d x)."""
    o = (x + 0.5) * 2. / (mu + 1)
    do = 2. / (mu + 1)
    a = _abs_tf(o)
    da = _abs_tf_grad(o)
    num = np.where(np.abs(o) <= 1e-12, 0.0, o)
    dnum = np.where(np.abs(o) <= 1e-12, 0.0, 1.0)
    sgn = num / a
    dsgn = (dnum * a - num * da) / (a * a)
    p = (1 + mu) ** a
    dp = p * np.log(1 + mu) * da
    out = sgn / mu * (p - 1)
    dout = (dsgn * (p - 1) + sgn * dp) / mu * do
    zero = np.equal(x, 0)
    return np.where(zero, x, out), np.where(zero, 1.0, dout)


# ----------------------------------------------------------------------------------------
# conv primitive (nsynth/wavenet/masked.py:110-160)
# ----------------------------------------------------------------------------------------
def conv1d_same(x, W, b, dilation=1):
    """masked.conv1d with causal=False.

    time_to_batch (masked.py:57-86) + conv2d 'SAME' (masked.py:139,154) + batch_to_time
    (masked.py:89-107) is, for T % dilation == 0 (asserted at masked.py:134), the symmetric
    dilated cross-correlation  y[t] = b + sum_k W[k]^T x[t + (k - (K-1)//2) * d]  with zeros
    outside [0, T).  ``W`` is HWIO [1, K, Cin, Cout] (masked.py:136).
    """
    T = x.shape[0]
    assert T % dilation == 0, "masked.py:134"
    Wk = W[0]
    Kf = Wk.shape[0]
    pad = (Kf - 1) // 2                     # TF SAME: left = (K-1)//2
    y = np.broadcast_to(b, (T, Wk.shape[2])).astype(x.dtype).copy()
    for k in range(Kf):
        s = (k - pad) * dilation
        if s == 0:
            y += x @ Wk[k]
        elif s > 0:
            y[:T - s] += x[s:] @ Wk[k]
        else:
            y[-s:] += x[:T + s] @ Wk[k]
    return y


def conv1d_same_bwd(gy, W, dilation=1):
    """d/dx of conv1d_same for upstream gy (weights frozen: var_list=[x], methods.py:135)."""
    T = gy.shape[0]
    Wk = W[0]
    Kf = Wk.shape[0]
    pad = (Kf - 1) // 2
    gx = np.zeros((T, Wk.shape[1]), dtype=gy.dtype)
    for k in range(Kf):
        s = (k - pad) * dilation
        Wt = Wk[k].T
        if s == 0:
            gx += gy @ Wt
        elif s > 0:
            gx[s:] += gy[:T - s] @ Wt
        else:
            gx[:T + s] += gy[-s:] @ Wt
    return gx


def relu(v):
    return np.maximum(v, 0)


# ----------------------------------------------------------------------------------------
# encoder (model.py:79-127)
# ----------------------------------------------------------------------------------------
def dilation_of(block):
    """model.py:98 — 2 ** (layer % ae_num_stages)."""
    return 2 ** (block % N_STAGES)


def encoder_forward(x, W, n_blocks=N_BLOCKS, need_bottleneck=False, dtype=np.float64):
    """model.py:80-127.  x: [T] in mu-law units (the optimised variable, methods.py:49-54).

    Returns (extracts, cache).  ``extracts[l]`` = output of block l (model.py:116); when all
    30 blocks run, extracts[30] is extracts[29] (model.py:118-119) and extracts[31] is the
    1x1 bottleneck (model.py:121-127).
    """
    x = np.asarray(x, dtype=dtype)
    xs = (x / 128.0)[:, None]                                       # model.py:82-83
    e = conv1d_same(xs, W['ae_startconv/W'].astype(dtype),
                    W['ae_startconv/biases'].astype(dtype), 1)      # model.py:88-93
    es, us = [e], []
    extracts = []
    for l in range(n_blocks):                                       # model.py:96-116
        d = dilation_of(l)
        h = relu(e)
        u = conv1d_same(h, W['ae_dilatedconv_%d/W' % (l + 1)].astype(dtype),
                        W['ae_dilatedconv_%d/biases' % (l + 1)].astype(dtype), d)
        v = relu(u)
        y = conv1d_same(v, W['ae_res_%d/W' % (l + 1)].astype(dtype),
                        W['ae_res_%d/biases' % (l + 1)].astype(dtype), 1)
        e = e + y
        es.append(e)
        us.append(u)
        extracts.append(e)
    if n_blocks == N_BLOCKS:
        extracts.append(e)                                           # model.py:118-119
        if need_bottleneck:
            extracts.append(conv1d_same(e, W['ae_bottleneck/W'].astype(dtype),
                                        W['ae_bottleneck/biases'].astype(dtype), 1))
    return extracts, {'es': es, 'us': us, 'n_blocks': n_blocks}


def encoder_backward(cache, W, ext_grads, dtype=np.float64):
    """Backprop d loss / d x given d loss / d extracts[i] (dict i -> [T, C])."""
    es, us, n_blocks = cache['es'], cache['us'], cache['n_blocks']
    T = es[0].shape[0]
    g = np.zeros((T, C), dtype=dtype)
    if 31 in ext_grads:
        g += conv1d_same_bwd(ext_grads[31], W['ae_bottleneck/W'].astype(dtype), 1)
    if 30 in ext_grads:
        g += ext_grads[30]
    for l in reversed(range(n_blocks)):
        if l in ext_grads:
            g = g + ext_grads[l]
        d = dilation_of(l)
        gv = conv1d_same_bwd(g, W['ae_res_%d/W' % (l + 1)].astype(dtype), 1)
        gu = gv * (us[l] > 0)
        gh = conv1d_same_bwd(gu, W['ae_dilatedconv_%d/W' % (l + 1)].astype(dtype), d)
        g = g + gh * (es[l] > 0)
    gxs = conv1d_same_bwd(g, W['ae_startconv/W'].astype(dtype), 1)
    return gxs[:, 0] / 128.0


# ----------------------------------------------------------------------------------------
# taps, Gram, l2-normalise (methods.py:58-76)
# ----------------------------------------------------------------------------------------
def style_layer_ids(stack=None, style_lyr_ids=None):
    """methods.py:60-66."""
    if style_lyr_ids is not None:
        return list(style_lyr_ids)
    if stack is not None:
        return list(range(stack * 10, stack * 10 + 10))
    return list(range(30))


def needed_blocks(cont_ids, style_ids):
    """Blocks that must run for the fetched taps (TF prunes the rest)."""
    top = max(list(cont_ids) + list(style_ids))
    return N_BLOCKS if top >= 29 else top + 1


def content_embeds(extracts, cont_ids, cnt_channels):
    """methods.py:58 — concat_i extracts[i][:, :cnt_channels] along channels."""
    return np.concatenate([extracts[i][:, :cnt_channels] for i in cont_ids], axis=1)


def gram(extracts, style_ids, gatys=False):
    """methods.py:62-73.  ours: [C, L, L] (G[c] = E_c E_c^T); Gatys: [L, C, C]."""
    stl = np.stack([extracts[i] for i in style_ids], axis=0)         # [L, T, C]
    if not gatys:
        s = np.ascontiguousarray(np.transpose(stl, (2, 0, 1)))        # [C, L, T]
    else:
        s = np.ascontiguousarray(np.transpose(stl, (0, 2, 1)))        # [L, C, T]
    return s @ np.ascontiguousarray(np.transpose(s, (0, 2, 1)))


def l2_normalize(G, eps=1e-12):
    """tf.nn.l2_normalize(axis=(1,2)) (methods.py:74): G * rsqrt(max(sum G^2, eps))."""
    ss = np.sum(G * G, axis=(1, 2), keepdims=True)
    return G / np.sqrt(np.maximum(ss, eps))


def l2_normalize_bwd(G, dGn, eps=1e-12):
    ss = np.sum(G * G, axis=(1, 2), keepdims=True)
    inv = 1.0 / np.sqrt(np.maximum(ss, eps))
    Gn = G * inv
    big = (ss >= eps).astype(G.dtype)                                 # Maximum -> first input
    dot = np.sum(Gn * dGn, axis=(1, 2), keepdims=True)
    return dGn * inv - big * Gn * dot * inv


def style_embeds(extracts, style_ids, gatys=False, nb_channels=C):
    """methods.py:68-76 (incl. truncation to the first nb_channels matrices, ours only)."""
    Gn = l2_normalize(gram(extracts, style_ids, gatys))
    if nb_channels < C and not gatys:
        Gn = Gn[:nb_channels]
    return Gn


# ----------------------------------------------------------------------------------------
# STFT regulariser (methods.py:121-123)
# ----------------------------------------------------------------------------------------
FRAME, HOP = 1024, 512


def _hann_periodic(n):
    return 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n) / n)


def stft_reg(x):
    """gamma term: mean(abs(Re S) + abs(Im S)), S = stft(inv_mu_law(x), 1024, 512)
    (tf.contrib.signal.stft defaults: periodic Hann, fft_length 1024, pad_end False)."""
    a, da_dx = inv_mu_law_tf(np.asarray(x, dtype=np.float64))
    T = a.shape[0]
    nf = 1 + (T - FRAME) // HOP
    idx = np.arange(FRAME)[None, :] + HOP * np.arange(nf)[:, None]
    w = _hann_periodic(FRAME)
    S = np.fft.rfft(a[idx] * w, n=FRAME, axis=1)                      # [nf, 513]
    re, im = S.real, S.imag
    N = re.size
    val = np.mean(_abs_tf(re) + _abs_tf(im))
    gre = _abs_tf_grad(re) / N
    gim = _abs_tf_grad(im) / N
    # Re S_k = sum_n w a cos(2pi kn/N),  Im S_k = -sum_n w a sin(2pi kn/N)
    n = np.arange(FRAME)
    k = np.arange(FRAME // 2 + 1)
    ang = 2 * np.pi * np.outer(k, n) / FRAME
    gframe = (gre @ np.cos(ang) - gim @ np.sin(ang)) * w              # [nf, FRAME]
    ga = np.zeros(T)
    np.add.at(ga, idx, gframe)
    return val, ga * da_dx


# ----------------------------------------------------------------------------------------
# loss + grad (methods.py:113-125) and the evaluation ScipyOptimizerInterface performs
# ----------------------------------------------------------------------------------------
def loss_and_grad(x, W, *, cont_ids, style_ids, phi_c, phi_s, lambd=100.0, gamma=0.0,
                  gatys=False, nb_channels=C, cnt_channels=C, dtype=np.float64):
    """One loss+grad evaluation (methods.py:113-125 + tf.gradients inside
    ScipyOptimizerInterface, methods.py:133-137,167).  Returns
    (parts = [total, content, style, reg], grad[T])."""
    nb = needed_blocks(cont_ids, style_ids)
    ext, cache = encoder_forward(x, W, nb, need_bottleneck=31 in cont_ids, dtype=dtype)
    T = ext[0].shape[0]
    content, style, grads = tap_terms(ext, cont_ids=cont_ids, style_ids=style_ids, phi_c=phi_c,
                                      phi_s=phi_s, lambd=lambd, gatys=gatys,
                                      nb_channels=nb_channels, cnt_channels=cnt_channels)
    g = encoder_backward(cache, W, grads, dtype=dtype)
    # TF evaluates the regulariser whatever gamma is (methods.py:121-125); its gradient
    # enters only through gamma.
    reg, greg = stft_reg(x) if x.shape[0] >= FRAME else (0.0, np.zeros(T))
    if gamma != 0.0:
        g = g + gamma * greg
    total = content + lambd * style + gamma * reg
    return np.array([total, content, style, reg]), g


def tap_terms(ext, *, cont_ids, style_ids, phi_c, phi_s, lambd=100.0, gatys=False,
              nb_channels=C, cnt_channels=C):
    """Content and style terms of methods.py:116-119 and their gradients w.r.t. the extracts
    (dict extract id -> [T, width]; the style part already scaled by lambd)."""
    T = ext[0].shape[0]
    dtype = ext[0].dtype
    grads = {}
    # content: 10 * mean((emb - phi_c)^2)                            methods.py:116-117
    emb = content_embeds(ext, cont_ids, cnt_channels)
    diff = emb - phi_c
    content = 10.0 * np.mean(diff * diff)
    gemb = 10.0 * 2.0 * diff / diff.size
    off = 0
    for i in cont_ids:
        w = ext[i].shape[1] if i == 31 else C
        ncol = min(cnt_channels, w)
        gi = np.zeros((T, w), dtype=dtype)
        gi[:, :ncol] = gemb[:, off:off + ncol]
        grads[i] = grads.get(i, 0) + gi
        off += ncol
    # style: 1e3 * mean((Gn - phi_s)^2)                              methods.py:118-119
    G = gram(ext, style_ids, gatys)
    Gn_full = l2_normalize(G)
    Gn = Gn_full[:nb_channels] if (nb_channels < C and not gatys) else Gn_full
    sdiff = Gn - phi_s
    style = 1e3 * np.mean(sdiff * sdiff)
    dGn = np.zeros_like(Gn_full)
    dGn[:Gn.shape[0]] = lambd * 1e3 * 2.0 * sdiff / sdiff.size
    dG = l2_normalize_bwd(G, dGn)
    S = dG + np.transpose(dG, (0, 2, 1))
    stl = np.stack([ext[i] for i in style_ids], axis=0)              # [L, T, C]
    if not gatys:   # dstl[i,t,c] = sum_j S[c,i,j] stl[j,t,c]
        sct = np.ascontiguousarray(np.transpose(stl, (2, 0, 1)))       # [C, L, T]
        dstl = np.transpose(S @ sct, (1, 2, 0))
    else:           # dstl[l,t,i] = sum_j S[l,i,j] stl[l,t,j]
        dstl = stl @ np.transpose(S, (0, 2, 1))
    for n_, i in enumerate(style_ids):
        grads[i] = grads.get(i, 0) + dstl[n_]
    return content, style, grads


def targets_from_audio(W, content_wav_mu, style_wavs_mu, source_wavs_mu, *, cont_ids,
                       style_ids, gatys=False, nb_channels=C, cnt_channels=C):
    """methods.py:192-212 — phi_c = emb(content); phi_s = l2norm(G(content) + mean G(style)
    - mean G(source)).  Inputs are already mu-law encoded (methods.py:95)."""
    nb = needed_blocks(cont_ids, style_ids)

    def feats(xmu):
        ext, _ = encoder_forward(xmu, W, nb, need_bottleneck=31 in cont_ids)
        return ext

    ext_c = feats(content_wav_mu)
    phi_c = content_embeds(ext_c, cont_ids, cnt_channels)
    phi = style_embeds(ext_c, style_ids, gatys, nb_channels)
    phi_t = np.mean([style_embeds(feats(s), style_ids, gatys, nb_channels)
                     for s in style_wavs_mu], axis=0)
    phi_src = np.mean([style_embeds(feats(s), style_ids, gatys, nb_channels)
                       for s in source_wavs_mu], axis=0)
    return phi_c, l2_normalize(phi + phi_t - phi_src)


def late_of(batch_size):
    """methods.py:39 — samples cropped from each side of the output."""
    return (batch_size - (batch_size // 4096) * 4000) // 2
