"""CPU emulation of candidate precision schemes for the encoder + Gram (diagnostics only).

Every conv / Gram product is evaluated in float64 on operands rounded the way a kernel would
round them, and the result is rounded to fp32 (the MFMA accumulates in fp32).  Schemes:
  fp32      operands fp32 (the fp32 MFMA path)
  f16x3     the same with fp16 halves under a per-tensor power-of-two scale (22 bits)
  split3    a = ah + al, ah = bf16(a), al = bf16(a - ah) for activations AND weights;
            a*b ~ ah*bh + ah*bl + al*bh (three bf16 MFMAs, the lo*lo term dropped)
  bf16      operands bf16 (one bf16 MFMA)
The gradient rel-L2 against the fp64 oracle is printed for each combination of
(encoder scheme, Gram forward scheme, Gram backward scheme).

  python tools/precision_emulate.py [T] [tag] [wino]   (wino: Winograd F(2,3) dilated convs)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import torch.nn.functional as F

from oracle import astyle_oracle as O
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips

torch.set_num_threads(os.cpu_count())


def r32(a):
    return a.float().double()


def bf(a):
    return a.float().to(torch.bfloat16).double()


def split(a):
    h = bf(a)
    return h, bf(a - h)


def pow2_scale(a):
    m = a.abs().max().item()
    return 2.0 ** (14 - int(np.ceil(np.log2(m)))) if m > 0 else 1.0


def split16(a):
    """a = ah + al: ah = fp16(a s) / s, al = fp16((a - ah) s 2^11) / (s 2^11); s a power of two
    that puts max|a| at 2^14 (fp16 max 65504), so neither part loses bits to the fp16 range."""
    s = pow2_scale(a)
    ah = (a * s).float().half().double() / s
    s2 = s * 2048.0
    al = ((a - ah) * s2).float().half().double() / s2
    return ah, al


def f16x2(a):
    """storage as a split fp16 pair (22 significant bits)"""
    ah, al = split16(r32(a))
    return ah + al


def prod(scheme, fn, a, b):
    """fn(a, b) bilinear, evaluated under `scheme`, result rounded to fp32."""
    if scheme == 'fp64':
        return fn(a, b)
    if scheme == 'fp32':
        return r32(fn(r32(a), r32(b)))
    if scheme == 'bf16':
        return r32(fn(bf(a), bf(b)))
    if scheme == 'split3':
        ah, al = split(r32(a))
        bh, bl = split(r32(b))
        return r32(fn(ah, bh) + fn(ah, bl) + fn(al, bh))
    if scheme == 'f16x3':     # fp16 two-term split, per-tensor power-of-two scale, lo*lo dropped
        ah, al = split16(r32(a))
        bh, bl = split16(r32(b))
        return r32(fn(ah, bh) + fn(ah, bl) + fn(al, bh))
    if scheme == 'split3a':   # activations split, weights as two bf16 terms, lo*lo kept
        ah, al = split(r32(a))
        bh, bl = split(r32(b))
        return r32(fn(ah, bh) + fn(ah, bl) + fn(al, bh) + fn(al, bl))
    raise ValueError(scheme)


def conv(x, W, d):
    """x [C, T] (float64), W OIK -> y [O, T], SAME padding."""
    k = W.shape[2]
    return F.conv1d(x[None], W, None, padding=((k - 1) // 2) * d, dilation=d)[0]


def conv_t(g, W, d):
    k = W.shape[2]
    return F.conv_transpose1d(g[None], W, None, padding=((k - 1) // 2) * d, dilation=d)[0]


def wino(x, W, d, scheme):
    """The dilated conv (x [C, T], W OIK, K = 3, SAME) as Winograd F(2,3) over output pairs
    (positions 2j, 2j+1 of each sub-sequence t = s + k d, masked.py:57-86): the transformed
    inputs d0 = x_{2j-1} - x_{2j+1}, d1 = x_{2j} + x_{2j+1}, d2 = x_{2j+1} - x_{2j},
    d3 = x_{2j} - x_{2j+2} formed in fp32 (as the kernel's conversion would), the transformed
    weights G = (W0, (W0+W1+W2)/2, (W0-W1+W2)/2, W2) in fp64 then split, four products m_i =
    G_i d_i under `scheme`, y_{2j} = m0 + m1 + m2, y_{2j+1} = m1 - m2 - m3 in fp32."""
    C, T = x.shape
    n = T // d
    assert n % 2 == 0
    X = x.reshape(C, n, d)                                    # X[:, k, s] = x[:, k d + s]
    Z = torch.zeros(C, 1, d, dtype=x.dtype)
    Xp = torch.cat([Z, X, Z, Z], 1)                           # k = -1 .. n + 1
    xm1, x0, x1, x2 = (Xp[:, 2 * np.arange(n // 2) + o] for o in (0, 1, 2, 3))
    ds = [r32(xm1 - x1), r32(x0 + x1), r32(x1 - x0), r32(x0 - x2)]
    W0, W1, W2 = W[:, :, 0], W[:, :, 1], W[:, :, 2]
    Gs = [W0, (W0 + W1 + W2) / 2, (W0 - W1 + W2) / 2, W2]
    mm = lambda a, b: torch.einsum('oc,cjs->ojs', b, a)
    m = [prod(scheme, mm, dd, G) for dd, G in zip(ds, Gs)]
    y0 = r32(r32(m[0] + m[1]) + m[2])
    y1 = r32(r32(m[1] - m[2]) - m[3])
    Y = torch.stack([y0, y1], 2).reshape(W.shape[0], n, d)   # k = 2j, 2j + 1
    return Y.reshape(W.shape[0], T)


def wino_t(g, W, d, scheme):
    """conv_transpose1d of the dilated conv = the conv with taps (W2^T, W1^T, W0^T)."""
    Wt = W.permute(1, 0, 2).flip(2).contiguous()
    return wino(g, Wt, d, scheme)


def run(x, Wd, phi_c, phi_s, kw, enc='fp32', gf='fp32', gb='fp32', store='fp32', winograd=False):
    R = r32 if store == 'fp32' else f16x2
    if enc == 'fp64':
        R = lambda a: a
    cont_ids, style_ids, lambd = kw['cont_ids'], kw['style_ids'], 100.0
    nb = O.needed_blocks(cont_ids, style_ids)
    xs = torch.tensor(x / 128.0)[None]
    W0, b0 = Wd['ae_startconv/W'], Wd['ae_startconv/biases']
    e = R(prod('fp32' if enc != 'fp64' else 'fp64', lambda a, b: conv(a, b, 1), xs, W0) + b0[:, None])
    es, us = [e], []
    for l in range(nb):
        dd = O.dilation_of(l)
        Wdl, bdl = Wd['ae_dilatedconv_%d/W' % (l + 1)], Wd['ae_dilatedconv_%d/biases' % (l + 1)]
        Wrl, brl = Wd['ae_res_%d/W' % (l + 1)], Wd['ae_res_%d/biases' % (l + 1)]
        if winograd and e.shape[1] // dd >= 2:
            u = R(wino(torch.relu(e), Wdl, dd, enc) + bdl[:, None])
        else:
            u = R(prod(enc, lambda a, b: conv(a, b, dd), torch.relu(e), Wdl) + bdl[:, None])
        y = prod(enc, lambda a, b: conv(a, b, 1), torch.relu(u), Wrl) + brl[:, None]
        e = R(e + y)
        es.append(e)
        us.append(u)
    ext = es[1:]
    if nb == 30:
        ext.append(ext[-1])
    # content
    emb = torch.cat([ext[i] for i in cont_ids], 0)           # [n*C, T]
    pc = torch.tensor(phi_c.T)
    diff = emb - pc
    content = 10.0 * torch.mean(diff * diff)
    gemb = 20.0 * diff / diff.numel()
    grads = {}
    for n_, i in enumerate(cont_ids):
        grads[i] = grads.get(i, 0) + gemb[n_ * 128:(n_ + 1) * 128]
    # ours Gram: E_c [L, T] per channel
    stl = torch.stack([ext[i] for i in style_ids], 0)        # [L, C, T]
    s = stl.permute(1, 0, 2)                                 # [C, L, T]
    G = prod(gf, lambda a, b: a @ b.transpose(1, 2), s, s)
    ss = (G * G).sum(dim=(1, 2), keepdim=True)
    inv = 1.0 / torch.sqrt(torch.clamp(ss, min=1e-12))
    Gn = G * inv
    ps = torch.tensor(phi_s)
    sd = Gn - ps
    style = 1e3 * torch.mean(sd * sd)
    dGn = lambd * 1e3 * 2.0 * sd / sd.numel()
    dot = (Gn * dGn).sum(dim=(1, 2), keepdim=True)
    dG = dGn * inv - Gn * dot * inv
    S = dG + dG.transpose(1, 2)
    dst = prod(gb, lambda a, b: a @ b, S, s)                 # [C, L, T]
    dst = dst.permute(1, 0, 2)
    for n_, i in enumerate(style_ids):
        grads[i] = grads.get(i, 0) + dst[n_]
    # backward
    g = torch.zeros_like(es[0])
    if 30 in grads:
        g = g + grads[30]
    for l in reversed(range(nb)):
        if l in grads:
            g = R(g + grads[l])
        dd = O.dilation_of(l)
        Wdl, Wrl = Wd['ae_dilatedconv_%d/W' % (l + 1)], Wd['ae_res_%d/W' % (l + 1)]
        gv = prod(enc, lambda a, b: conv_t(a, b, 1), g, Wrl)
        gu = R(gv * (us[l] > 0))
        if winograd and gu.shape[1] // dd >= 2:
            gh = wino_t(gu, Wdl, dd, enc)
        else:
            gh = prod(enc, lambda a, b: conv_t(a, b, dd), gu, Wdl)
        g = R(g + gh * (es[l] > 0))
    gx = conv_t(g, W0, 1)[0] / 128.0
    return float(content), float(style), gx.numpy()


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    tag = sys.argv[2] if len(sys.argv) > 2 else 'ours'
    W = synthetic_weights(0)
    Wd = {k: torch.tensor(np.asarray(v, np.float64)) for k, v in W.items()}
    for k in list(Wd):
        if k.endswith('/W'):
            Wd[k] = Wd[k][0].permute(2, 1, 0).contiguous()   # HWIO -> OIK
    cases = {'ours': dict(cont_ids=[25], style_ids=list(range(30))),
             'smoke': dict(cont_ids=[29], style_ids=list(range(30))),
             'c1': dict(cont_ids=[25], style_ids=list(range(10))),
             'def': dict(cont_ids=[29], style_ids=list(range(30)))}
    kw = cases[tag]
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
    full = dict(kw, gatys=False, nb_channels=128, cnt_channels=128)
    phi_c, phi_s = O.targets_from_audio(W, xc, [xs], [xc], **full)
    if tag == 'smoke':     # __graft_entry__.smoke(): x near the content clip
        x = xc + np.random.default_rng(0).normal(0, 4, T)
    else:                  # tests/golden/make_golden.py
        x = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(7).normal(0, 4, T)
    _, _, ref = run(x, Wd, phi_c, phi_s, kw, enc='fp64', gf='fp64', gb='fp64')
    _, ogr = O.loss_and_grad(x, W, phi_c=phi_c, phi_s=phi_s, **full)
    print('restatement vs oracle fp64: %.3g' % (np.linalg.norm(ref - ogr) / np.linalg.norm(ogr)))
    if 'wino' in sys.argv:   # Winograd F(2,3) dilated convs (fwd + bwd) vs the direct form
        _, _, w64 = run(x, Wd, phi_c, phi_s, kw, enc='fp64', gf='fp64', gb='fp64', winograd=True)
        print('winograd fp64 vs direct fp64: %.3g' % (np.linalg.norm(w64 - ref) / np.linalg.norm(ref)))
        for enc, gf, gb, wg in [('fp32', 'fp32', 'fp32', False), ('fp32', 'fp32', 'fp32', True),
                                ('f16x3', 'split3', 'split3', False), ('f16x3', 'split3', 'split3', True)]:
            c, s_, g = run(x, Wd, phi_c, phi_s, kw, enc=enc, gf=gf, gb=gb, winograd=wg)
            print('enc %-6s%s gram %-6s grad rel-L2 %.3g' % (enc, ' winograd' if wg else ' direct  ', gf,
                  np.linalg.norm(g - ref) / np.linalg.norm(ref)), flush=True)
        return
    for enc, gf, gb, st in [('fp32', 'fp32', 'fp32', 'fp32'), ('split3', 'fp32', 'fp32', 'fp32'),
                            ('f16x3', 'fp32', 'fp32', 'fp32'), ('f16x3', 'fp32', 'fp32', 'f16x2'),
                            ('f16x3', 'bf16', 'fp32', 'fp32'), ('f16x3', 'bf16', 'bf16', 'fp32'),
                            ('f16x3', 'bf16', 'f16x3', 'fp32'), ('f16x3', 'f16x3', 'f16x3', 'fp32'),
                            ('f16x3', 'split3', 'split3', 'fp32'),
                            ('bf16', 'bf16', 'bf16', 'fp32')]:
        c, s, g = run(x, Wd, phi_c, phi_s, kw, enc=enc, gf=gf, gb=gb, store=st)
        print('enc %-7s gram fwd %-7s bwd %-7s store %-6s grad rel-L2 %.3g' %
              (enc, gf, gb, st, np.linalg.norm(g - ref) / np.linalg.norm(ref)), flush=True)


if __name__ == '__main__':
    main()
