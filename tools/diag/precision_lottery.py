"""Diagnostic: where does a split / fp32 gradient error come from?

For the smoke case (T = 1024, content layer 29) and the bench's golden 'ours' case (T = 2048,
content layer 25, fp32 targets) this runs the library's loss+grad and forward, reconstructs the
relu pattern the kernels used (masked_oracle.masks_from_extracts), and splits the gradient error
against the fp64 oracle into the relu-decision lottery and the arithmetic on the run's own piece.

  python tools/diag/precision_lottery.py [--tree DIR] [--tag NAME] [--out FILE.npz]

--tree: a directory holding another build of the package (e.g. tools/_r3, the round-3 final
sources built in place), imported instead of this checkout's.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

ap = argparse.ArgumentParser()
ap.add_argument('--tree', default=ROOT)
ap.add_argument('--tag', default='head')
ap.add_argument('--out', default='')
ap.add_argument('--modes', default='split,fp32')
args = ap.parse_args()
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.abspath(args.tree))
import torch  # noqa: E402
from oracle import masked_oracle as M  # noqa: E402
from oracle import astyle_oracle as O  # noqa: E402
from audio_style_transfer_amd.engine import StyleEngine  # noqa: E402
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips  # noqa: E402
import audio_style_transfer_amd  # noqa: E402

print('package', os.path.dirname(audio_style_transfer_amd.__file__), flush=True)
W = synthetic_weights(0)


def smoke_case():
    T = 1024
    kw = dict(cont_ids=[29], style_ids=list(range(30)))
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
    phi_c, phi_s = O.targets_from_audio(W, xc, [xs], [xc], **kw)
    x = xc + np.random.default_rng(0).normal(0, 4, T)
    return x, phi_c.astype(np.float32), phi_s.astype(np.float32), kw


def golden_case():
    g = np.load(os.path.join(ROOT, 'tests', 'golden', 'oracle_T2048.npz'))
    tg = np.load(os.path.join(ROOT, 'tests', 'golden', 'oracle_T2048_targets.npz'))
    return g['ours_x'], tg['ours_phi_c'], tg['ours_phi_s'], dict(cont_ids=[25], style_ids=list(range(30)))


dev = torch.device('cuda', 0)
save = {}
for cname, case in (('smoke', smoke_case), ('golden', golden_case)):
    x, pc, ps, kw = case()
    T = x.shape[0]
    pc64, ps64 = pc.astype(np.float64), ps.astype(np.float64)
    p64, g64, e64, m64 = M.loss_and_grad(x, W, phi_c=pc64, phi_s=ps64, **kw)
    cache64 = M.forward(x, W)[1]
    for mode in args.modes.split(','):
        eng = StyleEngine(1, T, kw['cont_ids'], kw['style_ids'], weights=W, precision=mode, device=dev)
        eng.set_targets(torch.tensor(pc), torch.tensor(ps))
        xt = torch.tensor(x[None], dtype=torch.float32, device=dev)
        parts, grad = eng.loss_grad(xt)
        eng.forward(xt)
        ext = [eng.extract(i).cpu().numpy()[0] for i in range(30)]
        torch.cuda.synchronize()
        eng.close()
        g = grad.cpu().double().numpy()[0]
        mh = M.masks_from_extracts(x, W, ext)
        pm, gm, _, _ = M.loss_and_grad(x, W, phi_c=pc64, phi_s=ps64, me=mh[0], mu=mh[1], **kw)
        fe, fu = M.flips(mh, m64)
        xerr = [M.rel(ext[l], e64[l]) for l in range(30)]
        print('%s %s %s: grad vs fp64 %.3e | lottery fp64[run masks] vs fp64 %.3e | arithmetic run vs '
              'fp64[run masks] %.3e | flips e %d u %d | loss rel %.2e' % (
                  args.tag, cname, mode, M.rel(g, g64), M.rel(gm, g64), M.rel(g, gm), sum(fe), sum(fu),
                  abs(float(parts[0, 0]) - p64[0]) / abs(p64[0])), flush=True)
        if cname == 'golden':
            gold = np.load(os.path.join(ROOT, 'tests', 'golden', 'oracle_T2048.npz'))['ours_grad']
            print('   vs the committed golden gradient (fp64 targets; the bench check): %.3e' % M.rel(g, gold))
        print('   extract rel-L2 e1 %.2e e2 %.2e e10 %.2e e20 %.2e e30 %.2e' % (
            xerr[0], xerr[1], xerr[9], xerr[19], xerr[29]), flush=True)
        for kind, mm, ref in (('e', mh[0], m64[0]), ('u', mh[1], m64[1])):
            for l in range(30):
                for t, c in np.argwhere(mm[l] != ref[l]):
                    val = cache64['es' if kind == 'e' else 'us'][l][t, c]
                    print('   flip %s_%d t=%d c=%d fp64 value %.3e run says %s' % (
                        kind, l, t, c, val, 'pos' if mm[l][t, c] else 'nonpos'), flush=True)
        key = '%s_%s_%s' % (args.tag, cname, mode)
        save[key + '_grad'] = g.astype(np.float32)
        save[key + '_ebits'] = np.packbits(np.stack(mh[0]))
        save[key + '_ubits'] = np.packbits(np.stack(mh[1]))
        save[key + '_xerr'] = np.array(xerr)
if args.out:
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    np.savez_compressed(args.out, **save)
