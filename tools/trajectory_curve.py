"""One reference epoch (scipy L-BFGS-B, maxiter 100, methods.py:132-137) on the 'ours'
configuration at T samples, driven four ways: the HIP loss in fp32 mode and in split mode, the
torch fp32 restatement of the reference (its own precision, CPU) and the fp64 oracle (CPU).
Writes the loss per evaluation of each, and the final points' distances, to a JSON file
(profiles/r2_trajectory_ours_T<T>.json).  L-BFGS on an fp32 loss is chaotic over an epoch
(SURVEY F3): the curves, not the final points, are the comparison.

usage: python tools/trajectory_curve.py [T] [out.json]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import astyle_oracle as O, torch_restatement as TR   # noqa: E402  (checker)
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips   # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
OUT = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, 'profiles', 'r2_trajectory_ours_T%d.json' % T)
KW = dict(cont_ids=[25], style_ids=list(range(30)), gatys=False, nb_channels=128, cnt_channels=128)
W = synthetic_weights(0)
xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
phi_c, phi_s = O.targets_from_audio(W, xc, [xs], [xc], **KW)
x0 = np.full(T, np.float64(np.float32(1e-6)))


def lbfgs(fg):
    from scipy.optimize import minimize
    fs, its = [], []

    def wrapped(v):
        f, g = fg(v)
        fs.append(f)
        return f, g
    t = time.time()
    r = minimize(wrapped, x0, jac=True, method='L-BFGS-B', options={'maxiter': 100},
                 callback=lambda xk: its.append(len(fs)))
    return dict(f=fs, iter_end_eval=its, nit=int(r.nit), nfev=int(r.nfev), fun=float(r.fun),
                message=str(r.message), seconds=time.time() - t), r.x


def fg64(v):
    p, g = O.loss_and_grad(v, W, phi_c=phi_c, phi_s=phi_s, lambd=100.0, **KW)
    return float(p[0]), g


def fg32ref(v):
    xt = torch.tensor(v.astype(np.float32)).requires_grad_(True)
    tot, _, _, _ = TR.loss_fn(xt, W, phi_c=phi_c, phi_s=phi_s, lambd=100.0, dtype=torch.float32, **KW)
    g, = torch.autograd.grad(tot, xt)
    return float(tot.detach()), g.double().numpy()


def hip(precision):
    from audio_style_transfer_amd.engine import StyleEngine
    dev = torch.device('cuda', 0)
    eng = StyleEngine(1, T, KW['cont_ids'], KW['style_ids'], precision=precision, lambd=100.0,
                      weights=W, device=dev)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    xd = torch.empty(1, T, device=dev)

    def fg(v):
        xd.copy_(torch.from_numpy(v.astype(np.float32)).view(1, T))
        parts, grad = eng.loss_grad(xd)
        return float(parts[0, 0]), grad[0].double().cpu().numpy()
    return fg


runs, xs_ = {}, {}
for name, fg in (('hip_fp32', hip('fp32')), ('hip_split', hip('split')), ('torch_fp32_reference', fg32ref),
                 ('oracle_fp64', fg64)):
    runs[name], xs_[name] = lbfgs(fg)
    print(name, runs[name]['nit'], runs[name]['nfev'], '%.6g' % runs[name]['fun'],
          '%.1fs' % runs[name]['seconds'], flush=True)
ref = xs_['oracle_fp64']
for name in runs:
    runs[name]['x_rel_l2_vs_fp64_final'] = float(np.linalg.norm(xs_[name] - ref) / np.linalg.norm(ref))
json.dump(dict(config='ours (cont [25], style 0..29), T=%d, lambda 100, gamma 0, synthetic weights '
                      'seed 0, x0 = fp32(1e-6)' % T, runs=runs), open(OUT, 'w'), indent=1)
print('wrote', OUT)
