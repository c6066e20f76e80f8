"""Attribute bf16 gradient error: content-only (lambd=0) vs full, shallow vs deep taps."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
from oracle import astyle_oracle as O
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
from audio_style_transfer_amd.engine import StyleEngine
W = synthetic_weights(0)
def rel(a, b): return float(np.linalg.norm(np.asarray(a, np.float64) - b) / np.linalg.norm(b))
T = 2048
dev = torch.device('cuda', 0)
xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0]); xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
x = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(7).normal(0, 4, T)
for cont, sty, lam in [([29], list(range(30)), 0.0), ([5], [0,1,2], 0.0), ([29], list(range(30)), 100.0), ([0], [29], 100.0), ([0], [0], 100.0), ([0], list(range(30)), 1e4)]:
    kw = dict(cont_ids=cont, style_ids=sty, gatys=False, nb_channels=128, cnt_channels=128)
    phi_c, phi_s = O.targets_from_audio(W, xc, [xs], [xc], **kw)
    rp, rg = O.loss_and_grad(x, W, phi_c=phi_c, phi_s=phi_s, lambd=lam, **kw)
    eng = StyleEngine(1, T, cont, sty, weights=W, precision='bf16', lambd=lam)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    p, gr = eng.loss_grad(torch.tensor(x[None], dtype=torch.float32, device=dev))
    gr = gr.cpu().numpy()[0]
    print(cont, sty[:3], len(sty), lam, 'grad relL2 %.4f' % rel(gr, rg), 'parts', p.cpu().numpy()[0][:3], rp[:3])
