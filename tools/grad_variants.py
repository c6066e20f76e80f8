"""Diagnostic: split-mode gradient error of the golden T = 2048 cases against the fp64 oracle
fixtures, for the libastyle.so named by ASTYLE_LIB (one library per process).
usage: ASTYLE_LIB=... python tools/grad_variants.py"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from audio_style_transfer_amd.engine import StyleEngine
from audio_style_transfer_amd.weights import synthetic_weights
g = np.load(os.path.join(ROOT, 'tests', 'golden', 'oracle_T2048.npz'))
tg = np.load(os.path.join(ROOT, 'tests', 'golden', 'oracle_T2048_targets.npz'))
W = synthetic_weights(0)
CASES = {'ours': ([25], list(range(30)), False, 128, 128), 'c1': ([25], list(range(10)), False, 128, 128),
         'trunc': ([25, 31], [3, 7], False, 64, 16), 'gatys': ([29], list(range(30)), True, 128, 128)}
out = []
for tag, (cont, sty, gat, nb, cnt) in CASES.items():
    if tag + '_phi_c' not in tg.files:
        continue
    eng = StyleEngine(1, 2048, cont, sty, cnt_channels=cnt, nb_channels=nb, gatys=gat, weights=W,
                      precision=os.environ.get('PREC', 'split'))
    eng.set_targets(torch.tensor(tg[tag + '_phi_c']), torch.tensor(tg[tag + '_phi_s']))
    _, grad = eng.loss_grad(torch.tensor(g[tag + '_x'][None], dtype=torch.float32, device='cuda'))
    gr = grad.cpu().double().numpy()[0]
    ref = g[tag + '_grad']
    out.append('%s %.3g' % (tag, np.linalg.norm(gr - ref) / np.linalg.norm(ref)))
print(os.path.basename(os.environ.get('ASTYLE_LIB', 'libastyle.so')), ' '.join(out))
