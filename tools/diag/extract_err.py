"""Diagnostic: split-mode extract errors per layer (rel-L2 and mean signed relative error vs the
fp64 oracle) and the gradient error, for the library in ASTYLE_LIB."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
from oracle import astyle_oracle as O
from audio_style_transfer_amd.engine import StyleEngine
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
W = synthetic_weights(0)
T = 2048
x = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0]) + np.random.default_rng(0).normal(0, 4, T)
ext, _ = O.encoder_forward(x, W, 30, need_bottleneck=False)
eng = StyleEngine(1, T, [29], list(range(30)), weights=W, precision=os.environ.get('PREC', 'split'))
eng.forward(torch.tensor(x[None], dtype=torch.float32, device='cuda'))
row = []
for i in (0, 1, 2, 5, 9, 15, 19, 25, 29):
    g = eng.extract(i).cpu().double().numpy()[0]
    r = ext[i]
    row.append('%d:%.2e/%+.1e' % (i, np.linalg.norm(g - r) / np.linalg.norm(r), np.sum((g - r) * np.sign(r)) / np.sum(np.abs(r))))
print(os.path.basename(os.environ.get('ASTYLE_LIB', 'x')), ' '.join(row))
