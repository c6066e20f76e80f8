"""Debug: per-layer bf16 extract error vs the oracle (tools only)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np, torch
from oracle import astyle_oracle as O
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
from audio_style_transfer_amd.engine import StyleEngine
W = synthetic_weights(0)
for T, B in [(int(a.split('x')[1]), int(a.split('x')[0])) for a in sys.argv[1:]]:
    x = O.mu_law_numpy(synthetic_clips(B, T, 42)) + np.random.default_rng(3).normal(0, 4, (B, T))
    eng = StyleEngine(B, T, [29], list(range(30)), weights=W, precision='bf16', device=torch.device('cuda', 0))
    xt = torch.tensor(x, dtype=torch.float32, device='cuda')
    eng.forward(xt)
    ext, _ = O.encoder_forward(x[0], W, 30)
    out = []
    for i in range(30):
        e = eng.extract(i).cpu().numpy()[0]
        err = np.linalg.norm(e - ext[i]) / np.linalg.norm(ext[i])
        out.append('%d:%.2g%s' % (i, err, 'NaN' if np.isnan(e).any() else ''))
    print('T=%d B=%d' % (T, B), ' '.join(out), flush=True)
