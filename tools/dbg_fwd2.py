"""Debug: layer-0 bf16 output error pattern vs the oracle (tools only)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
from oracle import astyle_oracle as O
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
from audio_style_transfer_amd.engine import StyleEngine
W = synthetic_weights(0)
T, B = 2048, 1
x = O.mu_law_numpy(synthetic_clips(B, T, 42)) + np.random.default_rng(3).normal(0, 4, (B, T))
eng = StyleEngine(B, T, [29], list(range(30)), weights=W, precision='bf16', device=torch.device('cuda', 0))
xt = torch.tensor(x, dtype=torch.float32, device='cuda')
eng.forward(xt)
ext, _ = O.encoder_forward(x[0], W, 30)
e = eng.extract(0).cpu().numpy()[0]
r = ext[0]
d = np.abs(e - r)
print('rel', np.linalg.norm(e - r) / np.linalg.norm(r))
print('per 16-ch chunk rel:', ' '.join('%.2f' % (np.linalg.norm((e - r)[:, 8*k:8*k+8]) / np.linalg.norm(r[:, 8*k:8*k+8])) for k in range(16)))
print('per row mod 32 rel:', ' '.join('%.2f' % (np.linalg.norm((e - r)[m::32]) / np.linalg.norm(r[m::32])) for m in range(32)))
print('per tile rel:', ' '.join('%.2f' % (np.linalg.norm((e - r)[128*k:128*k+128]) / np.linalg.norm(r[128*k:128*k+128])) for k in range(T // 128)))
print('sample row 5 gpu', np.round(e[5, :16], 3)); print('sample row 5 ref', np.round(r[5, :16], 3))
# where could the right values be? search rows
for t in [5, 40]:
    dd = np.linalg.norm(r - e[t][None, :], axis=1); print('row', t, 'best match ref row', int(dd.argmin()), dd.min() / np.linalg.norm(r[t]))
    dd = np.linalg.norm(e - r[t][None, :], axis=1); print('ref row', t, 'best match gpu row', int(dd.argmin()), dd.min() / np.linalg.norm(r[t]))
