"""Debug: isolate one bf16 block: oracle block applied to the GPU's own input (tools only)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
from oracle import astyle_oracle as O
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
from audio_style_transfer_amd.engine import StyleEngine
W = synthetic_weights(0)
T, B = int(sys.argv[1]), 1
x = O.mu_law_numpy(synthetic_clips(B, T, 42)) + np.random.default_rng(3).normal(0, 4, (B, T))
eng = StyleEngine(B, T, [29], list(range(30)), weights=W, precision='bf16', device=torch.device('cuda', 0))
eng.forward(torch.tensor(x, dtype=torch.float32, device='cuda'))
for l in [int(v) for v in sys.argv[2:]]:
    ein = eng.extract(l - 1).cpu().numpy()[0].astype(np.float64)
    eo = eng.extract(l).cpu().numpy()[0].astype(np.float64)
    d = O.dilation_of(l)
    u = O.conv1d_same(O.relu(ein), W['ae_dilatedconv_%d/W' % (l + 1)], W['ae_dilatedconv_%d/biases' % (l + 1)], d)
    ref = ein + O.conv1d_same(O.relu(u), W['ae_res_%d/W' % (l + 1)], W['ae_res_%d/biases' % (l + 1)], 1)
    err = np.linalg.norm(eo - ref, axis=1) / np.linalg.norm(ref, axis=1)
    n = T // d
    pos = np.array([(t % d) * n + t // d for t in range(T)])   # t2b position of time t
    bad = np.where(err > 0.02)[0]
    print('layer', l, 'd', d, 'n', n, 'rel', np.linalg.norm(eo - ref) / np.linalg.norm(ref), 'bad rows', len(bad))
    print('  bad times', bad[:20], ' positions', pos[bad][:20], ' pos mod 128', sorted(set((pos[bad] % 128).tolist()))[:40])
