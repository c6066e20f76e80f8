"""GPU: the 16x16x32 form of the split block kernels (ASTYLE_MFMA16=1 both, block_fwd_split16.hip /
block_bwd_split16.hip, round 6; the default 2 runs the backward on it, the forward on 32x32x16):
the golden loss / gradient against the fp64 oracle at the split mode's bars, agreement with the
32x32x16 kernels (ASTYLE_MFMA16=0) to fp32 rounding (the K accumulation
order differs, so not bit for bit), and bit-exact batch invariance (a clip alone equals the same
clip in slot 2 of 4).  The knob is read once per process, so each setting runs in a child."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, numpy as np, torch
sys.path.insert(0, sys.argv[1])
import bench
from audio_style_transfer_amd.engine import StyleEngine
dev = torch.device('cuda', 0)
g = np.load(os.path.join(sys.argv[1], 'tests', 'golden', 'oracle_T2048.npz'))
tg = np.load(os.path.join(sys.argv[1], 'tests', 'golden', 'oracle_T2048_targets.npz'))
e = StyleEngine(1, 2048, [25], list(range(30)), precision='split', device=dev, lambd=100.0)
e.set_targets(torch.tensor(tg['ours_phi_c']), torch.tensor(tg['ours_phi_s']))
p, gr = e.loss_grad(torch.tensor(g['ours_x'][None], dtype=torch.float32, device=dev))
out = {'parts': p[0].cpu().tolist(), 'grad': gr[0].cpu().double().numpy().tolist()}
e.close()
# batch invariance at T = 4096: clip 6 alone and in slot 2 of clips 4..7
res = []
for clips in ([6], [4, 5, 6, 7]):
    e = StyleEngine(len(clips), 4096, [29], list(range(30)), precision='split', device=dev, lambd=100.0)
    x = bench.make_problem(e, clips, 4096, dev)
    p, gr = e.loss_grad(x)
    k = clips.index(6)
    res.append((p[k].cpu().tolist(), gr[k].cpu().numpy().tolist()))
    e.close()
out['alone'], out['slot'] = res
print(json.dumps(out))
'''


def _run(mfma16):
    env = dict(os.environ, ASTYLE_MFMA16='1' if mfma16 else '0')
    r = subprocess.run([sys.executable, '-c', CHILD, ROOT], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def test_mfma16_kernels_match_the_oracle_and_the_default_kernels():
    g = np.load(os.path.join(ROOT, 'tests', 'golden', 'oracle_T2048.npz'))
    a, b = _run(True), _run(False)
    ref_p, ref_g = g['ours_parts'], g['ours_grad']
    for o in (a, b):
        assert abs(o['parts'][0] - ref_p[0]) <= 1e-4 * abs(ref_p[0])
        assert rel(o['grad'], ref_g) <= 2e-3
    assert abs(a['parts'][0] - b['parts'][0]) <= 1e-5 * abs(b['parts'][0])
    # bit-exact batch invariance of the 16x16x32 kernels
    assert a['alone'][0] == a['slot'][0] and a['alone'][1] == a['slot'][1]
    # and the same clip agrees with the default kernels to fp32 rounding (+ near-tie relu flips)
    assert rel(a['alone'][1], b['alone'][1]) <= 2e-3
    assert abs(a['alone'][0][0] - b['alone'][0][0]) <= 1e-4 * abs(b['alone'][0][0])
