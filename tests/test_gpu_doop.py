"""D out of place (ASTYLE_DOOP=1: a buffer of its own) against the default in place over the
activations: the same loss parts and gradient bit for bit, ours and Gatys Gram (each setting in
its own process: the switch is read once per process).  And the split ours-Gram backward's two
kernels (ASTYLE_GRAM_BWD_H=0: 32-channel quarter rows, k_gram_bwd_s; default: 64-channel half
rows, k_gram_bwd_h): the same gradient bit for bit (the same MFMAs per element of D); the fused
content tap's squared errors are summed per 256- vs 128-row slot, so the content loss agrees to
fp32 round-off."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
import bench
from audio_style_transfer_amd.engine import StyleEngine
out = {}
for gatys in (0, 1):
    e = StyleEngine(3, 4096, [29], list(range(30)), precision='split', device=torch.device('cuda', 0),
                    lambd=100.0, gatys=bool(gatys))
    x = bench.make_problem(e, [5, 6, 7], 4096, torch.device('cuda', 0))
    p, g = e.loss_grad(x)
    out['p%d' % gatys] = p.cpu().numpy()
    out['g%d' % gatys] = g.cpu().numpy()
    e.close()
np.savez(sys.argv[2], **out)
'''


def _run(tmp_path, doop, **extra):
    f = str(tmp_path / ('doop%s%s.npz' % (doop, ''.join(extra.values()))))
    env = dict(os.environ, ASTYLE_DOOP=doop, **extra)
    r = subprocess.run([sys.executable, '-c', CHILD, ROOT, f], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return np.load(f)


def test_d_out_of_place_equals_in_place(tmp_path):
    a, b = _run(tmp_path, '0'), _run(tmp_path, '1')
    for k in ('p0', 'g0', 'p1', 'g1'):
        assert np.isfinite(a[k]).all()
        assert np.array_equal(a[k], b[k]), k


def test_gram_backward_half_rows_equals_quarter_rows(tmp_path):
    a, b = _run(tmp_path, '0'), _run(tmp_path, '0', ASTYLE_GRAM_BWD_H='0')
    assert np.array_equal(a['g0'], b['g0'])
    assert np.allclose(a['p0'], b['p0'], rtol=1e-6, atol=0)
    assert np.array_equal(a['p1'], b['p1']) and np.array_equal(a['g1'], b['g1'])   # (Gatys: not affected)
