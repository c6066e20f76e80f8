"""Where the HIP gradient's error against the fp64 oracle comes from, held per case and mode.

Round 4's split gradient error moved 4.2e-5 -> 3.1e-4 on the smoke case and 1.6e-4 -> 2.6e-5 on
the bench's golden 'ours' case with no change of the arithmetic.  The
cause (tools/diag/precision_lottery.py, DESIGN.md §4 "relu lottery"): the encoder is piecewise
linear in its relu decisions, and a run in any finite precision decides a few near-zero
elements (|value| ~1e-7 of the layer's max) the other way than fp64.  Each such flip moves the
gradient by 1e-4 .. 7e-4 on these problems; which elements flip changes with any change of
rounding anywhere upstream (round 4 moved the order of the start conv and of d loss / d x).

So each case is held on two separate claims, against the fp64 oracle forced onto the run's own
relu pattern (oracle/masked_oracle.py; the pattern is rebuilt from the run's extracts):
  * arithmetic: |g_run - g_fp64[run masks]| <= 2x its measured value (the precision claim);
  * lottery: every decision the run takes differently from fp64 is a near-tie,
    |fp64 value| <= 1e-6 x max |layer|;
and the total error <= the arithmetic bar + 1e-3 per flip (a flip moves the gradient by at most
7e-4 on these problems), so a harmless reordering that flips other near-ties passes while lost
bits or a flip that is no near-tie fail (round 5 held the total to 2x one lottery
draw).  Measured (round 5, split / fp32): smoke arithmetic 4.21e-5 / 4.94e-6, total 3.14e-4 /
3.37e-4 (one flip: u_22 / e_25); golden arithmetic 7.55e-6 / 9.96e-7, total 2.63e-5 / 2.28e-4.
Round 3's build measured the same arithmetic (4.20e-5, 7.53e-6) with other flips.
"""
import os

import numpy as np
import pytest
import torch

from oracle import astyle_oracle as O
from oracle import masked_oracle as M
from audio_style_transfer_amd.weights import synthetic_clips

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (case, mode): arithmetic bar = 2x the round-5 measurement
BARS = {
    ('smoke', 'split'): 8.5e-5,
    ('smoke', 'fp32'): 1.0e-5,
    ('golden', 'split'): 1.5e-5,
    ('golden', 'fp32'): 2.0e-6,
}
FLIP_ALLOWANCE = 1e-3   # per near-tie relu flip (measured 1e-4 .. 7e-4 each)


def _case(name, W):
    if name == 'smoke':     # __graft_entry__.smoke()'s problem
        T = 1024
        kw = dict(cont_ids=[29], style_ids=list(range(30)))
        xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
        xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
        pc, ps = O.targets_from_audio(W, xc, [xs], [xc], **kw)
        x = xc + np.random.default_rng(0).normal(0, 4, T)
        return x, pc.astype(np.float32), ps.astype(np.float32), kw
    g = np.load(os.path.join(ROOT, 'tests', 'golden', 'oracle_T2048.npz'))
    tg = np.load(os.path.join(ROOT, 'tests', 'golden', 'oracle_T2048_targets.npz'))
    return g['ours_x'], tg['ours_phi_c'], tg['ours_phi_s'], dict(cont_ids=[25], style_ids=list(range(30)))


@pytest.mark.parametrize('mode', ['split', 'fp32'])
@pytest.mark.parametrize('case', ['smoke', 'golden'])
def test_gradient_error_is_arithmetic_plus_near_tie_flips(case, mode, weights):
    from audio_style_transfer_amd.engine import StyleEngine
    dev = torch.device('cuda', 0)
    x, pc, ps, kw = _case(case, weights)
    T = x.shape[0]
    pc64, ps64 = pc.astype(np.float64), ps.astype(np.float64)
    _, g64, _, m64 = M.loss_and_grad(x, weights, phi_c=pc64, phi_s=ps64, **kw)
    eng = StyleEngine(1, T, kw['cont_ids'], kw['style_ids'], weights=weights, precision=mode,
                      device=dev)
    try:
        eng.set_targets(torch.tensor(pc), torch.tensor(ps))
        xt = torch.tensor(x[None], dtype=torch.float32, device=dev)
        _, grad = eng.loss_grad(xt)
        eng.forward(xt)
        ext = [eng.extract(i).cpu().numpy()[0] for i in range(29)]
        g = grad.cpu().double().numpy()[0]
    finally:
        eng.close()
    mh = M.masks_from_extracts(x, weights, ext)
    _, gm, _, _ = M.loss_and_grad(x, weights, phi_c=pc64, phi_s=ps64, me=mh[0], mu=mh[1], **kw)
    arith, total = M.rel(g, gm), M.rel(g, g64)
    cache = M.forward(x, weights)[1]
    ties = []
    for kind, k in (('e', 0), ('u', 1)):
        for l in range(30):
            ref = cache['es' if kind == 'e' else 'us'][l]
            for t, c in np.argwhere(mh[k][l] != m64[k][l]):
                ties.append((kind, l, int(t), int(c), abs(ref[t, c]) / np.abs(ref).max()))
    print('%s %s: total %.3e arithmetic %.3e flips %s' % (case, mode, total, arith, ties))
    a_bar = BARS[(case, mode)]
    assert arith <= a_bar, (arith, a_bar)
    assert all(r <= 1e-6 for *_, r in ties), ties
    assert total <= a_bar + FLIP_ALLOWANCE * len(ties), (total, a_bar, ties)
