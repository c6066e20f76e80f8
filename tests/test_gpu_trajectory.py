"""Trajectory parity: the reference's optimiser (scipy L-BFGS-B through ScipyOptimizerInterface,
methods.py:132-137,164-181) driven by the HIP loss+grad vs the same optimiser driven by the fp64
oracle (oracle/astyle_oracle.py loss_and_grad) — the achievable form of the north_star's "audio
within 1e-3 rel-L2" (SURVEY §4 "Trajectory").

Both runs start at fp32(1e-6) (the TF variable's initial value, methods.py:49-54) with the
reference's options (m 10, scipy defaults otherwise); the iterate after each of the first 3
iterations (scipy callback) is compared with the fp64 run's.

The bar is calibrated by the reference's own arithmetic: L-BFGS-B's line search interpolates
trial steps from loss VALUES, so the fp32 rounding of the loss (relative ~1e-7..1e-6) is
amplified by f / delta-f; the torch fp32 restatement of the reference (oracle/torch_restatement.py,
F.conv1d + autograd in fp32: the precision TF computes in) departs from the fp64 trajectory by
6.8e-4, 9.4e-4, 6.7e-3 after iterations 1..3 (ours, T=4096, measured here).  So a fixed 1e-3 at
iteration 3 is beyond the reference itself; the test asserts, per iteration k <= 3,
  rel-L2(x_HIP_k, x_fp64_k) <= max(1e-3, 2 * rel-L2(x_fp32ref_k, x_fp64_k))
for the fp32 mode and the split mode (the bench headline), and prints all three.
"""
import numpy as np
import pytest
import torch

from oracle import astyle_oracle as O
from audio_style_transfer_amd.weights import synthetic_clips

pytestmark = pytest.mark.gpu

CASES = {
    'ours': dict(cont_ids=[25], style_ids=list(range(30)), gatys=False, nb_channels=128,
                 cnt_channels=128),
    'c1': dict(cont_ids=[25], style_ids=list(range(10)), gatys=False, nb_channels=128,
               cnt_channels=128),
    'gatys': dict(cont_ids=[29], style_ids=list(range(30)), gatys=True, nb_channels=128,
                  cnt_channels=128),
}
ITERS = 3
BAR = 1e-3


@pytest.fixture(scope='module')
def dev():
    assert torch.cuda.is_available(), 'gpu tests need an MI355X'
    return torch.device('cuda', 0)


def _targets(kw, T, weights):
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
    return O.targets_from_audio(weights, xc, [xs], [xc], **kw)


def _lbfgs(fg, x0, maxiter):
    from scipy.optimize import minimize
    its = []
    res = minimize(fg, x0, jac=True, method='L-BFGS-B', options={'maxiter': maxiter},
                   callback=lambda xk: its.append(np.array(xk, copy=True)))
    return res, its


def _oracle_run(kw, T, weights, phi_c, phi_s, x0, maxiter):
    def fg(v):
        parts, g = O.loss_and_grad(v, weights, phi_c=phi_c, phi_s=phi_s, lambd=100.0, **kw)
        return float(parts[0]), g
    return _lbfgs(fg, x0, maxiter)


def _ref32_run(kw, T, weights, phi_c, phi_s, x0, maxiter):
    """The reference's precision on the CPU: torch fp32 restatement + autograd."""
    from oracle import torch_restatement as TR

    def fg(v):
        xt = torch.tensor(v.astype(np.float32)).requires_grad_(True)
        tot, _, _, _ = TR.loss_fn(xt, weights, phi_c=phi_c, phi_s=phi_s, lambd=100.0,
                                  dtype=torch.float32, **kw)
        g, = torch.autograd.grad(tot, xt)
        return float(tot.detach()), g.double().numpy()
    return _lbfgs(fg, x0, maxiter)


def _hip_run(kw, T, weights, phi_c, phi_s, x0, maxiter, precision, dev):
    from audio_style_transfer_amd.engine import StyleEngine
    eng = StyleEngine(1, T, kw['cont_ids'], kw['style_ids'], cnt_channels=kw['cnt_channels'],
                      nb_channels=kw['nb_channels'], gatys=kw['gatys'], weights=weights,
                      precision=precision, lambd=100.0, device=dev)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    xd = torch.empty(1, T, device=dev)

    def fg(v):
        xd.copy_(torch.from_numpy(v.astype(np.float32)).view(1, T))
        parts, grad = eng.loss_grad(xd)
        return float(parts[0, 0]), grad[0].double().cpu().numpy()
    out = _lbfgs(fg, x0, maxiter)
    eng.close()
    return out


_ORACLE = {}


@pytest.mark.parametrize('precision', ['fp32', 'split'])
@pytest.mark.parametrize('tag,T', [('ours', 4096), ('c1', 4096), ('gatys', 4096), ('ours', 16384)])
def test_first_iterations_match_fp64_oracle(tag, T, precision, weights, dev):
    kw = CASES[tag]
    x0 = np.full(T, np.float64(np.float32(1e-6)))
    key = (tag, T)
    if key not in _ORACLE:
        phi_c, phi_s = _targets(kw, T, weights)
        res_o, its_o = _oracle_run(kw, T, weights, phi_c, phi_s, x0, ITERS)
        _, its_r = _ref32_run(kw, T, weights, phi_c, phi_s, x0, ITERS)
        _ORACLE[key] = (phi_c, phi_s, res_o, its_o, its_r)
    phi_c, phi_s, res_o, its_o, its_r = _ORACLE[key]
    res_h, its_h = _hip_run(kw, T, weights, phi_c, phi_s, x0, ITERS, precision, dev)
    assert len(its_o) == ITERS and len(its_h) == ITERS and len(its_r) == ITERS
    rel = lambda a, b: float(np.linalg.norm(a - b) / np.linalg.norm(b))
    errs = [rel(a, b) for a, b in zip(its_h, its_o)]
    envs = [rel(a, b) for a, b in zip(its_r, its_o)]
    print('%s T=%d %s: x rel-L2 vs fp64 per iteration: HIP %s | fp32 reference %s | f hip %.8g '
          'fp64 %.8g | nfev %d / %d' % (tag, T, precision, ['%.2e' % e for e in errs],
                                        ['%.2e' % e for e in envs], res_h.fun, res_o.fun,
                                        res_h.nfev, res_o.nfev))
    for e, v in zip(errs, envs):
        assert e <= max(BAR, 2.0 * v)


@pytest.mark.parametrize('precision', ['fp32', 'split'])
def test_full_epoch_reaches_the_fp64_point(precision, weights, dev):
    """One reference epoch (maxiter 100) of 'ours' at T=4096 converges (projected-gradient
    test) to the fp64 oracle's point: final x within 1e-3 rel-L2 (measured 9e-5 fp32, 6e-5
    split, 7e-5 for the torch fp32 reference; profiles/r2_trajectory_ours_T4096.json)."""
    kw = CASES['ours']
    T = 4096
    x0 = np.full(T, np.float64(np.float32(1e-6)))
    key = ('epoch', T)
    if key not in _ORACLE:
        phi_c, phi_s = _targets(kw, T, weights)
        res_o, _ = _oracle_run(kw, T, weights, phi_c, phi_s, x0, 100)
        _ORACLE[key] = (phi_c, phi_s, res_o)
    phi_c, phi_s, res_o = _ORACLE[key]
    res_h, _ = _hip_run(kw, T, weights, phi_c, phi_s, x0, 100, precision, dev)
    e = float(np.linalg.norm(res_h.x - res_o.x) / np.linalg.norm(res_o.x))
    print('epoch %s: x rel-L2 %.3g | it %d / %d | f %.7g / %.7g | %s' % (precision, e, res_h.nit,
          res_o.nit, res_h.fun, res_o.fun, res_h.message))
    assert res_h.nit < 100 and res_o.nit < 100          # both converged inside the epoch
    assert e <= BAR
    assert abs(res_h.fun - res_o.fun) <= 1e-4 * abs(res_o.fun)
