"""HIP STFT regulariser (stft_reg.hip, methods.py:121-125) vs the fp64 oracle — run on an MI355X.

The regulariser is computed in fp32 whatever the context's precision.  Tolerances:
  * reg value:               rel <= 1e-5
  * d reg / d x:             rel-L2 <= 1e-4, plus 2/sqrt(n_bins) for each bin whose |Re| or
                             |Im| is within 1e-5 of zero relative to the frame's largest bin
                             (d abs / d v is a sign: such a bin may legitimately flip in fp32,
                             and one flip moves the gradient by ~2/sqrt(n_bins) rel-L2)
The gradient is isolated as (grad(gamma) - grad(0)) / gamma on a context whose content and
style terms are zero (lambd = 0, phi_c = the clip's own content embedding).
"""
import numpy as np
import pytest
import torch

from oracle import astyle_oracle as O

pytestmark = pytest.mark.gpu

KW = dict(cont_ids=[0], style_ids=[0])


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope='module')
def dev():
    assert torch.cuda.is_available(), 'gpu tests need an MI355X'
    return torch.device('cuda', 0)


def _inputs(B, T, seed):
    rng = np.random.default_rng(seed)
    x = rng.normal(0, 30, (B, T))
    x[0, :7] = 0.0                      # inv_mu_law's x == 0 branch (utils.py:89,104)
    x[0, 7:9] = -0.5                    # o == 0: utils.sign's |o| <= 1e-12 branch
    x[-1, -300:] = 0.0                  # a silent tail
    return x


def _near_zero_bins(x):
    a, _ = O.inv_mu_law_tf(x)
    T = a.shape[0]
    nf = 1 + (T - O.FRAME) // O.HOP
    idx = np.arange(O.FRAME)[None, :] + O.HOP * np.arange(nf)[:, None]
    S = np.fft.rfft(a[idx] * O._hann_periodic(O.FRAME), axis=1)
    m = np.abs(S).max(axis=1, keepdims=True) * 1e-5
    near = (np.abs(S.real) < m).sum() + (np.abs(S.imag[:, 1:-1]) < m).sum()
    return int(near), S.size


def _engine(B, T, weights, precision):
    from audio_style_transfer_amd.engine import StyleEngine
    return StyleEngine(B, T, KW['cont_ids'], KW['style_ids'], lambd=0.0, precision=precision,
                       weights=weights)


@pytest.mark.parametrize('T', [1024, 2048, 16384])
@pytest.mark.parametrize('precision', ['fp32', 'bf16'])
def test_stft_reg_matches_oracle(T, precision, weights, dev):
    B = 3
    x = _inputs(B, T, T)
    eng = _engine(B, T, weights, precision)
    xt = torch.tensor(x, dtype=torch.float32, device=dev)
    emb_c, emb_s = eng.embeds(xt)
    eng.set_targets(emb_c.clone(), emb_s[0].clone())
    p0, g0 = eng.loss_grad(xt)
    g0 = g0.clone()
    gamma = 2.5
    eng.set_gamma(gamma)
    p1, g1 = eng.loss_grad(xt)
    torch.cuda.synchronize()
    p0, p1 = p0.cpu().numpy(), p1.cpu().numpy()
    greg = (g1 - g0).cpu().numpy().astype(np.float64) / gamma
    for b in range(B):
        rv, rg = O.stft_reg(x[b].astype(np.float32).astype(np.float64))
        assert abs(p0[b, 3] - rv) <= 1e-5 * rv, (b, p0[b], rv)
        assert p1[b, 3] == p0[b, 3]                       # evaluated whatever gamma is
        assert abs(p1[b, 0] - (p0[b, 0] + gamma * p0[b, 3])) <= 1e-6 * abs(p1[b, 0])
        near, nb = _near_zero_bins(x[b].astype(np.float32).astype(np.float64))
        e = rel(greg[b], rg)
        tol = 1e-4 + near * 2.0 / np.sqrt(nb)
        print('T %d clip %d: reg %.7g (oracle %.7g) grad rel-L2 %.3g (tol %.3g, %d near-zero bins)'
              % (T, b, p0[b, 3], rv, e, tol, near))
        assert e <= tol


def test_stft_reg_short_clip_is_zero(weights, dev):
    """T = 512 < one frame: no frame, reg = 0 and the gradient is untouched (oracle)."""
    T = 512
    x = torch.tensor(_inputs(1, T, 1), dtype=torch.float32, device=dev)
    eng = _engine(1, T, weights, 'fp32')
    emb_c, emb_s = eng.embeds(x)
    eng.set_targets(emb_c.clone(), emb_s[0].clone())
    p0, g0 = eng.loss_grad(x)
    g0 = g0.clone()
    eng.set_gamma(1.0)
    p1, g1 = eng.loss_grad(x)
    assert float(p1[0, 3]) == 0.0 and float(p0[0, 3]) == 0.0
    assert torch.equal(g0, g1)


def test_stft_reg_in_full_loss(weights, dev):
    """gamma > 0 in the default-style loss: total and grad against the oracle's loss_and_grad."""
    from audio_style_transfer_amd.engine import StyleEngine
    from audio_style_transfer_amd.weights import synthetic_clips
    T = 4096
    kw = dict(cont_ids=[9], style_ids=list(range(10)), gatys=False, nb_channels=128,
              cnt_channels=128)
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
    phi_c, phi_s = O.targets_from_audio(weights, xc, [xs], [xc], **kw)
    x = xc + np.random.default_rng(3).normal(0, 8, T)
    gamma = 0.1
    ref_parts, ref_g = O.loss_and_grad(x, weights, phi_c=phi_c, phi_s=phi_s, lambd=100.0,
                                       gamma=gamma, **kw)
    eng = StyleEngine(1, T, kw['cont_ids'], kw['style_ids'], lambd=100.0, gamma=gamma,
                      weights=weights)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    parts, grad = eng.loss_grad(torch.tensor(x[None], dtype=torch.float32, device=dev))
    parts = parts.cpu().numpy()[0]
    for k in range(4):
        assert abs(parts[k] - ref_parts[k]) <= 1e-4 * abs(ref_parts[k]) + 1e-7, (k, parts, ref_parts)
    e = rel(grad.cpu().numpy()[0], ref_g)
    print('gamma %.2g: grad rel-L2 %.3g' % (gamma, e))
    assert e <= 2e-3
