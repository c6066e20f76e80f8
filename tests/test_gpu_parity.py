"""HIP path (libastyle.so through its C ABI) vs the CPU oracle — run on an MI355X.

Tolerances (fp32 storage + fp32 MFMA, fp32 accumulation, against the fp64 oracle):
  * extracts / embeddings:   rel-L2 <= 1e-5
  * loss parts:              rel   <= 1e-4
  * gradient d loss / d x:   rel-L2 <= 2e-3   (the fp32 floor: a plain fp32 restatement of the
                             reference is 3e-4 rel-L2 from fp64 on this problem)
Batch/shard invariance is checked bit-exactly.
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
    'trunc': dict(cont_ids=[25, 31], style_ids=[3, 7], gatys=False, nb_channels=64,
                  cnt_channels=16),
    'gatys': dict(cont_ids=[29], style_ids=list(range(30)), gatys=True, nb_channels=128,
                  cnt_channels=128),
}


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _engine(B, T, kw, weights, **extra):
    from audio_style_transfer_amd.engine import StyleEngine
    return StyleEngine(B, T, kw['cont_ids'], kw['style_ids'], cnt_channels=kw['cnt_channels'],
                       nb_channels=kw['nb_channels'], gatys=kw['gatys'], weights=weights, **extra)


_TGT = {}


def _targets(tag, T, weights):
    key = (tag, T)
    if key not in _TGT:
        kw = CASES[tag]
        xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
        xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
        _TGT[key] = O.targets_from_audio(weights, xc, [xs], [xc], **kw)
    return _TGT[key]


@pytest.fixture(scope='module')
def dev():
    assert torch.cuda.is_available(), 'gpu tests need an MI355X'
    return torch.device('cuda', 0)


@pytest.mark.parametrize('tag', list(CASES))
def test_loss_grad_matches_oracle(tag, weights, golden, dev):
    T = 2048
    kw = CASES[tag]
    phi_c, phi_s = _targets(tag, T, weights)
    x = golden[tag + '_x']
    eng = _engine(1, T, kw, weights)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    parts, grad = eng.loss_grad(torch.tensor(x[None], dtype=torch.float32, device=dev))
    torch.cuda.synchronize()
    parts = parts.cpu().numpy()[0]
    grad = grad.cpu().numpy()[0]
    ref_parts = golden[tag + '_parts']
    for k in range(4):      # parts[3]: the STFT regulariser, evaluated at gamma = 0 as TF does
        assert abs(parts[k] - ref_parts[k]) <= 1e-4 * abs(ref_parts[k]) + 1e-7, (k, parts, ref_parts)
    e = rel(grad, golden[tag + '_grad'])
    print('%s grad rel-L2 %.3g parts %s vs %s' % (tag, e, parts, ref_parts))
    assert e <= 2e-3


@pytest.mark.parametrize('T', [512, 2048])
def test_extracts_match_oracle(T, weights, dev):
    kw = CASES['trunc']
    x = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(3).normal(0, 4, T)
    ext, _ = O.encoder_forward(x, weights, 30, need_bottleneck=True)
    eng = _engine(1, T, dict(kw, cont_ids=[29, 31], style_ids=[0, 30]), weights)
    eng.forward(torch.tensor(x[None], dtype=torch.float32, device=dev))
    for i in [0, 1, 8, 9, 10, 19, 25, 29, 30, 31]:
        got = eng.extract(i).cpu().numpy()[0]
        e = rel(got, ext[i])
        assert e <= 1e-5, (i, e)


@pytest.mark.parametrize('tag', ['ours', 'trunc', 'gatys'])
def test_embeds_match_oracle(tag, weights, dev):
    T = 2048
    kw = CASES[tag]
    xmu = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    nb = O.needed_blocks(kw['cont_ids'], kw['style_ids'])
    ext, _ = O.encoder_forward(xmu, weights, nb, need_bottleneck=31 in kw['cont_ids'])
    ref_c = O.content_embeds(ext, kw['cont_ids'], kw['cnt_channels'])
    ref_s = O.style_embeds(ext, kw['style_ids'], kw['gatys'], kw['nb_channels'])
    eng = _engine(1, T, kw, weights)
    emb_c, emb_s = eng.embeds(torch.tensor(xmu[None], dtype=torch.float32, device=dev))
    assert rel(emb_c.cpu().numpy()[0], ref_c) <= 1e-5
    assert rel(emb_s.cpu().numpy()[0], ref_s) <= 1e-5


@pytest.mark.parametrize('precision,tol', [('fp32', 2e-3), ('bf16', None)])
def test_gatys_duplicate_taps(precision, tol, weights, dev):
    """--gatys with repeated / aliased style taps (extracts 29 and 30 are one tensor,
    model.py:119) and a tensor that is both a content and a style tap: the S~ fold and the
    in-place D + content-grad add."""
    T = 1024
    kw = dict(cont_ids=[4, 29], style_ids=[29, 30, 2, 4], gatys=True, nb_channels=128,
              cnt_channels=64)
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
    phi_c, phi_s = O.targets_from_audio(weights, xc, [xs], [xc], **kw)
    x = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(5).normal(0, 4, T)
    ref_parts, ref_g = O.loss_and_grad(x, weights, phi_c=phi_c, phi_s=phi_s, lambd=100.0, **kw)
    eng = _engine(2, T, kw, weights, precision=precision)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    parts, grad = eng.loss_grad(torch.tensor(np.stack([x, x]), dtype=torch.float32, device=dev))
    parts, grad = parts.cpu().numpy(), grad.cpu().numpy()
    assert np.array_equal(grad[0], grad[1])
    ptol = 1e-4 if tol else 1e-2
    for k in range(3):
        assert abs(parts[0][k] - ref_parts[k]) <= ptol * abs(ref_parts[k]) + 1e-7, (k, parts[0], ref_parts)
    if tol:
        assert rel(grad[0], ref_g) <= tol, rel(grad[0], ref_g)
    else:
        cos = float(np.dot(grad[0], ref_g) / np.linalg.norm(grad[0]) / np.linalg.norm(ref_g))
        assert cos >= 0.98 and rel(grad[0], ref_g) <= 0.25, (cos, rel(grad[0], ref_g))


def test_batch_and_shard_invariance(weights, dev):
    """A clip's result is bit-identical whichever batch slot (shard) it runs in."""
    T = 2048
    kw = CASES['ours']
    phi_c, phi_s = _targets('ours', T, weights)
    rng = np.random.default_rng(11)
    xs = O.mu_law_numpy(synthetic_clips(3, T, 77)) + rng.normal(0, 4, (3, T))
    x3 = torch.tensor(xs, dtype=torch.float32, device=dev)
    eng3 = _engine(3, T, kw, weights)
    eng3.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    p3, g3 = eng3.loss_grad(x3)
    eng1 = _engine(1, T, kw, weights)
    eng1.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    for b in range(3):
        p1, g1 = eng1.loss_grad(x3[b:b + 1].contiguous())
        assert torch.equal(p1[0], p3[b]) and torch.equal(g1[0], g3[b]), b
    # per-clip targets: a batch whose targets are all the shared one gives the same result
    eng3.set_targets(torch.tensor(phi_c, dtype=torch.float32)[None].repeat(3, 1, 1),
                     torch.tensor(phi_s, dtype=torch.float32)[None].repeat(3, 1, 1, 1))
    p3b, g3b = eng3.loss_grad(x3)
    assert torch.equal(p3b, p3) and torch.equal(g3b, g3)


def test_repeat_is_deterministic(weights, dev):
    T = 2048
    kw = CASES['ours']
    phi_c, phi_s = _targets('ours', T, weights)
    eng = _engine(2, T, kw, weights)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    x = torch.randn(2, T, device=dev) * 30
    pa, ga = eng.loss_grad(x)
    pa, ga = pa.clone(), ga.clone()
    pb, gb = eng.loss_grad(x)
    assert torch.equal(pa, pb) and torch.equal(ga, gb)


def test_adam_step(weights, dev):
    eng = _engine(2, 512, CASES['c1'], weights)
    g = torch.randn(2, 512, device=dev)
    x = torch.randn(2, 512, device=dev)
    m = torch.zeros_like(x)
    v = torch.zeros_like(x)
    xr, mr, vr = x.clone().double(), m.clone().double(), v.clone().double()
    for step in (1, 2, 3):
        eng.adam_step(x, m, v, g, step, lr=0.5)
        gd = g.double()
        mr = 0.9 * mr + 0.1 * gd
        vr = 0.999 * vr + 0.001 * gd * gd
        xr = xr - 0.5 * (mr / (1 - 0.9 ** step)) / ((vr / (1 - 0.999 ** step)).sqrt() + 1e-8)
    assert torch.allclose(x.double(), xr, rtol=1e-5, atol=1e-5)


def test_full_size_default_config(weights, dev):
    """BASELINE sizes (T=16384, 30 blocks, ours Gram L=30): one evaluation vs the oracle."""
    T = 16384
    kw = CASES['ours']
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
    phi_c, phi_s = O.targets_from_audio(weights, xc, [xs], [xc], **kw)
    x = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(5).normal(0, 4, T)
    ref_parts, ref_g = O.loss_and_grad(x, weights, phi_c=phi_c, phi_s=phi_s, lambd=100.0, **kw)
    eng = _engine(2, T, kw, weights)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    xt = torch.tensor(np.stack([x, x]), dtype=torch.float32, device=dev)
    parts, grad = eng.loss_grad(xt)
    parts = parts.cpu().numpy()
    grad = grad.cpu().numpy()
    assert np.array_equal(parts[0], parts[1]) and np.array_equal(grad[0], grad[1])
    for k in range(3):
        assert abs(parts[0][k] - ref_parts[k]) <= 1e-4 * abs(ref_parts[k]) + 1e-7
    e = rel(grad[0], ref_g)
    print('full-size grad rel-L2 %.3g' % e)
    assert e <= 2e-3


# --------------------------------------------------------------------------- bf16 path
# Tolerances for precision='bf16' (bf16 storage + bf16 MFMA, fp32 accumulation).  The bf16
# gradient is the exact gradient of the bf16-rounded network: a CPU emulation
# (tools/bf16_emulate.py) attributes ~11% rel-L2 of it to forward activation/weight rounding
# over 30 blocks and ~0.5% to the bf16 backward chain.  Bounds:
#   extracts / embeddings rel-L2 <= 2e-2, loss parts rel <= 1e-2,
#   gradient cosine >= 0.98 and rel-L2 <= 0.25.
@pytest.mark.parametrize('tag', list(CASES))
def test_bf16_loss_grad_close_to_oracle(tag, weights, golden, dev):
    T = 2048
    kw = CASES[tag]
    phi_c, phi_s = _targets(tag, T, weights)
    x = golden[tag + '_x']
    eng = _engine(1, T, kw, weights, precision='bf16')
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    parts, grad = eng.loss_grad(torch.tensor(x[None], dtype=torch.float32, device=dev))
    parts = parts.cpu().numpy()[0]
    grad = grad.cpu().numpy()[0]
    ref_parts, ref_g = golden[tag + '_parts'], golden[tag + '_grad']
    for k in range(3):
        assert abs(parts[k] - ref_parts[k]) <= 1e-2 * abs(ref_parts[k]) + 1e-6, (k, parts, ref_parts)
    cos = float(np.dot(grad, ref_g) / np.linalg.norm(grad) / np.linalg.norm(ref_g))
    assert cos >= 0.98 and rel(grad, ref_g) <= 0.25, (cos, rel(grad, ref_g))


def _bf16(a):
    """Round to bf16 (RNE) and back to float64."""
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(torch.bfloat16)
    return t.to(torch.float32).numpy().astype(np.float64)


@pytest.mark.parametrize('tag,T', [('c1', 2048), ('trunc', 2048), ('ours', 2048), ('gatys', 2048),
                                   ('ours', 16384)])
def test_bf16_backward_linearized(tag, T, weights, dev):
    """The bf16 backward against the fp64 backward linearised at the GPU's own bf16 forward:
    its activations (read back exactly), the relu patterns they imply, the bf16-rounded block
    weights and the loss gradients of its own extracts.  What remains is the backward's own
    rounding (g_u, D and the chain are stored in bf16), so a wrong halo row, mask bit, tap or
    direct-gradient add at any dilation shows up far above the bound.  T = 16384 is the bench
    size, where dilations 128 / 256 / 512 give the one-segment / 64 / 32-position layouts."""
    kw = CASES[tag]
    phi_c, phi_s = _targets(tag, T, weights)
    x = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(5).normal(0, 4, T)
    nb = O.needed_blocks(kw['cont_ids'], kw['style_ids'])
    eng = _engine(1, T, kw, weights, precision='bf16')
    xt = torch.tensor(x[None], dtype=torch.float32, device=dev)
    eng.forward(xt)
    ext = [eng.extract(i).cpu().numpy()[0].astype(np.float64) for i in range(nb)]
    if nb == 30:
        ext.append(ext[29])
        if 31 in kw['cont_ids']:
            ext.append(eng.extract(31).cpu().numpy()[0].astype(np.float64))
    Wq = {k: (_bf16(v) if k.endswith('/W') and ('dilated' in k or 'res_' in k) else np.asarray(v, np.float64))
          for k, v in weights.items()}
    e0 = _bf16(O.conv1d_same((x / 128.0)[:, None], Wq['ae_startconv/W'], Wq['ae_startconv/biases'], 1))
    es = [e0] + ext[:nb]
    us = [O.conv1d_same(O.relu(es[l]), Wq['ae_dilatedconv_%d/W' % (l + 1)],
                        Wq['ae_dilatedconv_%d/biases' % (l + 1)], O.dilation_of(l)) for l in range(nb)]
    _, _, grads = O.tap_terms(ext, cont_ids=kw['cont_ids'], style_ids=kw['style_ids'], phi_c=phi_c,
                              phi_s=phi_s, lambd=100.0, gatys=kw['gatys'],
                              nb_channels=kw['nb_channels'], cnt_channels=kw['cnt_channels'])
    ref = O.encoder_backward({'es': es, 'us': us, 'n_blocks': nb}, Wq, grads)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    _, grad = eng.loss_grad(xt)
    grad = grad.cpu().numpy()[0]
    e = rel(grad, ref)
    print('%s bf16 backward vs linearised fp64: rel-L2 %.3g' % (tag, e))
    assert e <= 1.5e-2, e


@pytest.mark.parametrize('T', [512, 1024, 2048])
def test_bf16_extracts_and_embeds(T, weights, dev):
    kw = dict(CASES['trunc'], cont_ids=[29, 31], style_ids=[0, 9, 30])
    x = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(3).normal(0, 4, T)
    ext, _ = O.encoder_forward(x, weights, 30, need_bottleneck=True)
    eng = _engine(1, T, kw, weights, precision='bf16')
    xt = torch.tensor(x[None], dtype=torch.float32, device=dev)
    eng.forward(xt)
    for i in [0, 9, 19, 29, 30, 31]:
        assert rel(eng.extract(i).cpu().numpy()[0], ext[i]) <= 2e-2, i
    emb_c, emb_s = eng.embeds(xt)
    assert rel(emb_c.cpu().numpy()[0], O.content_embeds(ext, kw['cont_ids'], kw['cnt_channels'])) <= 2e-2
    assert rel(emb_s.cpu().numpy()[0], O.style_embeds(ext, kw['style_ids'], False, kw['nb_channels'])) <= 2e-2


def test_bf16_batch_invariance(weights, dev):
    T = 2048
    kw = CASES['ours']
    phi_c, phi_s = _targets('ours', T, weights)
    xs = O.mu_law_numpy(synthetic_clips(3, T, 77)) + np.random.default_rng(11).normal(0, 4, (3, T))
    x3 = torch.tensor(xs, dtype=torch.float32, device=dev)
    eng3 = _engine(3, T, kw, weights, precision='bf16')
    eng3.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    p3, g3 = eng3.loss_grad(x3)
    eng1 = _engine(1, T, kw, weights, precision='bf16')
    eng1.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    for b in range(3):
        p1, g1 = eng1.loss_grad(x3[b:b + 1].contiguous())
        assert torch.equal(p1[0], p3[b]) and torch.equal(g1[0], g3[b]), b


def test_bf16_gatys_embeds(weights, dev):
    T = 2048
    kw = CASES['gatys']
    xmu = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    ext, _ = O.encoder_forward(xmu, weights, 30)
    ref_s = O.style_embeds(ext, kw['style_ids'], True)
    eng = _engine(1, T, kw, weights, precision='bf16')
    _, emb_s = eng.embeds(torch.tensor(xmu[None], dtype=torch.float32, device=dev), content=False)
    assert rel(emb_s.cpu().numpy()[0], ref_s) <= 2e-2


@pytest.mark.parametrize('precision', ['fp32', 'bf16'])
def test_graph_replay_matches_eager(precision, weights, dev):
    """The hipGraph-captured step (loss_grad + device-counter Adam) replays bit-identically to
    eager steps, and the device-counter Adam equals the host-counter one."""
    from audio_style_transfer_amd.engine import AdamLoop
    T = 2048
    kw = CASES['ours']
    phi_c, phi_s = _targets('ours', T, weights)
    eng = _engine(2, T, kw, weights, precision=precision)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    x0 = torch.tensor(O.mu_law_numpy(synthetic_clips(2, T, 77)), dtype=torch.float32, device=dev)
    runs = []
    for graph in (False, True):
        loop = AdamLoop(eng, x0.clone(), lr=0.5, graph=graph)
        for _ in range(4):
            loop.step()
        torch.cuda.synchronize()
        runs.append((loop.x.clone(), loop.parts.clone(), int(loop.step_dev.item())))
    assert runs[0][2] == runs[1][2] == 4
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])
    # host-counter Adam, eager
    x = x0.clone()
    m = torch.zeros_like(x)
    v = torch.zeros_like(x)
    for k in range(1, 5):
        _, g = eng.loss_grad(x)
        eng.adam_step(x, m, v, g, k, lr=0.5)
    torch.cuda.synchronize()
    assert torch.equal(x, runs[0][0])   # same pow_int bias correction on host and device
