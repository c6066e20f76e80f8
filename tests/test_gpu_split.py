"""Precision 2 ('split': fp32 storage, encoder GEMMs on split-fp16 MFMA, Gram on bf16 MFMA) vs
the fp64 CPU oracle — run on an MI355X through the C ABI.

This is configs[2]'s mode (BASELINE.json: "bf16 MFMA Gram") with the reference's fp32 encoder
arithmetic kept: every encoder operand is carried as two fp16 halves (22 significant bits,
splitwave.h), so it is held to the fp32 bars of test_gpu_parity.py:
  * extracts / embeddings:   rel-L2 <= 1e-5 (embeddings of the bf16 Gram: <= 1e-4)
  * loss parts:              rel   <= 1e-4
  * gradient d loss / d x:   rel-L2 <= 2e-3
Batch/shard invariance is bit-exact, at the bench size (B = 256, T = 16384) too.
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


@pytest.fixture(scope='module')
def dev():
    assert torch.cuda.is_available(), 'gpu tests need an MI355X'
    return torch.device('cuda', 0)


def _engine(B, T, kw, weights, precision='split'):
    from audio_style_transfer_amd.engine import StyleEngine
    return StyleEngine(B, T, kw['cont_ids'], kw['style_ids'], cnt_channels=kw['cnt_channels'],
                       nb_channels=kw['nb_channels'], gatys=kw['gatys'], weights=weights,
                       precision=precision)


_TGT = {}


def _targets(tag, T, weights):
    key = (tag, T)
    if key not in _TGT:
        kw = CASES[tag]
        xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
        xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
        _TGT[key] = O.targets_from_audio(weights, xc, [xs], [xc], **kw)
    return _TGT[key]


def _set(eng, tag, T, weights):
    phi_c, phi_s = _targets(tag, T, weights)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))


@pytest.mark.parametrize('tag', list(CASES))
def test_split_loss_grad_matches_oracle(tag, weights, golden, dev):
    T = 2048
    x = golden[tag + '_x']
    eng = _engine(1, T, CASES[tag], weights)
    _set(eng, tag, T, weights)
    parts, grad = eng.loss_grad(torch.tensor(x[None], dtype=torch.float32, device=dev))
    parts = parts.cpu().numpy()[0]
    grad = grad.cpu().numpy()[0]
    ref_parts = golden[tag + '_parts']
    for k in range(4):
        assert abs(parts[k] - ref_parts[k]) <= 1e-4 * abs(ref_parts[k]) + 1e-7, (k, parts, ref_parts)
    e = rel(grad, golden[tag + '_grad'])
    print('%s split grad rel-L2 %.3g' % (tag, e))
    assert e <= 2e-3


@pytest.mark.parametrize('T', [512, 1024, 2048, 3584])
def test_split_extracts_match_oracle(T, weights, dev):
    """Every dilation layout of the split kernels: one segment with halo rows (n >= 64),
    32-position segments with pad rows (n == 32), per-column tap masks (n < 32; and at
    T = 3584, n = 224 / 112 / 56 / 28 / 14 / 7, where a 64-position tile starts and ends inside
    a sub-sequence)."""
    kw = dict(CASES['trunc'], cont_ids=[29, 31], style_ids=[0, 30])
    x = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(3).normal(0, 4, T)
    ext, _ = O.encoder_forward(x, weights, 30, need_bottleneck=True)
    eng = _engine(1, T, kw, weights)
    eng.forward(torch.tensor(x[None], dtype=torch.float32, device=dev))
    for i in [0, 1, 4, 5, 6, 8, 9, 10, 19, 25, 29, 30, 31]:
        e = rel(eng.extract(i).cpu().numpy()[0], ext[i])
        assert e <= 1e-5, (i, e)


@pytest.mark.parametrize('tag', ['ours', 'trunc', 'gatys'])
def test_split_embeds_match_oracle(tag, weights, dev):
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
    e = rel(emb_s.cpu().numpy()[0], ref_s)
    print('%s split style embeds rel-L2 %.3g' % (tag, e))
    assert e <= 1e-4


def test_split_full_size(weights, dev):
    """BASELINE clip length (T = 16384, all 30 blocks, ours Gram L = 30) vs the oracle."""
    T = 16384
    kw = CASES['ours']
    phi_c, phi_s = _targets('ours', T, weights)
    x = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(5).normal(0, 4, T)
    ref_parts, ref_g = O.loss_and_grad(x, weights, phi_c=phi_c, phi_s=phi_s, lambd=100.0, **kw)
    eng = _engine(2, T, kw, weights)
    _set(eng, 'ours', T, weights)
    parts, grad = eng.loss_grad(torch.tensor(np.stack([x, x]), dtype=torch.float32, device=dev))
    parts, grad = parts.cpu().numpy(), grad.cpu().numpy()
    assert np.array_equal(parts[0], parts[1]) and np.array_equal(grad[0], grad[1])
    for k in range(3):
        assert abs(parts[0][k] - ref_parts[k]) <= 1e-4 * abs(ref_parts[k]) + 1e-7
    e = rel(grad[0], ref_g)
    print('split full-size grad rel-L2 %.3g' % e)
    assert e <= 2e-3


def test_split_batch_invariance_and_determinism(weights, dev):
    T = 2048
    kw = CASES['ours']
    xs = O.mu_law_numpy(synthetic_clips(3, T, 77)) + np.random.default_rng(11).normal(0, 4, (3, T))
    x3 = torch.tensor(xs, dtype=torch.float32, device=dev)
    eng3 = _engine(3, T, kw, weights)
    _set(eng3, 'ours', T, weights)
    p3, g3 = eng3.loss_grad(x3)
    p3, g3 = p3.clone(), g3.clone()
    pr, gr = eng3.loss_grad(x3)
    assert torch.equal(p3, pr) and torch.equal(g3, gr)
    eng1 = _engine(1, T, kw, weights)
    _set(eng1, 'ours', T, weights)
    for b in range(3):
        p1, g1 = eng1.loss_grad(x3[b:b + 1].contiguous())
        assert torch.equal(p1[0], p3[b]) and torch.equal(g1[0], g3[b]), b


@pytest.mark.parametrize('tag,precision', [('gatys', 'split'), ('gatys', 'fp32')])
def test_gatys_full_size(tag, precision, weights, dev):
    """configs[4]'s clip: T = 16384, all 30 blocks, Gatys Gram [30, 128, 128] (methods.py:68-74
    with --gatys) vs the oracle, in the headline split mode and in fp32 mode."""
    T = 16384
    kw = CASES[tag]
    phi_c, phi_s = _targets(tag, T, weights)
    x = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(5).normal(0, 4, T)
    ref_parts, ref_g = O.loss_and_grad(x, weights, phi_c=phi_c, phi_s=phi_s, lambd=100.0, **kw)
    eng = _engine(1, T, kw, weights, precision)
    _set(eng, tag, T, weights)
    parts, grad = eng.loss_grad(torch.tensor(x[None], dtype=torch.float32, device=dev))
    parts, grad = parts.cpu().numpy()[0], grad.cpu().numpy()[0]
    for k in range(3):
        assert abs(parts[k] - ref_parts[k]) <= 1e-4 * abs(ref_parts[k]) + 1e-7, (k, parts, ref_parts)
    e = rel(grad, ref_g)
    print('gatys %s T=16384 grad rel-L2 %.3g' % (precision, e))
    assert e <= 2e-3


@pytest.mark.parametrize('T,tag,precision', [(3584, 'ours', 'split'), (3584, 'ours', 'fp32'),
                                             (12800, 'gatys', 'split'), (12800, 'gatys', 'fp32')])
def test_odd_lengths_match_oracle(T, tag, precision, weights, dev):
    """Clip lengths whose Gram time chunks are not powers of two (T / 1024 = 3 chunks would not
    divide T = 3584 into whole stages; T / 4096 = 3 would drop rows of T = 12800): every row of
    every chunk is counted once, and D lands on its own rows only."""
    kw = dict(CASES[tag], cont_ids=[29])
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
    phi_c, phi_s = O.targets_from_audio(weights, xc, [xs], [xc], **kw)
    x = xc + np.random.default_rng(8).normal(0, 4, T)
    ref_parts, ref_g = O.loss_and_grad(x, weights, phi_c=phi_c, phi_s=phi_s, lambd=100.0, **kw)
    eng = _engine(2, T, kw, weights, precision)
    eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
    parts, grad = eng.loss_grad(torch.tensor(np.stack([x, x]), dtype=torch.float32, device=dev))
    parts, grad = parts.cpu().numpy(), grad.cpu().numpy()
    assert np.array_equal(parts[0], parts[1]) and np.array_equal(grad[0], grad[1])
    for k in range(3):
        assert abs(parts[0][k] - ref_parts[k]) <= 1e-4 * abs(ref_parts[k]) + 1e-7, (k, parts[0], ref_parts)
    e = rel(grad[0], ref_g)
    print('T=%d %s %s grad rel-L2 %.3g' % (T, tag, precision, e))
    assert e <= 2e-3


@pytest.mark.parametrize('tag,precision', [('ours', 'split'), ('ours', 'bf16'), ('gatys', 'split')])
def test_bench_size_batch(tag, precision, weights, dev):
    """configs[2] (ours) and configs[4] (--gatys) at their size: B = 256 clips of T = 16384.
    Four clip slots (first, last, two inside) are bit-identical to a B = 1 run of the same
    clip, and one matches the oracle.  At B = 256 every block-kernel workgroup walks one clip's
    tiles in order, so the split backward takes its rows 0 / 1 from the previous tile (CARRY
    rows across sub-sequences included, block_bwd_split.hip); at B = 1 each workgroup runs one
    tile and computes them with the halo MFMA tile: the bit-identity holds the two paths equal."""
    B, T = 256, 16384
    kw = dict(CASES[tag], cont_ids=[29])
    phi_c, phi_s = O.targets_from_audio(weights, O.mu_law_numpy(synthetic_clips(1, T, 1000)[0]),
                                        [O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])],
                                        [O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])], **kw)
    pc = torch.tensor(phi_c, dtype=torch.float32)
    ps = torch.tensor(phi_s, dtype=torch.float32)
    g = torch.Generator().manual_seed(5)
    xb = (torch.randn(B, T, generator=g) * 30).to(dev)
    slots = [0, 97, 180, B - 1]
    x42 = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(5).normal(0, 4, T)
    xb[97] = torch.tensor(x42, dtype=torch.float32, device=dev)
    eng = _engine(B, T, kw, weights, precision)
    eng.set_targets(pc, ps)
    pB, gB = eng.loss_grad(xb)
    pB, gB = pB.cpu(), gB.cpu()
    del eng
    torch.cuda.empty_cache()
    assert torch.isfinite(pB).all() and torch.isfinite(gB).all()
    eng1 = _engine(1, T, kw, weights, precision)
    eng1.set_targets(pc, ps)
    for b in slots:
        p1, g1 = eng1.loss_grad(xb[b:b + 1].contiguous())
        assert torch.equal(p1[0].cpu(), pB[b]) and torch.equal(g1[0].cpu(), gB[b]), b
    if precision == 'split':
        ref_parts, ref_g = O.loss_and_grad(x42, weights, phi_c=phi_c, phi_s=phi_s, lambd=100.0, **kw)
        for k in range(3):
            assert abs(float(pB[97, k]) - ref_parts[k]) <= 1e-4 * abs(ref_parts[k]) + 1e-7
        e = rel(gB[97].numpy(), ref_g)
        print('B=256 slot 97 %s split grad rel-L2 %.3g' % (tag, e))
        assert e <= 2e-3


def test_split_graph_replay_matches_eager(weights, dev):
    from audio_style_transfer_amd.engine import AdamLoop
    T = 2048
    kw = CASES['ours']
    eng = _engine(2, T, kw, weights)
    _set(eng, 'ours', T, weights)
    x0 = torch.tensor(O.mu_law_numpy(synthetic_clips(2, T, 77)), dtype=torch.float32, device=dev)
    runs = []
    for graph in (False, True):
        loop = AdamLoop(eng, x0.clone(), lr=0.5, graph=graph)
        for _ in range(4):
            loop.step()
        torch.cuda.synchronize()
        runs.append((loop.x.clone(), loop.parts.clone()))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])


@pytest.mark.parametrize('precision', ['split', 'fp32'])
def test_few_clip_gram_kernels_bit_identical(precision, dev):
    """At one clip the ours-Gram runs the 8-channel forward (k_gram_fwd_n / k_gram_fwd_fn) and a
    64-chunk backward; at 16 clips the 32-channel kernels and 4 chunks: the same clip gives the
    same loss parts and gradient bit for bit (the ours-Gram at few clips)."""
    import bench
    from audio_style_transfer_amd.engine import StyleEngine
    T, B = 16384, 16
    e16 = StyleEngine(B, T, [29], list(range(30)), precision=precision, device=dev, lambd=100.0)
    x16 = bench.make_problem(e16, list(range(B)), T, dev)
    p16, g16 = e16.loss_grad(x16)
    phi_c, phi_s = e16._targets
    k = 11
    e1 = StyleEngine(1, T, [29], list(range(30)), precision=precision, device=dev, lambd=100.0)
    e1.set_targets(phi_c[k:k + 1].clone(), phi_s[k:k + 1].clone())
    p1, g1 = e1.loss_grad(x16[k:k + 1].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(p1[0], p16[k]) and torch.equal(g1[0], g16[k])
    e16.close()
    e1.close()


def test_graph_replays_bitwise_at_bench_length(dev):
    """Every replay of a captured ast_loss_grad equals the eager call bit for bit, at the bench's
    clip length with 8 clips (one per XCD in the block kernels' tile order), with eager work
    between replays, and two engines' graphs interleaved.  (With hipMemsetAsync nodes for the
    per-call clears, replays after the first differed on 2 of 8 clips under the HIP runtime's
    graph packet capture: DESIGN.md §3, "Round 4: graph replays and the per-call clears".)"""
    import bench
    from audio_style_transfer_amd.engine import StyleEngine
    B, T = 8, 16384
    engs, xs, refs, outs, graphs = [], [], [], [], []
    for g in range(2):
        e = StyleEngine(B, T, [29], list(range(30)), precision='split', device=dev, lambd=100.0)
        x = bench.make_problem(e, list(range(g * B, (g + 1) * B)), T, dev)
        p, gr = e.loss_grad(x)
        engs.append(e)
        xs.append(x)
        refs.append((p.clone(), gr.clone()))
    for e, x in zip(engs, xs):
        p, gr = torch.empty(B, 4, device=dev), torch.empty_like(x)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            e.loss_grad(x, gr, p)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            e.loss_grad(x, gr, p)
        outs.append((p, gr))
        graphs.append(graph)
    for _ in range(3):
        for k in range(2):
            graphs[k].replay()
            torch.cuda.synchronize()
            assert torch.equal(outs[k][0], refs[k][0]) and torch.equal(outs[k][1], refs[k][1])
            engs[k].range_flags()   # eager library work between replays
    for e in engs:
        e.close()


def test_split_scale_range(weights, dev):
    """The power-of-two operand scales (splitwave.h) make the split path independent of the
    input's magnitude: the reference's initial point x = 1e-6 (methods.py:49-54, activations
    driven by the biases) and a loud x both match the oracle."""
    T = 1024
    kw = CASES['c1']
    phi_c, phi_s = _targets('c1', T, weights)
    eng = _engine(1, T, kw, weights)
    _set(eng, 'c1', T, weights)
    for x in (np.full(T, 1e-6), 3000.0 * np.sin(np.arange(T) * 0.05)):
        ref_parts, ref_g = O.loss_and_grad(x, weights, phi_c=phi_c, phi_s=phi_s, lambd=100.0, **kw)
        parts, grad = eng.loss_grad(torch.tensor(x[None], dtype=torch.float32, device=dev))
        parts = parts.cpu().numpy()[0]
        for k in range(3):
            assert abs(parts[k] - ref_parts[k]) <= 1e-4 * abs(ref_parts[k]) + 1e-7, (k, parts, ref_parts)
        e = rel(grad.cpu().numpy()[0], ref_g)
        print('x scale %.3g: grad rel-L2 %.3g' % (np.abs(x).max(), e))
        assert e <= 2e-3


@pytest.mark.parametrize('kind', ['dr4', 'dr025', 'alt2', 'student_t', 'bias100'])
def test_split_weight_statistics(kind, dev):
    """The split mode's range management (per-block weight exponents; the analytic bounds
    |u| <= wdn max|e| + bdm and |W_r tot| <= wrn max|tot| that set the intermediates' scales)
    under weight sets unlike uniform_unit_scaling — W_d / W_r scaled x4 / x0.25, blocks
    alternately x2 / x0.5, heavy-tailed Student-t(3) weights, biases x100 — held to the fp32
    bars against the fp64 oracle, the fp32 mode beside it, and no clip flagged."""
    from audio_style_transfer_amd.weights import stressed_weights
    T = 2048
    W = stressed_weights(kind)
    kw = dict(CASES['ours'], cont_ids=[29])
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
    phi_c, phi_s = O.targets_from_audio(W, xc, [xs], [xc], **kw)
    x = xc + np.random.default_rng(6).normal(0, 4, T)
    ref_parts, ref_g = O.loss_and_grad(x, W, phi_c=phi_c, phi_s=phi_s, lambd=100.0, **kw)
    errs = {}
    for precision in ('split', 'fp32'):
        eng = _engine(1, T, kw, W, precision)
        eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
        parts, grad = eng.loss_grad(torch.tensor(x[None], dtype=torch.float32, device=dev))
        flags = eng.range_flags().cpu().numpy()
        parts = parts.cpu().numpy()[0]
        assert flags[0] == 0, (precision, flags)
        for k in range(3):
            assert abs(parts[k] - ref_parts[k]) <= 1e-4 * abs(ref_parts[k]) + 1e-7, (precision, k, parts, ref_parts)
        errs[precision] = rel(grad.cpu().numpy()[0], ref_g)
        eng.close()
    print('%s: grad rel-L2 split %.3g, fp32 %.3g' % (kind, errs['split'], errs['fp32']))
    assert errs['split'] <= 2e-3


def test_range_flags(weights, dev):
    """ast_range_flags: 0 on ordinary inputs; a clip driven past the split representation
    (x ~ 1e30: max |e_0| ~ 1e28 > 2^74) is flagged, its neighbour is not; the flags are sticky
    (an in-range evaluation after it leaves them set) until ast_range_flags_reset."""
    T = 1024
    kw = CASES['c1']
    eng = _engine(2, T, kw, weights)
    _set(eng, 'c1', T, weights)
    x = O.mu_law_numpy(synthetic_clips(2, T, 77))
    good = torch.tensor(x, dtype=torch.float32, device=dev)
    eng.loss_grad(good)
    assert eng.range_flags().cpu().tolist() == [0, 0]
    x[1] = 1e30
    eng.loss_grad(torch.tensor(x, dtype=torch.float32, device=dev))
    f = eng.range_flags().cpu().tolist()
    assert f[0] == 0 and f[1] & 2, f
    eng.loss_grad(good)                       # back in range: the flag stays
    assert eng.range_flags().cpu().tolist() == f
    assert eng.range_flags(reset=True).cpu().tolist() == f
    eng.loss_grad(good)
    assert eng.range_flags().cpu().tolist() == [0, 0]


@pytest.mark.parametrize('gatys', [False, True])
def test_fused_content_tap_phi_at_buffer_end(gatys, weights, dev):
    """the fused content tap's phi loads (ours-Gram and, since round 4, Gatys backward)
    are masked by cnt_channels.  Per-clip phi_c of
    cnt_channels 32 for 6 clips of 16384 samples is exactly 12 MiB, a caching-allocator segment of
    its own (requests >= 10 MiB are rounded to 2 MiB and not split), so on the last clip's last row
    a quad past the tap's 32 channels would read past the allocation; the split result must
    equal the fp32 kernels' to the fp32 bars."""
    B, T = 6, 16384
    kw = dict(cont_ids=[29], style_ids=list(range(30)), gatys=gatys, nb_channels=128, cnt_channels=32)
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
    torch.manual_seed(0)
    phi_c = torch.randn(B, T, 32).mul_(0.5)
    x = torch.tensor(np.stack([xc + 3.0 * b for b in range(B)]), dtype=torch.float32, device=dev)
    out = {}
    for precision in ('split', 'fp32'):
        eng = _engine(B, T, kw, weights, precision)
        _, emb_s = eng.embeds(torch.tensor(np.stack([xs] * B), dtype=torch.float32, device=dev),
                              content=False)
        pc = torch.empty(B * T * 32, dtype=torch.float32, device=dev)
        assert pc.numel() * 4 == 12 << 20
        pc.copy_(phi_c.reshape(-1))
        eng.set_targets(pc.view(B, T, 32), emb_s[0].clone())
        parts, grad = eng.loss_grad(x)
        out[precision] = (parts.cpu().numpy(), grad.cpu().numpy())
        eng.close()
    for b in range(B):
        for k in range(3):
            assert abs(out['split'][0][b, k] - out['fp32'][0][b, k]) <= 1e-4 * abs(out['fp32'][0][b, k]) + 1e-7, (b, k, out)
        assert rel(out['split'][1][b], out['fp32'][1][b]) <= 2e-3


def test_loss_grad_phases_and_clip_groups(weights, dev):
    """ast_loss_grad_phase: phase 1 + phase 2 equal ast_loss_grad bit for bit, and phase 2 alone
    is refused.  engine.AdamGroups (two engines of 2 clips on half the CUs each, phase-shifted
    graphs on two streams) leaves every clip where one AdamLoop over all 4 clips leaves it."""
    from audio_style_transfer_amd._lib import AstError
    from audio_style_transfer_amd.engine import AdamGroups, AdamLoop
    T, B = 2048, 4
    kw = CASES['ours']
    x0 = torch.tensor(np.stack([O.mu_law_numpy(synthetic_clips(1, T, 300 + b)[0]) for b in range(B)]),
                      dtype=torch.float32, device=dev)
    eng = _engine(B, T, kw, weights)
    _set(eng, 'ours', T, weights)
    p0, g0 = eng.loss_grad(x0)
    p1, g1 = torch.empty_like(p0), torch.empty_like(g0)
    with pytest.raises(AstError, match='phase 1 first'):
        eng.loss_grad_phase(x0, g1, p1, 2)
    eng.loss_grad_phase(x0, g1, p1, 1)
    eng.loss_grad_phase(x0, g1, p1, 2)
    assert torch.equal(p0, p1) and torch.equal(g0, g1)
    # between the phases the tapped tensors hold D, not activations (extracts are
    # refused), and a forward / new targets / new gamma in between void phase 1
    for between in (lambda: eng.forward(x0), lambda: _set(eng, 'ours', T, weights),
                    lambda: eng.set_gamma(0.0)):
        eng.loss_grad_phase(x0, g1, p1, 1)
        with pytest.raises(AstError, match='ast_forward has not run'):
            eng.extract(29)
        between()
        with pytest.raises(AstError, match='phase 1 first'):
            eng.loss_grad_phase(x0, g1, p1, 2)
    eng.loss_grad_phase(x0, g1, p1, 1)
    eng.loss_grad_phase(x0, g1, p1, 2)
    assert torch.equal(p0, p1) and torch.equal(g0, g1)
    # ast_range_flags_last: the last evaluation alone; ast_range_flags: sticky since the reset
    assert not eng.range_flags_last().any()
    loop = AdamLoop(eng, x0.clone(), lr=1.0, graph=True)
    for _ in range(3):
        loop.step()
    torch.cuda.synchronize()
    ref = loop.x.clone()
    engs = [_engine(2, T, kw, weights) for _ in range(2)]
    for e in engs:
        _set(e, 'ours', T, weights)
    grp = AdamGroups(engs, [x0[:2].clone(), x0[2:].clone()], lr=1.0)
    for _ in range(3):
        grp.step()
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(grp.xs), ref)
    assert torch.equal(torch.cat(grp.parts), loop.parts)


@pytest.mark.parametrize('stages', ['2', '3'])
def test_gatys_split_kernels(stages, weights, golden, dev, monkeypatch):
    """The split Gatys kernels (16x16x32 backward with the fused content tap; the forward with 2
    or 3 load stages, ASTYLE_GATYS_STAGES) against the golden 'gatys' case at the fp32 bars, and
    at B = 3 every slot equal to that clip alone."""
    monkeypatch.setenv('ASTYLE_GATYS_STAGES', stages)
    form = stages
    T = 2048
    x = golden['gatys_x']
    eng = _engine(1, T, CASES['gatys'], weights)
    _set(eng, 'gatys', T, weights)
    parts, grad = eng.loss_grad(torch.tensor(x[None], dtype=torch.float32, device=dev))
    parts, grad = parts.cpu().numpy()[0], grad.cpu().numpy()[0]
    ref_parts = golden['gatys_parts']
    for k in range(4):
        assert abs(parts[k] - ref_parts[k]) <= 1e-4 * abs(ref_parts[k]) + 1e-7, (form, k, parts, ref_parts)
    e = rel(grad, golden['gatys_grad'])
    print('gatys form %s: grad rel-L2 %.3g' % (form, e))
    assert e <= 2e-3
    xs = np.stack([x, x + 3.0, x - 5.0])
    eng3 = _engine(3, T, CASES['gatys'], weights)
    _set(eng3, 'gatys', T, weights)
    p3, g3 = eng3.loss_grad(torch.tensor(xs, dtype=torch.float32, device=dev))
    assert np.array_equal(p3.cpu().numpy()[0], parts) and np.array_equal(g3.cpu().numpy()[0], grad)
