"""ast_restore (Saver.restore, methods.py:79-84) on a TF checkpoint-V2 bundle written by
tests/tf_ckpt_writer.py: the restored context computes bit-identically to one given the same
weights through ast_set_weight; GatysNet(checkpoint_path=<prefix>) loads them; a bundle
missing an encoder variable fails loudly."""
import numpy as np
import pytest
import torch

from audio_style_transfer_amd._lib import AstError
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
from tf_ckpt_writer import write_checkpoint

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('precision', ['fp32', 'split'])
def test_restore_matches_set_weight(tmp_path, precision):
    from audio_style_transfer_amd.engine import StyleEngine
    from oracle import astyle_oracle as O
    dev = torch.device('cuda', 0)
    W = synthetic_weights(3)
    t = dict(W)
    t['global_step'] = np.array(200000, dtype=np.int64)
    t['decoder/W'] = np.ones((4, 4), np.float32)
    pre = str(tmp_path / 'model.ckpt-200000')
    write_checkpoint(pre, t, num_shards=2, block_size=512)
    T = 2048
    kw = dict(cont_ids=[25], style_ids=list(range(30)))
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    phi_c = torch.randn(T, 128)
    phi_s = torch.rand(128, 30, 30) * 0.01
    x = torch.tensor(xc[None], dtype=torch.float32, device=dev)
    outs = []
    for mode in ('set', 'restore'):
        eng = StyleEngine(1, T, kw['cont_ids'], kw['style_ids'], precision=precision, device=dev,
                          weights=W if mode == 'set' else None)
        if mode == 'restore':
            eng.restore(pre)
        eng.set_targets(phi_c, phi_s)
        p, g = eng.loss_grad(x)
        outs.append((p.clone(), g.clone()))
        eng.close()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    # a bundle without one encoder variable
    bad = str(tmp_path / 'partial')
    write_checkpoint(bad, {k: v for k, v in W.items() if k != 'ae_dilatedconv_30/biases'})
    eng = StyleEngine(1, T, kw['cont_ids'], kw['style_ids'], precision=precision, device=dev)
    with pytest.raises(AstError, match='ae_dilatedconv_30/biases'):
        eng.restore(bad)
    # the right element count in another layout: refused, as Saver.restore does
    wrong = dict(W)
    wrong['ae_dilatedconv_7/W'] = np.ascontiguousarray(W['ae_dilatedconv_7/W'].reshape(3, 128, 128))
    bad2 = str(tmp_path / 'reshaped')
    write_checkpoint(bad2, wrong)
    with pytest.raises(AstError, match=r'ae_dilatedconv_7/W: checkpoint shape \[3,128,128\]'):
        eng.restore(bad2)
    eng.close()


def test_gatysnet_reads_checkpoint_prefix(tmp_path):
    from audio_style_transfer_amd.methods import GatysNet
    W = synthetic_weights(5)
    pre = str(tmp_path / 'model.ckpt-200000')
    write_checkpoint(pre, W)
    net = GatysNet(str(tmp_path), pre, str(tmp_path / 'log'), str(tmp_path / 'fig'), stack=0,
                   batch_size=4096, plots=False)
    assert sorted(net.weights) == sorted(W)
    assert all(np.array_equal(net.weights[k], W[k]) for k in W)
