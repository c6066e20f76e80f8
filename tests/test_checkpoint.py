"""CPU: the native TF checkpoint-V2 reader (csrc/ckpt.cpp via ast_ckpt_*; Saver.restore,
methods.py:79-84) on bundles written by tests/tf_ckpt_writer.py (the published format; no TF
and no NSynth checkpoint here, so parity against real TF files is unpinned)."""
import os

import numpy as np
import pytest

from audio_style_transfer_amd import checkpoint as CK
from audio_style_transfer_amd._lib import AstError
from audio_style_transfer_amd.weights import synthetic_weights, weight_shapes
from tf_ckpt_writer import write_checkpoint


def _tensors():
    W = synthetic_weights(3)
    t = dict(W)
    r = np.random.default_rng(0)
    # decoder-side and bookkeeping variables the real checkpoint also holds (ignored)
    t['global_step'] = np.array(200000, dtype=np.int64)
    t['decoder/dilated_conv_1/W'] = r.normal(size=(1, 2, 512, 1024)).astype(np.float32)
    t['x_double'] = r.normal(size=(3, 5))
    t['x_half'] = r.normal(size=(7,)).astype(np.float16)
    t['x_scalar'] = np.array(1.5, dtype=np.float32)
    return W, t


@pytest.mark.parametrize('shards,block,restart', [(1, 4096, 16), (3, 256, 4), (2, 64, 1)])
def test_round_trip(tmp_path, shards, block, restart):
    W, t = _tensors()
    pre = str(tmp_path / 'model.ckpt-200000')
    write_checkpoint(pre, t, num_shards=shards, block_size=block, restart=restart)
    assert CK.is_checkpoint(pre)
    lv = dict(CK.list_variables(pre))
    assert sorted(lv) == sorted(t)
    for n, a in t.items():
        assert tuple(lv[n]) == a.shape
    got = CK.encoder_weights(pre)
    assert sorted(got) == sorted(weight_shapes())
    for n in W:
        assert got[n].dtype == np.float32 and np.array_equal(got[n], W[n]), n
    v = CK.read_variables(pre, ['x_double', 'x_half', 'x_scalar'])
    assert np.array_equal(v['x_double'], t['x_double'].astype(np.float32))
    assert np.array_equal(v['x_half'], t['x_half'].astype(np.float32))
    assert v['x_scalar'].shape == () and float(v['x_scalar']) == 1.5


def test_errors(tmp_path):
    W, t = _tensors()
    pre = str(tmp_path / 'c')
    write_checkpoint(pre, t)
    with pytest.raises(AstError, match='not a floating-point'):
        CK.read_variables(pre, ['global_step'])
    with pytest.raises(AstError, match='no variable'):
        CK.read_variables(pre, ['ae_res_31/W'])
    for bad, msg in (('data', 'CRC'), ('magic', 'magic'), ('index', 'CRC|corrupt')):
        p = str(tmp_path / bad)
        write_checkpoint(p, W, corrupt=bad)
        with pytest.raises(AstError, match=msg):
            CK.encoder_weights(p)
    os.remove(pre + '.data-00000-of-00001')
    with pytest.raises(AstError, match='cannot read'):
        CK.encoder_weights(pre)
    with pytest.raises(AstError, match='cannot read'):
        CK.list_variables(str(tmp_path / 'absent'))
    # a checkpoint without an encoder variable
    p = str(tmp_path / 'partial')
    write_checkpoint(p, {k: v for k, v in W.items() if k != 'ae_res_7/W'})
    with pytest.raises(AstError, match='ae_res_7/W'):
        CK.encoder_weights(p)
