"""CPU: the drop-in host layer (methods.py CLI surface, style-layer resolution, output naming,
audio I/O) — no GPU."""
import json
import os

import numpy as np
import pytest

from audio_style_transfer_amd import methods, utils
from audio_style_transfer_amd.engine import resolve_style_ids

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def test_cli_surface_matches_reference():
    """Every option of the reference CLI (methods.py:244-267) exists with the same type,
    default and nargs (reference_cli.json was extracted from the reference's source)."""
    with open(os.path.join(GOLD, 'reference_cli.json')) as f:
        ref = json.load(f)
    parser = methods.make_parser()
    actions = {tuple(a.option_strings) or (a.dest,): a for a in parser._actions}
    for opt in ref:
        key = tuple(opt['names'])
        assert key in actions, key
        a = actions[key]
        kw = opt['kwargs']
        if 'type' in kw:
            assert a.type.__name__ == kw['type'], key
        if 'default' in kw:
            assert a.default == kw['default'], key
        if 'nargs' in kw:
            assert a.nargs == kw['nargs'], key
        if 'const' in kw:
            assert a.const == kw['const'], key


def test_cli_parses_readme_example():
    """README.md:17 example."""
    a = methods.make_parser().parse_args(
        'pachelbel organ --epochs 100 --cont_lyrs 25 --stack 0 --lambd 100 --gamma 0'.split())
    assert a.cont_lyrs == [25] and a.stack == 0 and a.lambd == 100.0 and a.gamma == 0.0
    assert a.batch_size == 16384 and a.gatys is False and a.precision == 'split'
    assert methods.make_parser().parse_args(['a', 'b', '--gatys']).gatys is True


def test_output_dir_ignores_added_flags(tmp_path):
    a = methods.make_parser().parse_args(['pachelbel', 'organ', '--stack', '0', '--precision', 'bf16'])
    d = methods.get_dir(str(tmp_path), a)
    assert 'precision' not in d and os.path.isdir(d)
    assert os.path.basename(d).startswith('ours__btch_16384_')


def test_split_range_guard():
    """GatysNet._split_out_of_range: AST_RANGE_* flags 1/2/4 of a split evaluation switch the run
    to the fp32 kernels; 8 (operands below 2^-60) only warns, once."""
    import torch
    from audio_style_transfer_amd import _lib

    class Eng:
        def __init__(self, f):
            self.f = f

        def range_flags(self):
            return torch.tensor([0, self.f], dtype=torch.int32)

    net = methods.GatysNet.__new__(methods.GatysNet)
    logs = []
    assert not net._split_out_of_range(Eng(0), logs.append)
    for f in (_lib.RANGE_NONFINITE, _lib.RANGE_ACT, _lib.RANGE_GRAD, _lib.RANGE_ACT | _lib.RANGE_TINY):
        assert net._split_out_of_range(Eng(f), logs.append)
    assert len(logs) == 4 and 'fp32' in logs[0]
    with pytest.warns(UserWarning):
        net2 = methods.GatysNet.__new__(methods.GatysNet)
        assert not net2._split_out_of_range(Eng(_lib.RANGE_TINY), logs.append)


def test_style_layer_resolution():
    """methods.py:60-66."""
    assert resolve_style_ids(None, None) == list(range(30))
    assert resolve_style_ids(1, None) == list(range(10, 20))
    assert resolve_style_ids(0, [3, 7]) == [3, 7]
    with pytest.raises(AssertionError):
        resolve_style_ids(None, 5)


def test_wav_roundtrip_and_channel_select(tmp_path):
    from scipy.io import wavfile
    sr = 16000
    t = np.arange(sr) / sr
    st = np.stack([np.sin(2 * np.pi * 440 * t), 0.5 * np.sin(2 * np.pi * 220 * t)], axis=1)
    p = str(tmp_path / 'a.wav')
    wavfile.write(p, sr, (st * 32767).astype(np.int16))
    a0, r = utils.load_audio(p, sr, audio_channel=0)
    a1, _ = utils.load_audio(p, sr, audio_channel=1)
    assert r == sr and a0.dtype == np.float32 and a0.shape == (sr,)
    assert abs(np.max(np.abs(a0)) - 1.0) < 1e-3 and abs(np.max(np.abs(a1)) - 0.5) < 1e-3
    a8, r8 = utils.load_audio(p, 8000, audio_channel=0)
    assert r8 == 8000 and a8.shape == (sr // 2,)
    q = str(tmp_path / 'b.wav')
    utils.write_wav(q, a0, sr)
    b, _ = utils.load_audio(q, sr)
    assert np.array_equal(b, a0)


def test_late_and_start_offsets():
    """methods.py:39 and 195: st = int(start*sr - late)."""
    late = (16384 - (16384 // 4096) * 4000) // 2
    assert late == 192 and int(1.0 * 16000 - late) == 15808


def test_stft_regularizer_matches_oracle():
    """torch.stft + autograd restatement vs the oracle's closed-form gradient
    (utils.py:92-104 abs/sign/inv_mu_law semantics, methods.py:121-123)."""
    torch = pytest.importorskip('torch')
    from oracle import astyle_oracle as O
    rng = np.random.default_rng(4)
    x = rng.normal(0, 30, (2, 4096))
    x[0, :7] = 0.0                      # inv_mu_law's x == 0 branch
    from oracle import torch_restatement as TR
    val, g = TR.stft_reg(torch.tensor(x))
    for b in range(2):
        rv, rg = O.stft_reg(x[b])
        assert abs(float(val[b]) - rv) <= 1e-10 * abs(rv)
        assert np.linalg.norm(g[b].numpy() - rg) <= 1e-9 * np.linalg.norm(rg)


def test_kaiser_best_resampler():
    """utils.resample_kaiser_best restates librosa's default resampler (resampy 0.2 'kaiser_best'
    + fix_length; parity unpinned: neither library is in the image): output length ceil(n r),
    float32, channels independent, identity at equal rates, and a 440 Hz tone reproduced to
    fp32 round-off for integer rate ratios (to 0.3 % at 44.1 -> 16 kHz, resampy's truncated
    table step)."""
    sr0 = 8000
    t = np.arange(sr0) / sr0
    x = np.sin(2 * np.pi * 440 * t).astype(np.float32)
    assert utils.resample_kaiser_best(x, sr0, sr0) is not None
    assert np.array_equal(utils.resample_kaiser_best(x, sr0, sr0), x)
    for sr1, tol in ((16000, 1e-5), (4000, 1e-5)):
        y = utils.resample_kaiser_best(x, sr0, sr1)
        assert y.dtype == np.float32 and y.shape == (int(np.ceil(sr0 * sr1 / sr0)),)
        ref = np.sin(2 * np.pi * 440 * np.arange(y.size) / sr1)
        assert np.abs(y[200:-200] - ref[200:-200]).max() <= tol, sr1
    x2 = np.stack([x, -0.25 * x])
    y2 = utils.resample_kaiser_best(x2, sr0, 11025)
    assert y2.shape == (2, int(np.ceil(sr0 * 11025 / sr0)))
    assert np.array_equal(y2[0], utils.resample_kaiser_best(x, sr0, 11025))
    y44 = utils.resample_kaiser_best(np.sin(2 * np.pi * 440 * np.arange(44100) / 44100).astype(np.float32), 44100, 16000)
    assert y44.shape == (16000,)
    ref = np.sin(2 * np.pi * 440 * np.arange(16000) / 16000)
    assert np.abs(y44[300:-300] - ref[300:-300]).max() <= 4e-3


@pytest.mark.parametrize('mode,fwd,bwd', [(None, 'k_block_fwd_s', 'k_block_bwd_s16'),
                                          ('0', 'k_block_fwd_s', 'k_block_bwd_s'),
                                          ('1', 'k_block_fwd_s16', 'k_block_bwd_s16'),
                                          ('3', 'k_block_fwd_s16', 'k_block_bwd_s'),
                                          ('7', 'k_block_fwd_s', 'k_block_bwd_s16')])
def test_bench_roofline_names_the_kernels_that_run(monkeypatch, mode, fwd, bwd):
    """bench.py's roofline names the block kernels ASTYLE_MFMA16 selects, as api.hip's
    mfma16_mode reads it (default 2: the backward on 16x16x32; out of range -> the default);
    the roofline arithmetic is the same either way."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    if mode is None:
        monkeypatch.delenv('ASTYLE_MFMA16', raising=False)
    else:
        monkeypatch.setenv('ASTYLE_MFMA16', mode)
    r = bench.block_roofline('split', 256, 16384, 1.57, 1.67, None, 130.0, 33.0)
    assert r['fwd']['kernel'] == fwd and r['bwd']['kernel'] == bwd
    assert r['kernel'] == bwd   # the backward is the longer one
    assert abs(r['bwd']['algorithmic_bytes'] - (3 * 256 * 16384 * 128 * 4 + 32 * 256 * 16384)) < 1
    assert bench.block_roofline('bf16', 256, 16384, 1.0, 1.2, None, 50.0, 20.0)['bwd']['kernel'] == 'k_block_bwd_c'
