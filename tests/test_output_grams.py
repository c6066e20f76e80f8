"""output-grams.py drop-in (audio_style_transfer_amd/output_grams.py): CLI contract and paths on
the CPU; per-slice Grams against the oracle on the GPU (output-grams.py:19-111)."""
import os

import numpy as np
import pytest

from oracle import astyle_oracle as O
from audio_style_transfer_amd.weights import synthetic_clips


def test_cli_defaults_match_reference():
    from audio_style_transfer_amd.output_grams import make_parser
    a = make_parser().parse_args(['song'])
    assert (a.filename, a.srcdir, a.figdir, a.stack, a.channels, a.length, a.ckpt_path) == (
        'song', './data/src', './data/fig', None, 128, 16384,
        './nsynth/model/wavenet-ckpt/model.ckpt-200000')
    a = make_parser().parse_args(['x', '--stack', '2', '--channels', '60', '--length', '4096'])
    assert (a.stack, a.channels, a.length) == (2, 60, 4096)


def test_paths_and_slices(tmp_path):
    from scipy.io import wavfile
    from audio_style_transfer_amd import output_grams as G, utils
    p = G.get_path(str(tmp_path), 'song', 1, 4096)
    assert os.path.isdir(p)
    assert os.path.basename(p) == 'showAcrosslayer::chan0-127f:songstack1length4096'
    assert os.path.dirname(p) == utils.crt_t_fol(str(tmp_path))
    assert G.stack_layers(None) == list(range(30)) and G.stack_layers(2) == list(range(20, 30))
    sig = synthetic_clips(1, 3 * 4096 + 100, 3)[0]
    wavfile.write(str(tmp_path / 's.wav'), 16000, (sig * 32767).astype(np.int16))
    sl = G.read_file(str(tmp_path / 's.wav'), 4096)
    assert len(sl) == 3 and all(s.shape == (4096,) for s in sl)


@pytest.mark.gpu
def test_show_matches_oracle(tmp_path, weights):
    import torch
    from scipy.io import wavfile
    from audio_style_transfer_amd import utils
    from audio_style_transfer_amd.output_grams import ShowNet
    assert torch.cuda.is_available(), 'gpu tests need an MI355X'
    T = 4096
    sig = synthetic_clips(1, 3 * T, 11)[0]
    src = tmp_path / 'src'
    src.mkdir()
    wavfile.write(str(src / 'song.wav'), 16000, (sig * 32767).astype(np.int16))
    net = ShowNet(str(src), None, str(tmp_path / 'fig'), 1, channels=64, length=T, weights=weights)
    embeds = net.show('song')
    aud, _ = utils.load_audio(str(src / 'song.wav'), sr=16000)
    assert len(embeds) == 3
    for i, e in enumerate(embeds):
        ext, _ = O.encoder_forward(O.mu_law_numpy(aud[i * T:(i + 1) * T]), weights, 20)
        ref = O.style_embeds(ext, list(range(10, 20)), False, 64)
        assert e.shape == ref.shape == (64, 10, 10)
        err = float(np.linalg.norm(e - ref) / np.linalg.norm(ref))
        assert err <= 1e-5, (i, err)
        saved = np.load(os.path.join(net_fig(tmp_path), 'gram-%d.npy' % i))
        assert np.array_equal(saved, e)


def net_fig(tmp_path):
    from audio_style_transfer_amd import utils
    return os.path.join(utils.crt_t_fol(str(tmp_path / 'fig')),
                        'showAcrosslayer::chan0-127f:songstack1length4096')
