"""Drop-in for the reference's ``output-grams.py`` (output-grams.py:19-123): the channel-wise
("ours") Gram of every consecutive ``length``-sample slice of one wav file, taken over one stack
of 10 encoder blocks (``--stack s``: extracts 10 s .. 10 s + 9) or all 30 (no ``--stack``),
l2-normalised and cut to ``--channels`` channels, one figure per slice (``show_our_gram``) under
``<figdir>/<MMDD>/showAcrosslayer::chan0-127f:<fn>stack<stack>length<length>``.

The Grams come from libastyle's ``ast_embeds`` (the same HIP path as the optimiser's style
taps), one slice per batch row.  Each slice's Gram is also written as ``gram-<i>.npy`` beside its
figure (the figures are skipped when matplotlib is absent, as here).

Usage (as the reference): ``python -m audio_style_transfer_amd.output_grams <name> --srcdir
DIR --figdir DIR [--stack S] [--channels N] [--length T] [--ckpt_path weights.npz]``."""
from __future__ import annotations

import argparse
import os
import warnings

import numpy as np
import torch

from . import utils
from .engine import StyleEngine
from .methods import load_weights
from .weights import synthetic_weights


def stack_layers(lyr_stack):
    """output-grams.py:29-32: one stack of 10 extracts, or all 30."""
    return list(range(lyr_stack * 10, lyr_stack * 10 + 10)) if lyr_stack is not None else list(range(30))


def build_graph(length, lyr_stack=1, nb_channels=128, weights=None, precision='fp32',
                device=None, batch=1):
    """output-grams.py:19-40: the encoder + "ours" style embeds, here one libastyle context."""
    sty = stack_layers(lyr_stack)
    return StyleEngine(batch, length, [sty[-1]], sty, nb_channels=nb_channels, gatys=False,
                       precision=precision, device=device, weights=weights)


def read_file(filename, length, sr=16000):
    """output-grams.py:60-63: consecutive, non-overlapping slices of ``length`` samples."""
    aud, _ = utils.load_audio(filename, sr=sr)
    return [aud[i * length:(i + 1) * length] for i in range(len(aud) // length)]


def get_path(figdir, filename, stack, length):
    """output-grams.py:66-71."""
    path = utils.crt_t_fol(figdir)
    path = os.path.join(path, 'showAcrosslayer::chan0-127f:{}stack{}length{}'.format(filename, stack, length))
    os.makedirs(path, exist_ok=True)
    return path


def get_embeds(engine, aud):
    """output-grams.py:55-58: mu-law encode, ast_embeds -> [channels, L, L] per slice."""
    aud = np.asarray(aud, dtype=np.float64)
    if aud.ndim == 1:
        aud = aud.reshape(1, -1)
    x = torch.tensor(utils.mu_law_numpy(aud), dtype=torch.float32, device=engine.device)
    _, emb_s = engine.embeds(x, content=False, style=True)
    return emb_s.cpu().numpy()


class ShowNet(object):
    """output-grams.py:84-111."""

    def __init__(self, srcdir, ckpt_path, figdir, stack, channels=60, length=16384, sr=16000,
                 weights=None, precision='fp32', device=None):
        assert ckpt_path or weights is not None, 'must provide a ckpt path for this model!'
        if weights is None:
            weights = load_weights(ckpt_path)
            if weights is None:
                warnings.warn('no checkpoint at %r (neither <prefix>.index nor an .npz); '
                              'using seeded synthetic encoder weights' % ckpt_path)
                weights = synthetic_weights(0)
        self.engine = build_graph(length, stack, channels, weights=weights, precision=precision,
                                  device=device)
        self.srcdir = srcdir
        self.ckpt_path = ckpt_path
        self.figdir = figdir
        self.sr = sr
        self.length = length
        self.stack = stack
        self.channels = channels

    def show(self, fn):
        """All slices of <srcdir>/<fn>.wav -> figures + gram-<i>.npy; returns the Grams."""
        filepath = os.path.join(self.srcdir, fn + '.wav')
        audios = read_file(filepath, self.length, self.sr)
        figdir = get_path(self.figdir, fn, self.stack, self.length)
        embeds = [get_embeds(self.engine, aud)[0] for aud in audios]
        for i, e in enumerate(embeds):
            np.save(os.path.join(figdir, 'gram-{}.npy'.format(i)), e)
            utils.show_gram(e, i, figdir)          # show_our_gram (utils.py:223-235)
        return embeds


def make_parser():
    """output-grams.py:113-121 (same options and defaults), + --precision."""
    parser = argparse.ArgumentParser()
    parser.add_argument('filename')
    parser.add_argument('--srcdir', nargs='?', default='./data/src')
    parser.add_argument('--figdir', nargs='?', default='./data/fig')
    parser.add_argument('--stack', nargs='?', default=None, type=int)
    parser.add_argument('--channels', nargs='?', default=128, type=int)
    parser.add_argument('--length', nargs='?', default=16384, type=int)
    parser.add_argument('--ckpt_path', nargs='?', default='./nsynth/model/wavenet-ckpt/model.ckpt-200000')
    parser.add_argument('--precision', default='fp32', choices=('fp32', 'split', 'bf16'))
    return parser


def main(argv=None):
    args = make_parser().parse_args(argv)
    net = ShowNet(args.srcdir, args.ckpt_path, args.figdir, args.stack, args.channels, args.length,
                  precision=args.precision)
    return net.show(args.filename)


if __name__ == '__main__':
    main()
