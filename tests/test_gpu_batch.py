"""The batch CLI's device path (audio_style_transfer_amd/batch.py, --optimizer device) on the GPU:
two pairs optimised together in one context by the device L-BFGS-B must leave each pair's
outputs (ep-0.wav, state.npz) equal to the single-pair GatysNet run with the same optimiser --
the kernels are batch-invariant, so each clip's trajectory does not depend on its neighbour."""
import glob
import os

import numpy as np
import pytest
import torch
from scipy.io import wavfile

pytestmark = pytest.mark.gpu

SR = 16000


def _wavs(d):
    os.makedirs(d, exist_ok=True)
    t = np.arange(2 * SR) / SR
    for k, (name, f) in enumerate((('a', 220.0), ('b', 330.0), ('c', 495.0))):
        a = 0.5 * np.sin(2 * np.pi * f * t) + 0.1 * np.random.default_rng(k).normal(size=t.size)
        wavfile.write(os.path.join(d, name + '.wav'), SR, (np.clip(a, -1, 1) * 32767).astype(np.int16))


def test_batch_device_pairs_equal_single_runs(tmp_path):
    assert torch.cuda.is_available(), 'gpu tests need an MI355X'
    from audio_style_transfer_amd import batch, methods, summary
    src = str(tmp_path / 'src')
    _wavs(src)
    common = ['--batch_size', '4096', '--epochs', '1', '--no_plots', '--stack', '0', '--dir', src]
    args = batch.make_parser().parse_args(['--pairs', 'a:b,c:a', '--outdir', str(tmp_path / 'ob'),
                                           '--logdir', str(tmp_path / 'lb'), *common])
    pairs = batch.read_pairs(args.pairs)
    got = batch.run_rank(args, pairs, 1, 0, torch.device('cuda', 0), log=print)
    for i, (c, s) in enumerate(pairs):
        a1 = methods.make_parser().parse_args([c, s, '--outdir', str(tmp_path / 'o1'),
                                               '--logdir', str(tmp_path / 'l1'), '--optimizer',
                                               'device', *common])
        x1 = methods.piece_work(a1)
        d_b = batch.pair_dirs(args, c, s)[0]
        d_1 = methods.get_dir(a1.outdir, a1)
        assert np.array_equal(wavfile.read(os.path.join(d_b, 'ep-0.wav'))[1],
                              wavfile.read(os.path.join(d_1, 'ep-0.wav'))[1]), (c, s)
        with np.load(os.path.join(d_b, 'state.npz')) as zb, np.load(os.path.join(d_1, 'state.npz')) as z1:
            assert np.array_equal(zb['x'], z1['x']) and int(zb['i_']) == int(z1['i_'])
        # every evaluation's scalars at the same steps (ast_lbfgs_history on both sides)
        fb = glob.glob(os.path.join(batch.pair_dirs(args, c, s)[1], 'events.out.tfevents.*'))
        f1 = glob.glob(os.path.join(methods.get_dir(a1.logdir, a1), 'events.out.tfevents.*'))
        assert len(fb) == 1 and len(f1) == 1
        eb = [(e['step'], sorted(e['scalars'].items())) for e in summary.read_events(fb[0]) if e['scalars']]
        e1 = [(e['step'], sorted(e['scalars'].items())) for e in summary.read_events(f1[0]) if e['scalars']]
        assert eb == e1
        with np.load(os.path.join(d_1, 'state.npz')) as z1:
            assert len(eb) == int(z1['i_']) and [st for st, _ in eb] == list(range(len(eb)))
