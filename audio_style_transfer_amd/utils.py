"""Host-side helpers of the drop-in (restates the path-relevant parts of the reference's
utils.py): mu-law codecs, output-directory naming, audio I/O without librosa, Gram plots.

The reference's ``load_audio`` uses librosa (absent here); ``load_audio`` below reads WAV with
scipy and resamples with ``scipy.signal.resample_poly`` (librosa's default 'kaiser_best'
resampler is not available, so resampled audio differs slightly; WAVs already at ``sr`` are
bit-identical to librosa's float conversion for PCM16/float files).
"""
from __future__ import annotations

import os
import time
from math import gcd

import numpy as np

ins = ['bass', 'brass', 'flute', 'guitar', 'keyboard', 'mallet', 'organ', 'reed', 'string',
       'synth_lead', 'vocal']

abbrevs = {'length': 'l', 'layers': 'lyr', 'n_components': 'cpn', 'examples': 'ex',
           'epochs': 'ep', 'qualities': 'qult', 'lambd': 'lbd', 'batch_size': 'btch',
           'stack': 'stk'}


def gt_s_path(suppath, **kwargs):
    """Output directory named from the CLI args (utils.py:18-64); created if missing."""
    parts = ''
    for name, value in sorted(kwargs.items()):
        if name == 'ins' and value is not None:
            assert len(value) == 2
            parts += '{}2{}_'.format(ins[value[0]], ins[value[1]])
        elif name == 'male2female':
            assert value <= 2
            parts += {0: 'f2m_', 1: 'm2f_'}.get(value, '')
        elif name == 'filename':
            parts = value + '_' + parts
        elif name == 'cont_fn':
            parts += '_cnt_{}_'.format(value)
        elif name == 'style_fn':
            parts += '_style_{}_'.format(value)
        elif name == 'gatys':
            parts = ('gatys_' if value else 'ours_') + parts
        elif name == 'sr':
            parts += '_sr{}kHz_'.format(value / 1000)
        elif not name.endswith(('dir', 'path', 'pieces')) and value is not None:
            key = abbrevs.get(name, name)
            if isinstance(value, (list, tuple)):
                value = ''.join('-%d' % i for i in value)
            parts += '_{}_{}_'.format(key, value)
    path = os.path.join(suppath, parts)
    os.makedirs(path, exist_ok=True)
    return path


def crt_t_fol(suppath, hour=False):
    """Dated sub-folder (utils.py:67-76): '<month><day>' (or + hour, minute)."""
    dte = time.localtime()
    if hour:
        fol = os.path.join(suppath, '{}{}{}{}'.format(dte[1], dte[2], dte[3], dte[4]))
    else:
        fol = os.path.join(suppath, '{}{}'.format(dte[1], dte[2]))
    os.makedirs(fol, exist_ok=True)
    return fol


def mu_law_numpy(x, mu=255):
    """utils.py:79-82: floor(128 * sign(x) ln(1 + mu|x|) / ln(1 + mu))."""
    x = np.asarray(x)
    out = np.sign(x) * np.log(1 + mu * np.abs(x)) / np.log(1 + mu)
    return np.floor(out * 128)


def inv_mu_law_numpy(x, mu=255.0):
    """utils.py:85-90 (the +0.5 offset; x == 0 passes through as 0)."""
    x = np.array(x).astype(np.float32)
    out = (x + 0.5) * 2. / (mu + 1)
    out = np.sign(out) / mu * ((1 + mu) ** np.abs(out) - 1)
    return np.where(np.equal(x, 0), x, out)


def _to_float(a):
    if a.dtype == np.int16:
        return a.astype(np.float32) / 32768.0
    if a.dtype == np.int32:
        return a.astype(np.float32) / 2147483648.0
    if a.dtype == np.uint8:
        return (a.astype(np.float32) - 128.0) / 128.0
    return a.astype(np.float32)


def load_audio(fn, sr, audio_channel=0):
    """utils.py:260-265 semantics: float32 in [-1, 1] at ``sr``; multi-channel files return
    channel ``audio_channel`` (librosa.load(mono=False) layout [channels, samples])."""
    from scipy.io import wavfile
    from scipy.signal import resample_poly
    fsr, a = wavfile.read(fn)
    a = _to_float(a)
    a = a.T if a.ndim > 1 else a
    if sr is not None and fsr != sr:
        g = gcd(int(sr), int(fsr))
        a = resample_poly(a, int(sr) // g, int(fsr) // g, axis=-1).astype(np.float32)
        fsr = sr
    if a.ndim > 1:
        return a[audio_channel], fsr
    return a, fsr


def write_wav(path, audio, sr):
    """librosa.output.write_wav equivalent (float32 WAV)."""
    from scipy.io import wavfile
    wavfile.write(path, int(sr), np.asarray(audio, dtype=np.float32))


def show_gram(mats, ep=None, figdir=None, gatys=False):
    """Per-epoch Gram figure (utils.py:223-257); skipped silently without matplotlib."""
    try:
        import matplotlib
        matplotlib.use('agg')
        import matplotlib.pyplot as plt
    except Exception:
        return
    mats = np.asarray(mats)
    cols = 2 if gatys else 8
    n = mats.shape[0] // cols
    if n == 0:
        return
    fig, axs = plt.subplots(cols, n, figsize=(3 * n, 3 * cols), squeeze=False)
    for i in range(cols):
        for j in range(n):
            axs[i, j].imshow(mats[i + j * cols], interpolation='nearest', cmap=plt.cm.plasma)
            axs[i, j].set_title('channel {}'.format(i + cols * j))
    name = 'gram-ep{}.png'.format(ep) if ep is not None else 'gram-style.png'
    fig.savefig(os.path.join(figdir, name), dpi=5 if not gatys else 20)
    plt.close(fig)
