"""Host-side helpers of the drop-in (restates the path-relevant parts of the reference's
utils.py): mu-law codecs, output-directory naming, audio I/O without librosa, Gram plots.

The reference's ``load_audio`` is ``librosa.load(fn, sr=sr, mono=False)`` (utils.py:260-265),
which resamples with librosa's default ``res_type='kaiser_best'`` = resampy's band-limited sinc
interpolation (resampy.resample + librosa's fix_length to ceil(n * ratio)).  Neither librosa nor
resampy is in this image, so ``resample_kaiser_best`` below restates resampy 0.2's published
algorithm (filters.sinc_window with the kaiser_best parameters, interpn.resample_f's loop order
and float32 accumulation) -- parity unpinned: no reference output exists here to check it
against.  WAVs already at ``sr`` are bit-identical to librosa's float conversion for
PCM16/float files.
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


# resampy's 'kaiser_best' filter (resampy/filters.py: sinc_window(num_zeros=64, precision=9,
# window=kaiser(beta=14.769656459379492), rolloff=0.9475937167399596))
_KB = dict(num_zeros=64, precision=9, beta=14.769656459379492, rolloff=0.9475937167399596)
_KB_WIN = None


def _kaiser_best_window():
    """resampy.filters.sinc_window: the right wing of a Kaiser-tapered sinc, 2^precision table
    entries per zero crossing."""
    global _KB_WIN
    if _KB_WIN is None:
        from scipy.signal.windows import kaiser
        num_bits = 2 ** _KB['precision']
        n = num_bits * _KB['num_zeros']
        r = _KB['rolloff']
        sinc_win = r * np.sinc(r * np.linspace(0, _KB['num_zeros'], num=n + 1, endpoint=True))
        taper = kaiser(2 * n + 1, _KB['beta'])[n:]
        _KB_WIN = (taper * sinc_win, num_bits)
    return _KB_WIN


def resample_kaiser_best(y, sr_orig, sr_new):
    """librosa.resample(y, sr_orig, sr_new, res_type='kaiser_best', fix=True, scale=False):
    resampy.resample (interpn.resample_f: per output sample, the left then the right wing of the
    interpolated filter, each product added into the float32 output) along the last axis, then
    fix_length to ceil(n * ratio) (zero padding or truncation)."""
    y = np.asarray(y, dtype=np.float32)
    if sr_orig == sr_new:
        return y
    ratio = float(sr_new) / sr_orig
    win, num_table = _kaiser_best_window()
    if ratio < 1:
        win = win * ratio
    delta = np.zeros_like(win)
    delta[:-1] = np.diff(win)
    n_orig = y.shape[-1]
    n_out = int(n_orig * ratio)
    if n_out < 1:
        raise ValueError('input too short to resample')
    scale = min(1.0, ratio)
    index_step = int(scale * num_table)
    nwin = win.shape[0]
    # time_register: the sequential float64 sum of resample_f (np.cumsum adds in order)
    tr = np.concatenate([[0.0], np.cumsum(np.full(n_out - 1, 1.0 / ratio))]) if n_out > 1 else np.zeros(1)
    n = tr.astype(np.int64)
    x2 = y.reshape(-1, n_orig)
    out = np.zeros((x2.shape[0], n_out), np.float32)

    def wing(frac, count, sign):
        index_frac = frac * num_table
        offset = index_frac.astype(np.int64)
        eta = index_frac - offset
        kmax = int(count.max()) if count.size else 0
        for i in range(kmax):
            m = i < count
            idx = np.where(m, offset + i * index_step, 0)
            w = np.where(m, win[idx] + eta * delta[idx], 0.0)
            src = np.clip(n - i if sign < 0 else n + i + 1, 0, n_orig - 1)
            out[:] = (out.astype(np.float64) + w * x2[:, src]).astype(np.float32)

    frac = scale * (tr - n)
    wing(frac, np.minimum(n + 1, (nwin - (frac * num_table).astype(np.int64)) // index_step), -1)
    frac = scale - frac
    wing(frac, np.minimum(n_orig - n - 1, (nwin - (frac * num_table).astype(np.int64)) // index_step), +1)
    n_fix = int(np.ceil(n_orig * ratio))
    if n_fix > n_out:
        out = np.concatenate([out, np.zeros((out.shape[0], n_fix - n_out), np.float32)], 1)
    out = out[:, :n_fix]
    return out.reshape(y.shape[:-1] + (n_fix,))


def load_audio(fn, sr, audio_channel=0, res_type='kaiser_best'):
    """utils.py:260-265 semantics: float32 in [-1, 1] at ``sr``; multi-channel files return
    channel ``audio_channel`` (librosa.load(mono=False) layout [channels, samples]).
    res_type 'kaiser_best' (librosa's default, resample_kaiser_best) or 'polyphase'
    (scipy.signal.resample_poly, the round-1..3 behaviour)."""
    from scipy.io import wavfile
    fsr, a = wavfile.read(fn)
    a = _to_float(a)
    a = a.T if a.ndim > 1 else a
    if sr is not None and fsr != sr:
        if res_type == 'kaiser_best':
            a = resample_kaiser_best(a, int(fsr), int(sr))
        else:
            from scipy.signal import resample_poly
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
