"""Encoder weights: TF variable names, shapes, and the seeded synthetic generator.

The reference restores ``model.ckpt-200000`` (methods.py:79-84) — absent offline.
Every run here uses seeded synthetic weights with the reference's initialiser
(``tf.uniform_unit_scaling_initializer(1.0)``, masked.py:116: U(+-sqrt(3 / prod(shape[:-1])))).
Biases are zero-initialised in the reference (masked.py:117); the generator gives them a
small non-zero value so the bias path is exercised.  Names/shapes follow masked.py:136-145
(HWIO ``[1, K, Cin, Cout]``) so a real checkpoint's tensors drop in by name.
"""
from __future__ import annotations

import numpy as np

C = 128
N_BLOCKS = 30
BOTTLENECK = 16


def weight_shapes():
    """Ordered {tf_name: shape} for the encoder (model.py:88-127)."""
    shapes = {'ae_startconv/W': (1, 3, 1, C), 'ae_startconv/biases': (C,)}
    for l in range(1, N_BLOCKS + 1):
        shapes['ae_dilatedconv_%d/W' % l] = (1, 3, C, C)
        shapes['ae_dilatedconv_%d/biases' % l] = (C,)
        shapes['ae_res_%d/W' % l] = (1, 1, C, C)
        shapes['ae_res_%d/biases' % l] = (C,)
    shapes['ae_bottleneck/W'] = (1, 1, C, BOTTLENECK)
    shapes['ae_bottleneck/biases'] = (BOTTLENECK,)
    return shapes


def synthetic_weights(seed: int = 0, bias_scale: float = 0.05):
    """Deterministic (PCG64) weights, float32, keyed by TF variable name."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, shape in weight_shapes().items():
        if name.endswith('/W'):
            fan_in = int(np.prod(shape[:-1]))
            lim = np.sqrt(3.0 / fan_in)
            out[name] = rng.uniform(-lim, lim, size=shape).astype(np.float32)
        else:
            out[name] = rng.uniform(-bias_scale, bias_scale, size=shape).astype(np.float32)
    return out


def synthetic_clips(n: int, T: int, seed0: int, sr: int = 16000):
    """Seeded test audio: per clip a mixture of 3 sinusoids (80-2000 Hz)
    plus 0.05*N(0,1), peak-normalised to 0.9; float32 in [-1, 1]."""
    out = np.empty((n, T), dtype=np.float32)
    t = np.arange(T) / sr
    for b in range(n):
        rng = np.random.default_rng(seed0 + b)
        f = rng.uniform(80, 2000, size=3)
        ph = rng.uniform(0, 2 * np.pi, size=3)
        a = rng.uniform(0.2, 1.0, size=3)
        s = (a[:, None] * np.sin(2 * np.pi * f[:, None] * t[None, :] + ph[:, None])).sum(0)
        s = s + 0.05 * rng.standard_normal(T)
        out[b] = 0.9 * s / np.max(np.abs(s))
    return out


STRESS_KINDS = ('dr4', 'dr025', 'alt2', 'student_t', 'bias100')


def stressed_weights(kind: str, seed: int = 0):
    """Weight sets whose statistics differ from uniform_unit_scaling, for range tests of the
    split-fp16 mode (per-block weight exponents, analytic operand bounds; splitwave.h):
      dr4        every block's W_d x 4, W_r x 0.25 (u 4x wider, per-block exponents shift)
      dr025      W_d x 0.25, W_r x 4
      alt2       blocks alternately x 2 / x 0.5 (both W): max |e| grows to ~3e5 by block 30
      student_t  heavy-tailed W ~ Student-t(3) at the same variance (max |W| ~ 9, not 1)
      bias100    biases x 100 (activations ~1e3)"""
    import re
    W = synthetic_weights(seed)
    if kind == 'student_t':
        rng = np.random.Generator(np.random.PCG64(seed + 7))
        out = {}
        for name, v in W.items():
            if name.endswith('/W'):
                fan_in = int(np.prod(v.shape[:-1]))
                t = rng.standard_t(3, size=v.shape) / np.sqrt(3.0)      # unit variance
                out[name] = (t * np.sqrt(1.0 / fan_in)).astype(np.float32)
            else:
                out[name] = v
        return out
    out = {}
    for name, v in W.items():
        m = re.match(r'ae_(dilatedconv|res)_(\d+)/W$', name)
        f = 1.0
        if kind == 'bias100':
            f = 100.0 if name.endswith('/biases') else 1.0
        elif m:
            conv, l = m.group(1) == 'dilatedconv', int(m.group(2))
            f = {'dr4': 4.0 if conv else 0.25, 'dr025': 0.25 if conv else 4.0,
                 'alt2': 2.0 if l % 2 == 0 else 0.5}[kind]
        elif kind not in STRESS_KINDS:
            raise ValueError('unknown stress kind %r' % kind)
        out[name] = (v * np.float32(f)).astype(np.float32)
    return out
