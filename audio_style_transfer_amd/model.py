"""Drop-in for the reference's model.py ``cfg`` (encoder half), running on libastyle.so.

``cfg().build({'quantized_wav': x}, is_training)`` runs the 30-block non-causal WaveNet
encoder (model.py:79-127) on the GPU and fills ``cfg.extracts`` with the 32 tapped tensors
(extracts[0..29] = block outputs, extracts[30] = extracts[29], extracts[31] = bottleneck), as
float32 torch tensors [B, T, C] on the device.  The returned dict carries 'quantized_input',
'before_enc' (= extracts[30]) and 'encoding' (the 512-hop average-pooled bottleneck,
model.py:128).  The WaveNet decoder (model.py:133-194) is not built: no fetch on the style
transfer path depends on it.
"""
from __future__ import annotations

import numpy as np
import torch

from .engine import StyleEngine
from .weights import synthetic_weights


class cfg(object):
    def __init__(self, train_path=None, weights=None, precision='fp32', device=None):
        self.ae_hop_length = 512                    # model.py:22
        self.ae_bottleneck_width = 16               # model.py:23
        self.train_path = train_path
        self.extracts = []
        self.weights = weights if weights is not None else synthetic_weights(0)
        self.precision = precision
        self.device = device
        self._engine = None

    def build(self, quantized_inputs, is_training=True):
        del is_training
        x = quantized_inputs['quantized_wav']
        x = torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x, dtype=torch.float32)
        if x.dim() == 1:
            x = x[None]
        dev = self.device or torch.device('cuda', torch.cuda.current_device())
        x = x.to(dev).contiguous()
        B, T = x.shape
        if self._engine is None or (self._engine.batch, self._engine.T) != (B, T):
            # a new (B, T) needs a context of its own: the old one's device workspace (76 GB at
            # B = 256) is released now, not whenever the garbage collector gets to it (extracts
            # are copies, so nothing the caller holds points into it)
            self.close()
            # taps 29 (content) + 31 (bottleneck) and style 0 + 30 make every block run
            self._engine = StyleEngine(B, T, [29, 31], [0, 30], cnt_channels=16,
                                       precision=self.precision, device=dev, weights=self.weights)
        self._engine.forward(x)
        self.extracts = [self._engine.extract(i) for i in range(32)]
        bott = self.extracts[31]
        enc = torch.nn.functional.avg_pool1d(bott.transpose(1, 2), self.ae_hop_length,
                                             self.ae_hop_length).transpose(1, 2)
        return {'quantized_input': x, 'encoding': enc, 'before_enc': self.extracts[30]}

    def close(self):
        """Destroy the library context (its device workspace); build() makes a new one."""
        if self._engine is not None:
            self._engine.close()
            self._engine = None
