"""MI355X-native audio style transfer (drop-in for winlp4ever/audio_style_transfer's
methods.py / model.py hot path).  The compute path is libastyle.so (hand-written HIP for
gfx950) behind a C ABI (include/astyle.h)."""
from .weights import synthetic_weights, synthetic_clips, weight_shapes  # noqa: F401

__all__ = ['synthetic_weights', 'synthetic_clips', 'weight_shapes']
