"""The per-evaluation scalar log (audio_style_transfer_amd/summary.py): TF event files in the
format tf.summary.FileWriter writes (methods.py:141,156), without TensorFlow."""
import struct

import numpy as np

from audio_style_transfer_amd import summary


def test_crc32c_known_answers():
    # RFC 3720 B.4 / the standard CRC-32C check value
    assert summary.crc32c(b'123456789') == 0xE3069283
    assert summary.crc32c(bytes(32)) == 0x8A9136AA
    assert summary.crc32c(bytes([0xFF] * 32)) == 0x62A8AB43
    assert summary.crc32c(bytes(range(32))) == 0x46DD794E


def test_event_encoding_fields():
    b = summary.encode_event(1.5, 7, scalars={'loss/main_loss': 2.0})
    # wall_time: tag 0x09 + double; step: tag 0x10 + varint; summary: tag 0x2a
    assert b[:9] == b'\x09' + struct.pack('<d', 1.5)
    assert b[9:11] == b'\x10\x07' and b[11] == 0x2A
    ev = summary.decode_event(b)
    assert ev['step'] == 7 and ev['scalars'] == {'loss/main_loss': 2.0}
    big = summary.decode_event(summary.encode_event(0.0, 2 ** 40 + 3))
    assert big['step'] == 2 ** 40 + 3


def test_writer_round_trip(tmp_path):
    w = summary.EventWriter(str(tmp_path))
    vals = np.random.default_rng(0).normal(size=(5, 4)).astype(np.float32)
    for i, v in enumerate(vals):
        w.add_scalars({'loss/content_loss': v[1], 'loss/style_loss': v[2],
                       'loss/regularizer': v[3], 'loss/main_loss': v[0]}, i)
    w.close()
    ev = summary.read_events(w.path)
    assert ev[0]['file_version'] == 'brain.Event:2' and len(ev) == 6
    for i, (e, v) in enumerate(zip(ev[1:], vals)):
        assert e['step'] == i
        assert e['scalars']['loss/main_loss'] == v[0] and e['scalars']['loss/regularizer'] == v[3]
    # a flipped payload byte fails the CRC
    raw = bytearray(open(w.path, 'rb').read())
    raw[20] ^= 1
    open(w.path, 'wb').write(bytes(raw))
    try:
        summary.read_events(w.path)
    except ValueError:
        pass
    else:
        raise AssertionError('corruption not detected')
