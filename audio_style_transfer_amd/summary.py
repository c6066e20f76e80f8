"""Per-evaluation scalar log, the reference's ``tf.summary.FileWriter`` (methods.py:127-130,
141,145,156): every loss evaluation writes the four scalars ``loss/content_loss``,
``loss/style_loss``, ``loss/regularizer``, ``loss/main_loss`` as one ``Summary`` at
``global_step = i_ + i`` into ``<logdir>/events.out.tfevents.<time>.<host>``.

TensorFlow is not in the image, so the file is written directly: TFRecord framing (u64 length,
masked CRC-32C of the length, payload, masked CRC-32C of the payload) around hand-encoded
``tensorflow.Event`` protobufs (wall_time = 1 double, step = 2 int64, file_version = 3 string,
summary = 5 {value = 1 {tag = 1 string, simple_value = 2 float}}).  TensorBoard reads it as it
reads the reference's logs.  ``read_events`` parses the same subset back (tests)."""
from __future__ import annotations

import os
import socket
import struct
import time

_POLY = 0x82F63B78          # CRC-32C (Castagnoli), reflected


def _table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ _POLY if c & 1 else c >> 1
        t.append(c)
    return t


_T = _table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _T[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int) -> bytes:
    return _varint((num << 3) | wire)


def _bytes_field(num: int, payload: bytes) -> bytes:
    return _field(num, 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int = 0, file_version: str = None,
                 scalars: dict = None) -> bytes:
    msg = _field(1, 1) + struct.pack('<d', wall_time)
    if step:
        msg += _field(2, 0) + _varint(int(step))
    if file_version is not None:
        msg += _bytes_field(3, file_version.encode())
    if scalars:
        summ = b''
        for tag, v in scalars.items():
            val = _bytes_field(1, tag.encode()) + _field(2, 5) + struct.pack('<f', float(v))
            summ += _bytes_field(1, val)
        msg += _bytes_field(5, summ)
    return msg


def frame(payload: bytes) -> bytes:
    head = struct.pack('<Q', len(payload))
    return head + struct.pack('<I', masked_crc(head)) + payload + struct.pack('<I', masked_crc(payload))


class EventWriter(object):
    """tf.summary.FileWriter(logdir) for scalar summaries; one file per writer."""

    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, 'events.out.tfevents.%010d.%s' % (int(time.time()),
                                                                          socket.gethostname()))
        self._f = open(self.path, 'wb')
        self._f.write(frame(encode_event(time.time(), file_version='brain.Event:2')))
        self._f.flush()

    def add_scalars(self, scalars: dict, global_step: int):
        self._f.write(frame(encode_event(time.time(), global_step, scalars=scalars)))

    def flush(self):
        self._f.flush()

    def close(self):
        if not self._f.closed:
            self._f.close()


# -- reader (the subset above) ----------------------------------------------------------------

def _read_varint(b: bytes, i: int):
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return v, i


def _fields(b: bytes):
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wire = key >> 3, key & 7
        if wire == 0:
            v, i = _read_varint(b, i)
        elif wire == 1:
            v, i = b[i:i + 8], i + 8
        elif wire == 5:
            v, i = b[i:i + 4], i + 4
        elif wire == 2:
            n, i = _read_varint(b, i)
            v, i = b[i:i + n], i + n
        else:
            raise ValueError('unsupported wire type %d' % wire)
        yield num, v


def decode_event(b: bytes) -> dict:
    ev = {'step': 0, 'scalars': {}}
    for num, v in _fields(b):
        if num == 1:
            ev['wall_time'] = struct.unpack('<d', v)[0]
        elif num == 2:
            ev['step'] = v
        elif num == 3:
            ev['file_version'] = v.decode()
        elif num == 5:
            for n2, val in _fields(v):
                if n2 != 1:
                    continue
                tag, x = None, None
                for n3, w in _fields(val):
                    if n3 == 1:
                        tag = w.decode()
                    elif n3 == 2:
                        x = struct.unpack('<f', w)[0]
                ev['scalars'][tag] = x
    return ev


def read_events(path: str):
    """All events of one file; raises on a CRC mismatch."""
    out = []
    with open(path, 'rb') as f:
        data = f.read()
    i = 0
    while i < len(data):
        head = data[i:i + 8]
        if struct.unpack('<I', data[i + 8:i + 12])[0] != masked_crc(head):
            raise ValueError('length CRC mismatch at %d' % i)
        n = struct.unpack('<Q', head)[0]
        payload = data[i + 12:i + 12 + n]
        if struct.unpack('<I', data[i + 12 + n:i + 16 + n])[0] != masked_crc(payload):
            raise ValueError('payload CRC mismatch at %d' % i)
        out.append(decode_event(payload))
        i += 16 + n
    return out
