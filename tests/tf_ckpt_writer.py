"""Test infrastructure: writes a TensorFlow checkpoint-V2 bundle (the format tf.train.Saver
writes and methods.py:79-84 restores) from numpy arrays, independently of the native reader
under test (csrc/ckpt.cpp).  No TensorFlow here, and no NSynth checkpoint to read: the reader's
parity against real TF files is unpinned; these files follow the published format:

  <prefix>.index: LevelDB table — data blocks of (shared, non_shared, value_len, key delta,
      value) entries with a restart array every `restart` entries, each block followed by a
      type byte (0 = uncompressed) and the masked CRC-32C of block + type; an empty metaindex
      block; an index block mapping a key >= each data block's last key to its BlockHandle
      (varint offset, size); a 48-byte footer (metaindex and index handles, zero padding to 40
      bytes, magic 0xdb4775248b80fb57 little-endian).
  keys: "" -> BundleHeaderProto {num_shards = 1, endianness = 2, version = 3 {producer = 1}};
      each variable name -> BundleEntryProto {dtype = 1, shape = 2 {dim = 2 {size = 1}},
      shard_id = 3, offset = 4, size = 5, crc32c = 6 (fixed32, masked)}.
  <prefix>.data-%05d-of-%05d: the raw little-endian tensor bytes."""
import struct

import numpy as np

from audio_style_transfer_amd.summary import crc32c, masked_crc, _varint, _field, _bytes_field

DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3,
      np.dtype(np.int64): 9, np.dtype(np.float16): 19}


def _crc_ext(data, init):
    # crc32c continuing from a previous value (summary.crc32c starts fresh)
    from audio_style_transfer_amd.summary import _T
    c = init ^ 0xFFFFFFFF
    for b in data:
        c = _T[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _block(entries, restart):
    out, restarts, last = bytearray(), [], b''
    for i, (k, v) in enumerate(entries):
        if i % restart == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(k), len(last)) and k[shared] == last[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(k) - shared) + _varint(len(v)) + k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack('<I', r)
    out += struct.pack('<I', len(restarts))
    return bytes(out)


def _with_trailer(block, btype=0):
    c = _crc_ext(bytes([btype]), crc32c(block))
    m = (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF
    return block + bytes([btype]) + struct.pack('<I', m)


def entry_proto(dtype, shape, shard, offset, size, crc):
    dims = b''.join(_bytes_field(2, _field(1, 0) + _varint(int(d))) for d in shape)
    msg = _field(1, 0) + _varint(dtype) + _bytes_field(2, dims)
    if shard:
        msg += _field(3, 0) + _varint(shard)
    if offset:
        msg += _field(4, 0) + _varint(offset)
    msg += _field(5, 0) + _varint(size) + _field(6, 5) + struct.pack('<I', crc)
    return msg


def write_checkpoint(prefix, tensors, num_shards=1, block_size=4096, restart=16,
                     corrupt=None):
    """tensors: {name: ndarray}.  Tensors are spread over shards round-robin in name order.
    Returns the .index layout: [(offset, size)] of every table block (without its 5-byte
    trailer), data blocks first, then the metaindex and the index block."""
    names = sorted(tensors)
    shards = [bytearray() for _ in range(num_shards)]
    kv = [(b'', _field(1, 0) + _varint(num_shards) + _bytes_field(3, _field(1, 0) + _varint(1)))]
    for i, n in enumerate(names):
        a = np.require(tensors[n], requirements='C')
        raw = a.astype(a.dtype.newbyteorder('<'), copy=False).tobytes()
        s = i % num_shards
        off = len(shards[s])
        shards[s] += raw
        kv.append((n.encode(), entry_proto(DT[a.dtype], a.shape, s, off, len(raw), masked_crc(raw))))
    for s in range(num_shards):
        data = bytes(shards[s])
        if corrupt == 'data' and s == 0 and data:
            data = bytes([data[0] ^ 1]) + data[1:]
        with open('%s.data-%05d-of-%05d' % (prefix, s, num_shards), 'wb') as f:
            f.write(data)
    # table: data blocks, metaindex, index, footer
    out = bytearray()
    index = []
    cur = []
    size = 0

    blocks = []

    def flush():
        nonlocal cur, size
        if not cur:
            return
        blk = _block(cur, restart)
        index.append((cur[-1][0], len(out), len(blk)))
        blocks.append((len(out), len(blk)))
        out.extend(_with_trailer(blk))
        cur, size = [], 0
    for k, v in kv:
        cur.append((k, v))
        size += len(k) + len(v) + 3
        if size >= block_size:
            flush()
    flush()
    meta = _block([], restart)
    meta_h = (len(out), len(meta))
    blocks.append(meta_h)
    out.extend(_with_trailer(meta))
    iblk = _block([(k, _varint(o) + _varint(n)) for k, o, n in index], 1)
    index_h = (len(out), len(iblk))
    blocks.append(index_h)
    out.extend(_with_trailer(iblk))
    foot = _varint(meta_h[0]) + _varint(meta_h[1]) + _varint(index_h[0]) + _varint(index_h[1])
    foot = foot + bytes(40 - len(foot))
    magic = 0xdb4775248b80fb57
    if corrupt == 'magic':
        magic ^= 1
    foot += struct.pack('<II', magic & 0xFFFFFFFF, magic >> 32)
    out.extend(foot)
    if corrupt == 'index':
        out[5] ^= 0x40
    with open(prefix + '.index', 'wb') as f:
        f.write(bytes(out))
    return blocks


def retrailer(index: bytearray, off: int, size: int) -> None:
    """Recompute the masked CRC-32C trailer of the block at [off, off + size) in place (its type
    byte included), so a mutated block passes the CRC check and reaches the parser."""
    index[off + size + 1:off + size + 5] = _with_trailer(bytes(index[off:off + size]),
                                                          index[off + size])[-4:]
