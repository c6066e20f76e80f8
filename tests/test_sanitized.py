"""CPU: the ASan + UBSan host build of the C ABI (tests/san/build.py; SURVEY §5 sanitizers)
driven with hostile inputs (tests/san/fuzz_driver.cpp):

* the TF checkpoint-V2 reader (ckpt.cpp, what Saver.restore reads for methods.py:79-84) on
  every truncation of a written bundle's .index and data shard, a few thousand seeded bit
  flips (raw, and with the hit block's CRC recomputed so the flip reaches the parser), and
  footers whose block handles point far past the file (offset + size wrapping 2^64);
* ast_workspace_bytes (ast_create's validation and sizing) on seeded random configurations.

Each case must end in 0 or an AST_E_* code with no sanitizer report (the build aborts on the
first one)."""
import os
import random
import shutil
import subprocess

import numpy as np
import pytest

from tf_ckpt_writer import write_checkpoint, retrailer
from audio_style_transfer_amd.summary import _varint

ENV = dict(os.environ, ASAN_OPTIONS='detect_leaks=0:halt_on_error=1:abort_on_error=0',
           UBSAN_OPTIONS='halt_on_error=1:print_stacktrace=1')


@pytest.fixture(scope='module')
def driver():
    import san.build as SB
    return SB.build()


def _tensors():
    r = np.random.default_rng(1)
    return {'ae_res_1/W': r.normal(size=(1, 1, 4, 4)).astype(np.float32),
            'ae_res_1/biases': r.normal(size=(4,)).astype(np.float32),
            'ae_startconv/W': r.normal(size=(1, 3, 1, 5)).astype(np.float32),
            'global_step': np.array(7, dtype=np.int64),
            'x_double': r.normal(size=(3, 2)),
            'x_half': r.normal(size=(5,)).astype(np.float16),
            'x_scalar': np.array(1.5, dtype=np.float32)}


def _run(driver, tmp, prefixes):
    lst = os.path.join(tmp, 'list.txt')
    with open(lst, 'w') as f:
        f.write('\n'.join(prefixes) + '\n')
    r = subprocess.run([driver, 'ckpt', lst], capture_output=True, text=True, env=ENV, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert 'ERROR: AddressSanitizer' not in r.stderr and 'runtime error' not in r.stderr, r.stderr[-4000:]
    rows = [tuple(int(v) for v in ln.split()) for ln in r.stdout.splitlines()]
    assert len(rows) == len(prefixes)
    return rows


def _variant(tmp, k, index, data):
    pre = os.path.join(tmp, 'v%05d' % k)
    with open(pre + '.index', 'wb') as f:
        f.write(bytes(index))
    with open(pre + '.data-00000-of-00001', 'wb') as f:
        f.write(bytes(data))
    return pre


def test_checkpoint_fuzz(driver, tmp_path):
    tmp = str(tmp_path)
    base = os.path.join(tmp, 'base')
    blocks = write_checkpoint(base, _tensors(), block_size=64, restart=2)
    index = bytearray(open(base + '.index', 'rb').read())
    data = bytearray(open(base + '.data-00000-of-00001', 'rb').read())
    (ok,) = _run(driver, tmp, [base])
    assert ok == (0, 6, 1)                         # six float tensors read, global_step refused
    crc_covered = set()      # data and index blocks (the metaindex block is never read)
    for off, size in blocks[:-2] + blocks[-1:]:
        crc_covered.update(range(off, off + size + 5))
    cases, expect_fail = [], []
    # every truncation of the index (the data shard intact), then of the data shard
    for n in range(len(index)):
        cases.append(_variant(tmp, len(cases), index[:n], data))
        expect_fail.append('open')
    for n in range(len(data)):
        cases.append(_variant(tmp, len(cases), index, data[:n]))
        expect_fail.append('read')
    rng = random.Random(1234)
    # raw bit flips anywhere in the index: inside a CRC-covered block they must be refused
    for _ in range(1500):
        i = rng.randrange(len(index))
        v = bytearray(index)
        v[i] ^= 1 << rng.randrange(8)
        cases.append(_variant(tmp, len(cases), v, data))
        expect_fail.append('open' if i in crc_covered else None)
    # structure-aware flips: 1-3 bits of one block, its CRC recomputed (reaches the parser)
    for _ in range(1500):
        off, size = blocks[rng.randrange(len(blocks))]
        if not size:
            continue
        v = bytearray(index)
        for _ in range(rng.randint(1, 3)):
            v[off + rng.randrange(size)] ^= 1 << rng.randrange(8)
        retrailer(v, off, size)
        cases.append(_variant(tmp, len(cases), v, data))
        expect_fail.append(None)
    # data-shard flips (caught by the tensors' CRC-32C; global_step, an int64, is never read)
    t = _tensors()
    offs = np.cumsum([0] + [t[n].nbytes for n in sorted(t)])
    gs = sorted(t).index('global_step')
    for _ in range(300):
        v = bytearray(data)
        i = rng.randrange(len(v))
        v[i] ^= 1 << rng.randrange(8)
        cases.append(_variant(tmp, len(cases), index, v))
        expect_fail.append(None if offs[gs] <= i < offs[gs + 1] else 'read')
    # footers whose handles point past the end, offset + size + 5 wrapping 2^64
    foot0 = len(index) - 48
    for mo, ms, io, isz in [(0, 0, 2 ** 64 - 3, 2), (2 ** 64 - 1, 1, 0, 4), (0, 2 ** 63, 0, 2 ** 63),
                            (len(index), 0, 2 ** 62, 2 ** 62), (0, 0, 0, 2 ** 64 - 1)]:
        f = _varint(mo) + _varint(ms) + _varint(io) + _varint(isz)
        v = bytearray(index)
        v[foot0:foot0 + 40] = (f + bytes(40))[:40]
        cases.append(_variant(tmp, len(cases), v, data))
        expect_fail.append('open')
    rows = _run(driver, tmp, cases)
    nfail_open = 0
    for (rc, nread, nbad), exp, pre in zip(rows, expect_fail, cases):
        assert rc in (0, -1, -4), (pre, rc)
        if exp == 'open':
            assert rc != 0, pre
        if exp == 'read' and rc == 0:
            assert nread < 6, pre
        nfail_open += rc != 0
    print('%d checkpoint variants, %d refused at open' % (len(cases), nfail_open))
    shutil.rmtree(tmp, ignore_errors=True)


def test_workspace_config_fuzz(driver):
    r = subprocess.run([driver, 'cfg', '7', '4000'], capture_output=True, text=True, env=ENV,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert 'runtime error' not in r.stderr and 'AddressSanitizer' not in r.stderr
    rcs = [int(ln.split()[0]) for ln in r.stdout.splitlines()]
    assert len(rcs) == 4000 and set(rcs) <= {0, -1} and rcs.count(0) > 100
