"""Test infrastructure: the ASan + UBSan host build of libastyle's C ABI (SURVEY §5 "race
detection / sanitizers") and the fuzz driver tests/san/fuzz_driver.cpp linked against it.

Every source of libastyle.so is compiled as for the product (gfx950 device code included, so
the objects link as they do there), with -fsanitize=address,undefined and no recovery on the
host side only (-Xarch_host; nothing here launches a kernel); ckpt.cpp and the driver with the
same clang; all linked into one executable.  It
runs on the CPU; GPU AddressSanitizer is not available on the MI355X pool, and the device
kernels are checked against the oracle instead."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from audio_style_transfer_amd import _build  # noqa: E402

OUT = os.path.join(ROOT, 'audio_style_transfer_amd', 'build_san')
EXE = os.path.join(OUT, 'fuzz_driver')
SAN = ['-fsanitize=address,undefined', '-fno-sanitize-recover=all', '-fno-omit-frame-pointer']
COMMON = ['-g', '-O1', '-fPIC', '-std=c++17']


def _stale(srcs):
    if not os.path.exists(EXE):
        return True
    t = os.path.getmtime(EXE)
    deps = list(srcs) + [os.path.join(ROOT, 'include', 'astyle.h')]
    deps += [os.path.join(_build.CSRC, f) for f in os.listdir(_build.CSRC)]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False) -> str:
    drv = os.path.join(HERE, 'fuzz_driver.cpp')
    srcs = [os.path.join(_build.CSRC, s) for s in _build.SOURCES] + [drv]
    if not force and not _stale(srcs):
        return EXE
    os.makedirs(OUT, exist_ok=True)

    def cc(src):
        obj = os.path.join(OUT, os.path.basename(src).rsplit('.', 1)[0] + '.o')
        if src.endswith('.hip'):
            flags = ['--offload-arch=gfx950', *COMMON, *[f for x in SAN for f in ('-Xarch_host', x)],
                     *_build.EXTRA.get(os.path.basename(src), [])]
        else:
            flags = ['-x', 'c++', *COMMON, *SAN]
        cmd = [_build.HIPCC, *flags, '-c', src, '-o', obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError('%s failed:\n%s' % (' '.join(cmd), r.stderr))
        return obj

    with ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(cc, srcs))
    cmd = [_build.HIPCC, '--offload-arch=gfx950', *SAN, *objs, '-o', EXE + '.tmp']
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError('link failed:\n' + r.stderr)
    os.replace(EXE + '.tmp', EXE)
    return EXE


if __name__ == '__main__':
    print(build(force='--force' in sys.argv))
