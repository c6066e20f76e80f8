"""Build libastyle.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the
repo snapshot to the GPU box)."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, 'csrc')
LIB = os.path.join(PKG, 'libastyle.so')
SOURCES = ['encoder.hip', 'block_fwd_bf16.hip', 'block_bwd_bf16.hip', 'block_fwd_split.hip',
           'block_bwd_split.hip', 'block_fwd_split16.hip', 'block_bwd_split16.hip', 'gram.hip', 'gram_bf16.hip', 'gram_split.hip', 'gram_gatys.hip',
           'stft_reg.hip', 'lbfgs.hip', 'ot_admm.hip', 'api.hip', 'ckpt.cpp']
# tools-only A/B builds (ASTYLE_VARIANT=<name> [ASTYLE_DEFS=...] -> libastyle_<name>.so) may add
# sources from tools/variants here; round 6 retired the round-3/4 alternative forward kernels
# (role split, double-buffered image, Winograd timing probes: written for the 32x32x16 fragment
# layout, measured slower)
VARIANTS = os.path.join(os.path.dirname(PKG), 'tools', 'variants')
VARIANT_SOURCES = {}
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
CXX = os.environ.get('CXX', 'g++')          # host-only sources (.cpp)
CXXFLAGS = ['-O2', '-fPIC', '-std=c++17', '-Wall']
FLAGS = ['--offload-arch=gfx950', '-O3', '-fPIC', '-std=c++17', '-Wall',
         '-Wno-unused-function', '-munsafe-fp-atomics']
# per-source extras: the column-owning block kernels keep their weights in AGPRs and need the
# MFMA accumulators in arch VGPRs, where the epilogues read them without copies; their fully
# unrolled tile loops exceed the default pragma-unroll size limit (a partly unrolled loop would
# index the register-resident weight arrays dynamically and demote them to scratch)
_CW = ['-mllvm', '-amdgpu-mfma-vgpr-form=1', '-mllvm', '-amdgpu-atomic-optimizer-strategy=None', '-mllvm', '-pragma-unroll-threshold=1000000', '-fno-slp-vectorize']
if os.environ.get('ASTYLE_NO_VGPR_FORM'):   # A/B builds: let the compiler place MFMA accumulators (AGPRs)
    _CW = _CW[2:]
EXTRA = {'block_fwd_bf16.hip': _CW, 'block_bwd_bf16.hip': _CW, 'block_fwd_split.hip': _CW,
         'block_bwd_split.hip': _CW, 'block_fwd_split16.hip': _CW, 'block_bwd_split16.hip': _CW}


def _stale(lib: str = LIB, extra=()) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + list(extra)
    deps.append(os.path.join(os.path.dirname(PKG), 'include', 'astyle.h'))
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > t for d in deps)


def build_variant(name: str, force: bool = False) -> str:
    """The tools-only A/B library libastyle_<name>.so of VARIANT_SOURCES[name], rebuilt from the
    committed sources whenever they changed."""
    lib = os.path.join(PKG, 'libastyle_%s.so' % name)
    extra = [os.path.join(VARIANTS, f) for f in VARIANT_SOURCES.get(name, ([], []))[0]]
    if not force and not _stale(lib, extra):
        return lib
    # built from VARIANT_SOURCES' own defines only: an ASTYLE_DEFS of the caller's environment
    # (e.g. a diagnostic define) must not leak into it
    old = {k: os.environ.get(k) for k in ('ASTYLE_VARIANT', 'ASTYLE_DEFS')}
    os.environ['ASTYLE_VARIANT'] = name
    os.environ.pop('ASTYLE_DEFS', None)
    try:
        return build(force=True)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def build(force: bool = False, verbose: bool = False, stamps: bool = False) -> str:
    """The shipped libastyle.so; stamps=True: the phase-stamp diagnostic build
    (libastyle_stamps.so, tools/stamps.py).  ASTYLE_VARIANT=<name> (+ ASTYLE_DEFS): an A/B build
    libastyle_<name>.so, with the tools/variants sources of VARIANT_SOURCES[name] if any."""
    lib = LIB if not stamps else os.path.join(PKG, 'libastyle_stamps.so')
    variant = os.environ.get('ASTYLE_VARIANT', '')   # A/B builds: libastyle_<variant>.so
    defs = os.environ.get('ASTYLE_DEFS', '').split()
    sources = list(SOURCES)
    if variant:
        lib = os.path.join(PKG, 'libastyle_%s.so' % variant)
        extra_src, extra_defs = VARIANT_SOURCES.get(variant, ([], []))
        sources += [os.path.join(VARIANTS, f) for f in extra_src]
        defs += extra_defs
    if not force and not stamps and not variant and not _stale():
        return LIB
    objdir = os.path.join(PKG, 'build_' + variant if variant else 'build' if not stamps else 'build_stamps')
    flags = FLAGS + (['-DASTYLE_STAMPS'] if stamps else []) + defs
    os.makedirs(objdir, exist_ok=True)

    def cc(src):
        name = os.path.basename(src)
        obj = os.path.join(objdir, name.rsplit('.', 1)[0] + '.o')
        path = src if os.path.isabs(src) else os.path.join(CSRC, src)
        if src.endswith('.cpp'):
            cmd = [CXX, *CXXFLAGS, '-c', path, '-o', obj]
        else:
            cmd = [HIPCC, *flags, '-I', CSRC, *EXTRA.get(name, []), '-c', path, '-o', obj]
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('%s failed for %s:\n%s' % (cmd[0], src, r.stderr))
        if r.stderr and verbose:
            print(r.stderr, file=sys.stderr)
        return obj

    with ThreadPoolExecutor(len(sources)) as ex:
        objs = list(ex.map(cc, sources))
    tmp = lib + '.tmp'
    cmd = [HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', *objs, '-o', tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('link failed:\n' + r.stderr)
    os.replace(tmp, lib)
    return lib


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True, stamps='--stamps' in sys.argv))
