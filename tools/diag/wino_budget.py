"""Compiled register budget of a Winograd F(2,3) dilated conv in the split block kernels
(build it or close it with compiled-ISA evidence).

Winograd F(2,3) for the K = 3 dilated conv (forward GEMM 1 / backward GEMM 2) needs, per wave,
four transformed weight matrices (G0 = W0, G1 = (W0+W1+W2)/2, G2 = (W0-W1+W2)/2, G3 = W2) as
split-fp16 A fragments instead of three taps: +64 registers; the shipped kernels already hold
W_d's three taps and W_r (256 registers) in the 256 AGPRs, so one matrix moves to the
architectural VGPRs.  And four m accumulators over the tile's 32 output pairs instead of two
column halves: +32 VGPRs.  So the kernels need 96 more VGPRs live across the tile loop.

This script compiles the shipped kernels twice for gfx950 with the shipped flags: as they are,
and with 96 extra VGPRs (24 uint4 loaded before the loop, kept live to its end) -- the
Winograd kernels' register footprint without their (extra) code -- and prints VGPRs, AGPRs,
spills and LDS per kernel instance.  Nothing here runs on a GPU.

usage: python tools/diag/wino_budget.py [out.txt]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, 'audio_style_transfer_amd', 'csrc')
sys.path.insert(0, ROOT)
from audio_style_transfer_amd import _build  # noqa: E402

EXTRA_IN = '''
    // (wino_budget.py) the Winograd footprint: the 4th transformed matrix (64) + two more m
    // accumulators (32) = 96 VGPRs live across the tile loop
    uint4 wino_x[24];
#pragma unroll
    for (int q = 0; q < 24; ++q) wino_x[q] = reinterpret_cast<const uint4*>(a.WSRC)[q * 64 + lane];
'''
EXTRA_OUT = '''
#pragma unroll
    for (int q = 0; q < 24; ++q)
        asm volatile("" :: "v"(wino_x[q].x), "v"(wino_x[q].y), "v"(wino_x[q].z), "v"(wino_x[q].w));
'''


def compile_res(path):
    flags = _build.FLAGS + ['-I', CSRC] + _build.EXTRA['block_fwd_split.hip']
    r = subprocess.run([_build.HIPCC, *flags, '--cuda-device-only', '-S', path, '-o', os.devnull,
                        '-Rpass-analysis=kernel-resource-usage'], capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-3000:])
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r'remark: +(.*?): (.*?) \[-Rpass', line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == 'Function Name':
            name = subprocess.run(['c++filt', v], capture_output=True, text=True).stdout.strip()
            cur = {'name': re.sub(r'ast::\(anonymous namespace\)::', '', name).split('(')[0]}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    return [r for r in rows if 'k_block' in r['name']]


def main():
    out = []
    with tempfile.TemporaryDirectory() as d:
        for f, wsrc in (('block_fwd_split.hip', 'wdf'), ('block_bwd_split.hip', 'wdb')):
            src = open(os.path.join(CSRC, f)).read()
            assert src.count('    pin_all(wd, wr);\n') == 1 and src.count('    STAMP_FLUSH(a.stamps)\n') == 1
            probe = src.replace('    pin_all(wd, wr);\n', '    pin_all(wd, wr);\n' + EXTRA_IN.replace('WSRC', wsrc))
            probe = probe.replace('    STAMP_FLUSH(a.stamps)\n', EXTRA_OUT + '    STAMP_FLUSH(a.stamps)\n')
            pa, pb = os.path.join(d, f), os.path.join(d, 'wino_' + f)
            open(pa, 'w').write(src)
            open(pb, 'w').write(probe)
            base = compile_res(pa)
            wino = compile_res(pb)
            for a, b in zip(base, wino):
                assert a['name'] == b['name']
                out.append('%-52s shipped: VGPR %3s AGPR %3s spill %s | +96 live VGPRs: VGPR %3s AGPR %3s '
                           'VGPR spill %4s  (LDS %s B)' % (
                               a['name'], a.get('VGPRs'), a.get('AGPRs'), a.get('VGPRs Spill'),
                               b.get('VGPRs'), b.get('AGPRs'), b.get('VGPRs Spill'),
                               a.get('LDS Size [bytes/block]')))
    text = '\n'.join(out) + '\n'
    print(text, end='')
    if len(sys.argv) > 1:
        with open(sys.argv[1], 'w') as fh:
            fh.write('# tools/diag/wino_budget.py: the shipped split block kernels as compiled (gfx950, shipped '
                     'flags) and with the\n# Winograd F(2,3) register footprint added (+96 VGPRs live across '
                     'the tile loop: 4th transformed matrix + 2 more m accumulators)\n' + text)


if __name__ == '__main__':
    main()
