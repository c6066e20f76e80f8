"""Instruction mix of a kernel's hot loop from hipcc -S output (diagnostic).

usage: python tools/isa_mix.py file.s [kernel-substring]
For every kernel in the file (or those whose symbol contains the substring): the counts of
MFMA / VALU / DS / VMEM / SALU / waitcnt instructions in the largest loop (the span between a
label and the last backward branch to it), and in the whole kernel.
"""
import collections
import re
import sys


def classify(op):
    if op.startswith('v_mfma'):
        return 'mfma'
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('ds_'):
        return 'ds'
    if op.startswith(('global_', 'buffer_', 'flat_')):
        return 'vmem'
    if op.startswith('s_waitcnt'):
        return 'waitcnt'
    if op.startswith(('s_barrier', 's_setprio', 's_nop', 's_sleep')):
        return op
    if op.startswith('s_'):
        return 'salu'
    return 'other'


def main():
    src = open(sys.argv[1]).read()
    want = sys.argv[2] if len(sys.argv) > 2 else ''
    parts = re.split(r'\n(_Z\S+):[^\n]*\n', src)
    for i in range(1, len(parts), 2):
        name, body = parts[i], parts[i + 1]
        if want not in name:
            continue
        lines = [l.split(';')[0].strip() for l in body.split('\n')]
        lines = [l for l in lines if l and not l.startswith('.') or re.match(r'^\.LBB\S+:', l)]
        pos = {}
        best = None
        for j, l in enumerate(lines):
            m = re.match(r'^(\.LBB\S+):', l)
            if m:
                pos[m.group(1)] = j
                continue
            m = re.match(r'^s_(cbranch_\w+|branch)\s+(\.LBB\S+)', l)
            if m and m.group(2) in pos and pos[m.group(2)] < j:
                span = (pos[m.group(2)], j)
                if best is None or span[1] - span[0] > best[1] - best[0]:
                    best = span
        def count(a, b):
            c = collections.Counter()
            for l in lines[a:b + 1]:
                if l.startswith('.'):
                    continue
                c[classify(l.split()[0])] += 1
            return dict(sorted(c.items()))
        print(name[:90])
        print('  kernel:', count(0, len(lines) - 1))
        if best:
            print('  loop  :', count(*best))


if __name__ == '__main__':
    main()
