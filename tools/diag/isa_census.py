"""Instruction census of a kernel's main loop (the back-edge region holding the most MFMAs) from a
hipcc -S listing: counts per instruction class, for pricing VALU / LDS / MFMA changes per tile.

usage: python tools/diag/isa_census.py <file.s> <kernel-name substring> [...]"""
import collections
import re
import sys


def classify(m):
    if m.startswith('v_mfma'):
        return 'mfma'
    if m.startswith('v_accvgpr'):
        return 'accvgpr'
    if m.startswith(('v_mov', 'v_pk_mov')):
        return 'v_mov'
    if m.startswith('v_'):
        return 'valu'
    if m.startswith(('ds_read', 'ds_load')):
        return 'ds_read'
    if m.startswith(('ds_write', 'ds_store')):
        return 'ds_write'
    if m.startswith('ds_'):
        return 'ds_other'
    if m.startswith('s_waitcnt'):
        return 'waitcnt'
    if m.startswith('s_nop'):
        return 's_nop'
    if m.startswith(('s_barrier',)):
        return 'barrier'
    if m.startswith('s_'):
        return 'salu'
    if m.startswith(('buffer_load', 'global_load')):
        return 'vmem_load'
    if m.startswith(('buffer_store', 'global_store', 'global_atomic', 'buffer_atomic')):
        return 'vmem_store'
    return 'other'


def kernels(path):
    txt = open(path).read().splitlines()
    out, name, body = {}, None, []
    for l in txt:
        m = re.match(r'^(_Z\S+):', l)
        if m:
            name, body = m.group(1), []
            continue
        if name and l.startswith('.Lfunc_end'):
            out[name] = body
            name = None
            continue
        if name:
            body.append(l)
    return out


def main_loop(body):
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r'^(\.LBB\S+):', l)
        if m:
            labels[m.group(1)] = i
    best = None
    for i, l in enumerate(body):
        m = re.search(r'\bs_cbranch_\w+\s+(\.LBB\S+)', l) or re.search(r'\bs_branch\s+(\.LBB\S+)', l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            seg = body[labels[m.group(1)]:i + 1]
            n = sum(1 for s in seg if 'v_mfma' in s)
            if best is None or n > best[0]:
                best = (n, seg)
    return best[1] if best else body


def census(lines):
    c = collections.Counter()
    for l in lines:
        l = l.strip()
        if not l or l.startswith(('.', ';', '//')) or l.split()[0].endswith(':'):
            continue
        c[classify(l.split()[0])] += 1
    return c


if __name__ == '__main__':
    ks = kernels(sys.argv[1])
    for pat in sys.argv[2:]:
        for k, body in ks.items():
            if pat in k:
                c = census(main_loop(body))
                print(k[-60:], dict(sorted(c.items())))
