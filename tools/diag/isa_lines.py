"""Per-source-line VALU / SALU counts of a kernel's main loop (tools/diag/isa_census.py's loop),
from a hipcc -S -gline-tables-only listing: where the loop's vector instructions come from.

usage: python tools/diag/isa_lines.py <file.s> <kernel-name substring> [top N]"""
import collections
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_census as I  # noqa: E402


def main():
    path, pat = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    txt = open(path).read().splitlines()
    files = {}
    for l in txt:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split('/')[-1]
    for k, body in I.kernels(path).items():
        if pat not in k:
            continue
        loop = I.main_loop(body)
        cur, per = None, collections.Counter()
        for l in loop:
            s = l.strip()
            m = re.match(r'\.loc\s+(\d+)\s+(\d+)', s)
            if m:
                cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
                continue
            if not s or s.startswith(('.', ';', '//')) or s.split()[0].endswith(':'):
                continue
            per[(cur, I.classify(s.split()[0]))] += 1
        tot = collections.Counter()
        for (loc, cls), n in per.items():
            if cls in ('valu', 'v_mov'):
                tot[loc] += n
        print(k[-70:], 'loop MFMAs', sum(n for (l, c), n in per.items() if c == 'mfma'),
              'VALU', sum(tot.values()))
        for loc, n in tot.most_common(top):
            print('%5d  %s:%s  salu %d' % (n, loc[0] if loc else '?', loc[1] if loc else '?',
                                           per[(loc, 'salu')]))


if __name__ == '__main__':
    main()
