#!/usr/bin/env python3
"""Static VALU / LDS / VMEM counts of the basic blocks of a kernel's busiest
depth-4 loop (the sweep's step loop) in a device .s file.
usage: tools/loop_valu.py <file.s> <mangled kernel name>"""
import collections
import re
import sys


def main():
    txt = open(sys.argv[1]).read()
    m = re.search(re.escape(sys.argv[2]) + r":[^\n]*\n(.*?)\.Lfunc_end", txt, re.S)
    lines = m.group(1).split('\n')
    hdrs = collections.Counter(mm.group(1) for l in lines for mm in [re.search(r'Header=(BB\d+_\d+) Depth=4', l)] if mm)
    top = hdrs.most_common(1)[0][0]
    cur, blocks = None, collections.OrderedDict()
    for l in lines:
        s = l.strip()
        mm = re.match(r'^\.L(BB\d+_\d+):\s*;?\s*(.*)', s)
        if mm:
            cur = mm.group(1)
            blocks[cur] = (mm.group(2), [])
            continue
        if cur:
            blocks[cur][1].append(s)
    tot = collections.Counter()
    for lab, (h, b) in blocks.items():
        if f'Header={top} Depth=4' in h or lab == top:
            c = collections.Counter()
            for s in b:
                if s.startswith('v_'):
                    c['valu'] += 1
                elif s.startswith('ds_'):
                    c['lds'] += 1
                elif s.startswith(('buffer_', 'global_')):
                    c['vmem'] += 1
                elif s.startswith('s_') and not s.startswith('s_waitcnt'):
                    c['salu'] += 1
            if c['valu']:
                print(lab, dict(c))
            tot.update(c)
    print('loop', top, dict(tot))


if __name__ == '__main__':
    main()
