#!/usr/bin/env python3
"""Static instruction mix of one kernel in a device .s file (hipcc
--cuda-device-only -S): totals and the largest basic blocks (the brick loops).
usage: tools/isa_stats.py <file.s> <mangled kernel name> [n_blocks]"""
import collections
import re
import sys


def classify(block):
    c = collections.Counter()
    for l in block:
        s = l.strip()
        if not s or s.startswith(('.', ';', '//')) or s.split()[0].endswith(':'):
            continue
        i = s.split()[0]
        c['total'] += 1
        if i.startswith('v_mov'): c['v_mov'] += 1
        if i.startswith('v_cndmask'): c['v_cndmask'] += 1
        if i.startswith('v_'): c['valu'] += 1
        if i.startswith('s_') and not i.startswith('s_waitcnt'): c['salu'] += 1
        if i.startswith('ds_'): c['ds'] += 1
        if i.startswith(('buffer_', 'global_')): c['vmem'] += 1
        if i.startswith('s_waitcnt'): c['waitcnt'] += 1
        if 'dpp' in s: c['dpp'] += 1
        if i.startswith('v_sqrt'): c['sqrt'] += 1
    return dict(c)


def main():
    txt = open(sys.argv[1]).read()
    name = sys.argv[2]
    m = re.search(re.escape(name) + r":[^\n]*\n(.*?)\.Lfunc_end", txt, re.S)
    lines = m.group(1).split('\n')
    print('whole', classify(lines))
    bbs, cur, lab = [], [], 'entry'
    for l in lines:
        s = l.strip()
        if re.match(r'^\.LBB\d+_\d+:', s):
            bbs.append((lab, cur))
            cur, lab = [], s.split(':')[0]
        else:
            cur.append(l)
    bbs.append((lab, cur))
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    for lab, b in sorted(bbs, key=lambda b: -len(b[1]))[:nb]:
        print(lab, classify(b))


if __name__ == '__main__':
    main()
