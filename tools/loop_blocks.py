#!/usr/bin/env python3
"""Per-basic-block instruction counts of the innermost loop that contains the
largest basic block of a kernel (the brick step loop of the sweep kernel).
usage: tools/loop_blocks.py <file.s> <mangled kernel name> [--all]"""
import re
import sys


def main():
    txt = open(sys.argv[1]).read()
    name = sys.argv[2]
    m = re.search(re.escape(name) + r":[^\n]*\n(.*?)\.Lfunc_end", txt, re.S)
    lines = m.group(1).split('\n')
    bbs, cur, lab, start = [], [], 'entry', 0
    for i, l in enumerate(lines):
        s = l.strip()
        mm = re.match(r'^(\.LBB\d+_\d+):', s) or re.match(r'^; %bb\.(\d+):', s)
        if mm:
            bbs.append((lab, start, cur))
            cur, lab, start = [], mm.group(1), i
        else:
            cur.append(s)
    bbs.append((lab, start, cur))
    big = max(range(len(bbs)), key=lambda k: sum(1 for s in bbs[k][2] if s.startswith('v_')))
    # header: nearest preceding block labelled as a loop header; back edge: branch to it
    hdr = None
    for k in range(big, -1, -1):
        if any('Loop Header' in s for s in bbs[k][2]) and bbs[k][0].startswith('.LBB'):
            if any(('s_branch ' + bbs[k][0]) == s or s.endswith(' ' + bbs[k][0]) for b in bbs[big:] for s in b[2]):
                hdr = k
                break
    end = max(k for k in range(len(bbs)) if any(s.endswith(' ' + bbs[hdr][0]) for s in bbs[k][2]))
    tot = 0
    for lab, st, b in bbs[hdr:end + 1]:
        v = sum(1 for s in b if s.startswith('v_'))
        sa = sum(1 for s in b if s.startswith('s_') and not s.startswith('s_waitcnt'))
        ds = sum(1 for s in b if s.startswith('ds_'))
        vm = sum(1 for s in b if s.startswith(('buffer_', 'global_', 'scratch_')))
        mv = sum(1 for s in b if s.startswith('v_mov'))
        br = ' '.join(s for s in b if s.startswith(('s_cbranch', 's_branch')))
        tot += v
        if v or '--all' in sys.argv:
            print(f"{lab:12s} v={v:4d} mov={mv:3d} s={sa:3d} ds={ds:2d} vm={vm} {br[:60]}")
    print('loop total VALU', tot)


if __name__ == '__main__':
    main()
