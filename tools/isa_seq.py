#!/usr/bin/env python3
"""Event sequence of the full-tile path of a k_contig kernel: L global load,
S global store, W s_waitcnt vmcnt, B branch, vN a run of N VALU ops; starting
at the first run of >= 2U loads (the unrolled tile's loads).

usage: isa_seq.py file.s SUBSTRING [U]"""
import re
import sys

sys.path.insert(0, __import__('os').path.dirname(__file__))
import isa_loop as I  # noqa: E402


def seq(body, U=4):
    ev = []
    for l in body:
        s = l.strip()
        if 'global_load_dwordx4' in s:
            ev.append('L')
        elif 'global_store_dwordx4' in s:
            ev.append('S')
        elif s.startswith('s_cbranch') or s.startswith('s_branch'):
            ev.append('B')
        elif s.startswith('s_waitcnt') and 'vmcnt' in s:
            ev.append('W')
        elif s.startswith('v_') and not s.startswith('v_lshl_add_u64'):
            ev.append('v')
    txt = ''.join(ev)
    # the tile: first window holding 2U loads before U stores
    for start in range(len(txt)):
        if txt[start] != 'L':
            continue
        w = txt[start:]
        if w[:80].count('L') >= 2 * U - 2:
            end = start
            st = 0
            while end < len(txt) and st < U:
                st += txt[end] == 'S'
                end += 1
            return re.sub(r'v+', lambda m: 'v%d' % len(m.group(0)), txt[start:end])
    return None


if __name__ == '__main__':
    path, sub = sys.argv[1], sys.argv[2]
    U = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    ks = list(I.kernels(path))
    for (m, body), dn in zip(ks, I.demangle([k for k, _ in ks])):
        if sub in dn and 'k_contig<' in dn:
            print(dn.split('(')[0].replace('mpix::', ''))
            print('   ', seq(body, U))
