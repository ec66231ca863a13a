#!/usr/bin/env python3
"""Instruction mix of the full-tile path of k_contig kernels, from a device
assembly file (hipcc --cuda-device-only -S).  For every kernel whose
demangled name matches the pattern: number of VALU ops, the position of every
global load/store in the unrolled full-tile block (the block holding U loads
of each operand and U stores), and how many loads are issued before the first
VALU op that consumes loaded data (s_waitcnt vmcnt).

usage: isa_loop.py file.s PATTERN [PATTERN ...]
"""
import re
import subprocess
import sys


def kernels(path):
    cur, name = None, None
    for line in open(path):
        m = re.match(r'^(_Z\S+):', line)
        if m:
            cur, name = [], m.group(1)
            continue
        if cur is not None:
            cur.append(line.rstrip('\n'))
            if 's_endpgm' in line:
                yield name, cur
                cur = None


def demangle(names):
    out = subprocess.run(['c++filt'], input='\n'.join(names), capture_output=True, text=True).stdout
    return out.splitlines()


def blocks(body):
    b, cur = [], []
    for l in body:
        if re.match(r'^\.LBB\d+_\d+:', l) or l.startswith('; %bb.'):
            if cur:
                b.append(cur)
            cur = [l]
        else:
            cur.append(l)
    if cur:
        b.append(cur)
    return b


def analyse(body):
    best = None
    for blk in blocks(body):
        nl = sum('global_load_dwordx4' in l for l in blk)
        ns = sum('global_store_dwordx4' in l for l in blk)
        if ns >= 2 and (best is None or nl + ns > best[0]):
            best = (nl + ns, blk)
    if best is None:
        return None
    blk = best[1]
    ins = [l.strip() for l in blk if l.startswith('\t') and not l.strip().startswith(';')]
    valu = [i for i in ins if i.startswith('v_') and not i.startswith('v_lshl_add_u64')]
    loads_before = 0
    for i in ins:
        if i.startswith('s_waitcnt') and 'vmcnt' in i:
            break
        loads_before += 'global_load' in i
    return dict(loads=sum('global_load' in i for i in ins),
                stores=sum('global_store' in i for i in ins), valu=len(valu),
                loads_before_first_wait=loads_before, instructions=len(ins))


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    ks = list(kernels(path))
    names = demangle([k for k, _ in ks])
    for (mangled, body), dn in zip(ks, names):
        if 'k_contig<' not in dn or not any(re.search(p, dn) for p in pats):
            continue
        r = analyse(body)
        short = dn.split('(')[0].replace('mpix::', '')
        print(short, r)


if __name__ == '__main__':
    main()
