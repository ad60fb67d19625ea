"""Instruction-class counts of a kernel's ISA, per basic block (hipcc --save-temps .s file).

usage: python tools/isa_stats.py FILE.s NAME_SUBSTRING [--min-mfma N]
Prints each basic block with at least N MFMAs (default 1): MFMAs, VALU (with transcendental and
packed-f32 counts), LDS reads / writes, vector memory loads / stores, waitcnts, barriers, and the VALU
issue cycles per MFMA (MI355X_MICROARCH.md issue costs: 4 cycles a VALU op, 8 a transcendental) --
the number that says whether the fillers fit the 24 free issue cycles of a 32x32x16 MFMA gap."""
import collections
import re
import sys


def blocks(lines):
    cur, name = [], 'entry'
    for ln in lines:
        m = re.match(r'^(\.LBB\S+|\S+):', ln)
        if m and not ln.startswith('\t'):
            if cur:
                yield name, cur
            cur, name = [], m.group(1)
            continue
        t = ln.strip()
        if ln.startswith('\t') and t and not t.startswith(';') and not t.startswith('.'):
            cur.append(t)
    if cur:
        yield name, cur


def classify(op):
    if op.startswith('v_mfma'):
        return 'mfma'
    if op.startswith('scratch_'):
        return 'scratch'
    if op.startswith('ds_read') or op.startswith('ds_load'):
        return 'ds_read'
    if op.startswith('ds_write') or op.startswith('ds_store'):
        return 'ds_write'
    if re.match(r'(buffer|global)_load', op):
        return 'vmem_ld'
    if re.match(r'(buffer|global)_store', op):
        return 'vmem_st'
    if re.match(r'v_(exp|rcp|log|rsq|sqrt|sin|cos)_', op):
        return 'trans'
    if op.startswith('v_pk_'):
        return 'valu_pk'
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('s_waitcnt'):
        return 'waitcnt'
    if op.startswith('s_barrier'):
        return 'barrier'
    if op.startswith('s_'):
        return 'salu'
    return 'other'


def main():
    path, name = sys.argv[1], sys.argv[2]
    min_mfma = int(sys.argv[sys.argv.index('--min-mfma') + 1]) if '--min-mfma' in sys.argv else 1
    lines = open(path).read().split('\n')
    start = next(i for i, ln in enumerate(lines) if re.match(r'^_Z\S*:', ln) and name in ln.split(':')[0])
    end = next(j for j in range(start, len(lines)) if lines[j].startswith('.Lfunc_end'))
    print(lines[start].split(':')[0])
    tot = collections.Counter()
    for bname, body in blocks(lines[start + 1:end]):
        c = collections.Counter(classify(t.split()[0]) for t in body)
        tot.update(c)
        if c['mfma'] >= min_mfma:
            issue = 4 * (c['valu'] + c['valu_pk']) + 8 * c['trans']
            print(f'{bname:>12}: {len(body):5d} instr  mfma {c["mfma"]:4d}  valu {c["valu"]:4d} (+pk {c["valu_pk"]}, '
                  f'trans {c["trans"]})  ds_rd {c["ds_read"]:3d}  ds_wr {c["ds_write"]:3d}  vmem_ld {c["vmem_ld"]:3d}  '
                  f'vmem_st {c["vmem_st"]:3d}  scr {c["scratch"]:3d}  wait {c["waitcnt"]:3d}  bar {c["barrier"]}  salu {c["salu"]:3d}  '
                  f'valu issue cyc/mfma {issue / max(c["mfma"], 1):.1f}')
    print('total', dict(tot))


if __name__ == '__main__':
    main()
