"""Instruction mix per basic block of one kernel in a hipcc -S listing (register / spill forensics).

    python tools/isa_blocks.py <file.s> <kernel-name-substring>
"""
import collections
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    s = open(path).read()
    m = re.search(r'^(_Z\w*' + re.escape(name) + r'\w*):', s, re.M)
    body = s[m.end():]
    body = body[:body.index('.Lfunc_end')]
    blocks, cur, label = [], [], 'entry'
    for line in body.split('\n'):
        t = line.strip()
        if re.match(r'^\.LBB\d+_\d+:', t):
            blocks.append((label + (' ' + t.split(';', 1)[1].strip() if ';' in t else ''), cur))
            label, cur = t.split(':')[0], []
        elif t and not t.startswith(';') and not t.startswith('.'):
            cur.append(t)
    blocks.append((label, cur))
    tot = collections.Counter()
    for lab, b in blocks:
        c = collections.Counter()
        for t in b:
            op = t.split()[0]
            k = ('mfma' if op.startswith('v_mfma') else 'valu' if op.startswith('v_') else 'ds' if op.startswith('ds_')
                 else 'vmem' if op.startswith(('buffer_', 'global_')) else 'bar' if op.startswith('s_barrier')
                 else 'spill_st' if op.startswith('scratch_store') else 'spill_ld' if op.startswith('scratch_load')
                 else 'salu' if op.startswith('s_') else 'other')
            c[k] += 1
        tot += c
        print(f"{lab[:60]:60s} {len(b):5d} {dict(c)}")
    print('total', dict(tot))


if __name__ == '__main__':
    main()
