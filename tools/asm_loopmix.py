"""Instruction mix of a kernel's largest basic blocks (the K loop) from hipcc --cuda-device-only -S output.
usage: asm_loopmix.py FILE.s SYMBOL_SUBSTRING [SYMBOL_SUBSTRING ...]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
for pat in sys.argv[2:]:
    m = re.search(r'^(\S*' + re.escape(pat) + r'\S*):\s*;', s, re.M)
    if not m:
        print("no symbol", pat)
        continue
    start = m.end()
    end = s.index('.Lfunc_end', start)
    lines = [ln.strip() for ln in s[start:end].split('\n')]
    lines = [ln for ln in lines if ln and (re.match(r'^\.LBB\w+:', ln) or not ln.startswith(('.', ';', '//')))]
    blocks, cur, lab = [], [], 'entry'
    for ln in lines:
        if re.match(r'^[.\w$]+:', ln):
            blocks.append((lab, cur))
            cur, lab = [], ln.split()[0]
        else:
            cur.append(ln)
    blocks.append((lab, cur))
    print(m.group(1)[:90], 'instructions', len(lines))
    for lab, ins in sorted(blocks, key=lambda x: -len(x[1]))[:2]:
        c = collections.Counter()
        for ln in ins:
            op = ln.split()[0]
            key = ('mfma' if op.startswith('v_mfma') else 'ds_read' if op.startswith(('ds_read', 'ds_load'))
                   else 'ds_write' if op.startswith(('ds_write', 'ds_store')) else
                   'vmem_load' if op.startswith(('global_load', 'buffer_load')) else 'waitcnt' if op.startswith('s_waitcnt')
                   else 'valu' if op.startswith('v_') else 'salu' if op.startswith('s_') else op)
            c[key] += 1
        print('   ', lab, len(ins), dict(c))
