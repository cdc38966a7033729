"""Instruction-mix summary of one kernel in a hipcc -S output: asm_stats.py file.s kernel_substring"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
m = [mm for mm in re.finditer(r'^(\S+):\s*; @', s, re.M) if pat in mm.group(1)]
name = m[0].group(1)
start = m[0].end()
end = s.index('.Lfunc_end', start)
body = s[start:end]
lines = [l.strip() for l in body.split('\n')]
ins = [l for l in lines if l and not l.startswith(('.', ';')) and not re.match(r'^\S+:', l)]
c = collections.Counter()
for l in ins:
    op = l.split()[0]
    if op.startswith('v_mfma'): k = 'mfma'
    elif op.startswith('ds_'): k = op
    elif op.startswith('v_'): k = 'valu'
    elif op.startswith('s_waitcnt'): k = 's_waitcnt'
    elif op.startswith('s_barrier'): k = 's_barrier'
    elif op.startswith('s_'): k = 'salu'
    else: k = op
    c[k] += 1
print(name, 'instructions:', len(ins))
for k, v in sorted(c.items(), key=lambda x: -x[1]):
    print(f'  {k:28s} {v}')
meta = re.search(r'\.name:\s+' + re.escape(name) + r'.*?(?=\n  - \.|\Z)', s, re.S)
