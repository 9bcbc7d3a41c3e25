"""Per-basic-block instruction counts of one kernel in the saved gfx950 assembly.
usage: python3 tools/asm_blocks.py <file.s> <kernel-name-substring> [out.s]"""
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r'^(\S*' + re.escape(sys.argv[2]) + r'\S*):', s, re.M)
i = m.start()
j = s.index('.Lfunc_end', i)
body = s[i:j].split('\n')
if len(sys.argv) > 3:
    open(sys.argv[3], 'w').write('\n'.join(body))
blocks = []
cur = None
for ln in body:
    if re.match(r'^\.LBB\S+:', ln) or cur is None:
        cur = [ln.split(':')[0][:24], 0, 0, 0, 0, 0, ''];
        blocks.append(cur)
        continue
    t = ln.strip()
    if not t or t.startswith(';') or t.startswith('.'):
        continue
    cur[1] += 1
    op = t.split()[0]
    if op.startswith('v_'): cur[2] += 1
    if op.startswith('ds_'): cur[3] += 1
    if op.startswith('s_'): cur[4] += 1
    if op.startswith(('global_', 'buffer_')): cur[5] += 1
    if op.startswith('s_cbranch') or op == 's_branch': cur[6] += ' ' + t.split()[-1]
print('%-24s %5s %5s %4s %4s %4s  branches' % ('block', 'all', 'valu', 'ds', 'salu', 'vmem'))
for b in blocks:
    print('%-24s %5d %5d %4d %4d %4d %s' % tuple(b))
