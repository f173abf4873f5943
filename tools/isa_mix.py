"""Instruction mix of selected kernels in a gfx950 device assembly file (hipcc -S --offload-device-only).
usage: python tools/isa_mix.py file.s SUBSTRING [SUBSTRING ...]   (substrings of the mangled names)"""
import re
import subprocess
import sys

s = open(sys.argv[1]).read()
names = re.findall(r'^(_Z\w+):', s, re.M)
for n in names:
    if not all(k in n for k in sys.argv[2:]):
        continue
    i = s.index(n + ':')
    j = s.index('.Lfunc_end', i)
    body = s[i:j]
    lines = [l for l in body.split('\n') if l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;')]
    ops = {}
    for l in lines:
        op = l.split()[0]
        ops[op] = ops.get(op, 0) + 1
    dem = subprocess.run(['c++filt', n], capture_output=True, text=True).stdout.strip()
    print(dem[:90], 'instructions:', len(lines))
    for k, v in sorted(ops.items(), key=lambda x: -x[1])[:30]:
        print('   %-28s %d' % (k, v))
