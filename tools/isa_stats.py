#!/usr/bin/env python3
"""Per-kernel ISA statistics from build/obj/kernels.s (make -C quadiron_amd/csrc asm):
VGPR/SGPR counts, spills, and static instruction mix.
    python tools/isa_stats.py [substring ...]"""
import re
import sys
from collections import Counter

import os
s = open(os.environ.get('QI_ASM', os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'build', 'obj', 'kernels.s'))).read()
pats = sys.argv[1:] or ['encode_fnt_kernelILi16ELi2ELb1ELb1E', 'matrix_kernelILi8ELi4ELb1E']
meta = {}
for m in re.finditer(r'\.name:\s+(\S+)\n', s):
    pass
for m in re.finditer(r'- \.agpr_count:(.*?)\.name:\s+(\S+)(.*?)\.vgpr_spill_count:\s+(\d+)', s, re.S):
    body = m.group(1) + m.group(3)
    g = lambda k: re.search(r'\.' + k + r':\s+(\d+)', body)
    meta[m.group(2)] = {k: int(g(k).group(1)) for k in ('vgpr_count', 'sgpr_count') if g(k)}
    meta[m.group(2)]['vspill'] = int(m.group(4))
for m in re.finditer(r'^(_ZN2qi\S+):[^\n]*\n(.*?)^\.Lfunc_end', s, re.M | re.S):
    name, body = m.group(1), m.group(2)
    if not any(p in name for p in pats):
        continue
    ins = []
    for l in body.split('\n'):
        t = l.strip()
        if not t or t[0] in '.;_' or t.endswith(':'):
            continue
        ins.append(t.split()[0])
    c = Counter(ins)
    v = sum(n for k, n in c.items() if k.startswith('v_'))
    print(name[:70], meta.get(name, {}), 'total', len(ins), 'valu', v,
          'st', sum(n for k, n in c.items() if 'store' in k),
          'ld', sum(n for k, n in c.items() if 'buffer_load' in k or 'global_load' in k),
          'mul24', c['v_mul_i32_i24_e32'] + c['v_mul_i32_i24_e64'],
          'sdwa', sum(n for k, n in c.items() if k.endswith('_sdwa')))
