"""Per-basic-block instruction census of one kernel in a hipcc -S listing.

usage: python tools/isa_blocks.py k.s <kernel-symbol-substring> [min_instrs]
Prints, for each block with at least min_instrs instructions, its size, VALU
count and the counts of a few instructions worth watching (SGPR spill
traffic, selects, LDS and global memory operations).
"""
import sys
from collections import Counter

src, pat = sys.argv[1], sys.argv[2]
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 100
s = open(src).read()
name_at = None
for line in s.split('\n'):
    line = line.split(';')[0].strip()
    if line.endswith(':') and pat in line and not line.startswith('.'):
        name_at = line[:-1]
        break
i = s.index(name_at + ':')
j = s.index('.Lfunc_end', i)
blocks, cur, label = [], [], 'entry'
for line in s[i:j].split('\n'):
    head = line.split(';')[0].rstrip()
    if head and not line.startswith(('\t', ' ', ';')) and head.endswith(':'):
        blocks.append((label, cur))
        label, cur = head[:-1], []
    elif line.startswith('\t') and not line.strip().startswith(('.', ';')):
        cur.append(line.strip().split()[0])
blocks.append((label, cur))
watch = ['scratch_load_dword', 'scratch_store_dword', 'scratch_load_dwordx2', 'scratch_store_dwordx2', 'v_readlane_b32', 'v_writelane_b32', 'v_cndmask_b32_e64', 'v_cndmask_b32_e32', 'ds_read_b128',
         'global_load_dwordx4', 'global_store_dwordx4', 'v_pk_maximum3_f16', 'v_perm_b32', 's_cbranch_scc1',
         'v_add_u32_e32', 'v_pk_add_u16', 's_waitcnt']
for label, ins in blocks:
    if len(ins) < lim:
        continue
    c = Counter(ins)
    valu = sum(v for k, v in c.items() if k.startswith('v_'))
    print(f"{label:24s} n={len(ins):5d} valu={valu:5d} " + ' '.join(f"{w.replace('_b32','').replace('v_','')}={c[w]}" for w in watch if c[w]))
