"""Census of a kernel's DP loop in a hipcc -S listing: sums the blocks that
hold packed adds (the column steps) and reports VALU per column and any
spill traffic inside them.

usage: python tools/hotloop.py k.s <kernel-symbol-substring> <rows-per-column>
"""
import sys
from collections import Counter

src, pat, rows = sys.argv[1], sys.argv[2], int(sys.argv[3])
s = open(src).read()
name = None
for line in s.split('\n'):
    t = line.split(';')[0].strip()
    if t.endswith(':') and pat in t and not t.startswith('.'):
        name = t[:-1]
        break
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
blocks, cur = [], Counter()
for line in s[i:j].split('\n'):
    head = line.split(';')[0].rstrip()
    if head and not line.startswith(('\t', ' ', ';')) and head.endswith(':'):
        blocks.append(cur)
        cur = Counter()
    elif line.startswith('\t') and not line.strip().startswith(('.', ';')):
        cur[line.strip().split()[0]] += 1
blocks.append(cur)
tot = Counter()
for b in blocks:
    if b['v_pk_maximum3_f16'] >= 2 * rows:
        tot.update(b)
cols = tot['ds_read_b128'] / (rows / 4)     # each column loads its next pair row
valu = sum(v for k, v in tot.items() if k.startswith('v_'))
print(f"{name}: {cols:.0f} columns, VALU/column {valu / cols:.1f}, VALU/cell {valu / cols / (2 * rows):.3f}")
print("  per column:", {k: round(v / cols, 2) for k, v in sorted(tot.items(), key=lambda x: -x[1])})
