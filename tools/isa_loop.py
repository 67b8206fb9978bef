"""Per-loop instruction counts of one kernel in a hipcc --save-temps .s file (dev
tool): groups basic blocks by their 'Loop: Header=' annotation."""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
start = next(i for i, l in enumerate(lines) if l.split(':')[0] == key)
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
cur = 'top'
loops = collections.defaultdict(collections.Counter)
for l in lines[start:end]:
    m = re.search(r'Loop: Header=(\S+) Depth=(\d)', l)
    if l.startswith('.LBB') or l.startswith('; %bb'):
        cur = 'top'
        if m:
            cur = m.group(1) + '/d' + m.group(2)
        continue
    if m:
        cur = m.group(1) + '/d' + m.group(2)
        continue
    t = l.strip().split(' ')[0]
    if t and not t.startswith(('.', ';')) and not t.endswith(':'):
        loops[cur][t] += 1
for name, c in sorted(loops.items(), key=lambda kv: -sum(kv[1].values())):
    tot = sum(c.values())
    if tot < 20:
        continue
    valu = sum(v for k, v in c.items() if k.startswith('v_'))
    print('%-16s total %5d valu %5d scratch %3d  top: %s' % (
        name, tot, valu, sum(v for k, v in c.items() if 'scratch' in k),
        ', '.join('%s %d' % kv for kv in c.most_common(8))))
