"""Per-basic-block VALU / total instruction counts of one loop of a kernel in a
hipcc --save-temps .s file (dev tool): python3 tools/isa_blocks.py file.s kernel loop_header"""
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
key, hdr = sys.argv[2], sys.argv[3]
start = next(i for i, l in enumerate(lines) if l.split(':')[0] == key)
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
blk, inloop, cnt = None, False, {}
order = []
for l in lines[start:end]:
    m = re.match(r'^(\.LBB\S+|; %bb\.\d+):', l)
    if m:
        blk = m.group(1)
        inloop = ('Header=' + hdr) in l
        order.append(blk)
        cnt[blk] = [0, 0, inloop]
        continue
    if blk is None:
        continue
    if ('Header=' + hdr) in l:
        cnt[blk][2] = True
    t = l.strip().split(' ')[0]
    if t and not t.startswith(('.', ';')) and not t.endswith(':'):
        cnt[blk][0] += 1
        if t.startswith('v_'):
            cnt[blk][1] += 1
for b in order:
    if cnt[b][2]:
        print('%-14s total %5d valu %5d' % (b, cnt[b][0], cnt[b][1]))
