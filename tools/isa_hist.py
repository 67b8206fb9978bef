"""Instruction histogram of one kernel in a hipcc --save-temps .s file (dev tool)."""
import collections
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2]
a = next(i for i in range(len(s)) if s.startswith(key, i) and s[i:].split('\n', 1)[0].rstrip().endswith(key.split(':')[0] + ': ; @' + key.split(':')[0]) or False) if False else None
lines = s.split('\n')
start = next(i for i, l in enumerate(lines) if l.startswith(key) and l.split(':')[0] == key)
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
body = lines[start:end]
c = collections.Counter()
for l in body:
    t = l.strip().split(' ')[0]
    if t and not t.startswith(('.', ';')) and not t.endswith(':'):
        c[t] += 1
print('instructions', sum(c.values()))
for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(v, k)
print('scratch ops', sum(v for k, v in c.items() if 'scratch' in k))
