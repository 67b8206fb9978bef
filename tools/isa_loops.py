"""dev: instruction mix of a kernel's loops in a hipcc -S listing.
usage: python tools/isa_loops.py file.s <kernel-substring>"""
import collections
import re
import sys


def classify(op):
    if op.startswith('v_'):
        if '_f64' in op:
            return 'f64'
        if op.startswith('v_pk_'):
            return 'pk'
        if op.startswith('v_cmp'):
            return 'cmp'
        return 'valu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('global_', 'buffer_', 'flat_')):
        return 'vmem'
    if op.startswith('s_'):
        return 'salu'
    return 'other'


def main():
    lines = open(sys.argv[1]).read().split('\n')
    key = sys.argv[2]
    i0 = next(i for i, l in enumerate(lines) if re.match(r'^\S+:', l) and key in l.split(':')[0] and not l.startswith('.'))
    body = []
    for l in lines[i0 + 1:]:
        s = l.strip()
        if s.startswith('s_endpgm') or s.startswith('.Lfunc_end'):
            break
        if re.match(r'^\.LBB\S+:', s):
            body.append(('label', s.split(':')[0]))
        elif s and not s.startswith(('.', ';')):
            body.append(('ins', s.split()[0], s))
    labels = {b[1]: k for k, b in enumerate(body) if b[0] == 'label'}
    print('total', collections.Counter(classify(b[1]) for b in body if b[0] == 'ins'))
    for k, b in enumerate(body):
        if b[0] == 'ins' and b[1].startswith('s_cbranch') or (b[0] == 'ins' and b[1] == 's_branch'):
            tgt = b[2].split()[-1]
            if tgt in labels and labels[tgt] < k:
                seg = [x for x in body[labels[tgt]:k + 1] if x[0] == 'ins']
                c = collections.Counter(classify(x[1]) for x in seg)
                print('loop %s..%d: %d ins' % (tgt, k, len(seg)), dict(c))


main()
