"""Host-side list helpers (mirrors hiccup/utils.py:15-139).

Same names, arguments and results as the reference; ``flatten`` is linear
instead of the reference's quadratic ``reduce(+)`` (utils.py:109-113).
"""
import datetime
import functools
import itertools

from . import settings


def debug_msg(msg):
    if settings.DEBUG:
        print("%s %s" % (datetime.datetime.utcnow(), msg))


def group_tuples(l, n):
    assert len(l) % n == 0
    return [tuple(l[i:i + n]) for i in range(0, len(l), n)]


def num_bits_for_int(n):
    return abs(int(n)).bit_length()


def differences(arr):
    if len(arr) == 0:
        return []
    return [arr[0]] + [arr[i] - arr[i - 1] for i in range(1, len(arr))]


def invert_differences(arr):
    arr[0]  # the reference indexes arr[0] first (IndexError on an empty list)
    return list(itertools.accumulate(arr))


def identity(x):
    return x


def group_by(data, key_func=identity, value_func=identity):
    out = {}
    for ele in data:
        out.setdefault(key_func(ele), []).append(value_func(ele))
    return out


def first(l, predicate):
    for ele in l:
        if predicate(ele):
            return ele
    raise RuntimeError("Found nothing to match predicate")


def flatten(l):
    l = list(l)
    if not l:
        # the reference's functools.reduce raises on an empty sequence
        return functools.reduce(lambda x, y: x + y, l)
    if isinstance(l[0], str):
        return "".join(l)
    head = l[0]
    out = list(itertools.chain.from_iterable(l))
    return tuple(out) if isinstance(head, tuple) else out


def img_as_list(img):
    return flatten(img.tolist())


def size(shape):
    return shape[0] * shape[1]


def dict_map(d, f):
    return dict((k, f(k, v)) for k, v in d.items())


def is_gray(img):
    return len(img.shape) == 2 and img.shape[0] > 1 and img.shape[1] > 1
