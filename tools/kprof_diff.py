"""Per-operator diff of two bench.py --kprof files: python tools/kprof_diff.py A.json B.json [min_us]"""
import json
import sys


def main(a, b, min_us=0.5):
    A = {x['op']: x['ms'] * 1e3 for x in json.load(open(a))}
    B = {x['op']: x['ms'] * 1e3 for x in json.load(open(b))}
    print('total %.1f -> %.1f us' % (sum(A.values()), sum(B.values())))
    for op in sorted(A, key=lambda o: B.get(o, 0) - A[o]):
        d = B.get(op, 0) - A[op]
        if abs(d) >= float(min_us):
            print('%-45s %7.2f -> %7.2f  (%+.2f)' % (op, A[op], B.get(op, 0), d))


if __name__ == '__main__':
    main(*sys.argv[1:])
