"""HBM traffic per launch from two rocprofv3 PMC passes (MI355X_MICROARCH.md section HBM).

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR 'KERNEL_SUBSTRING=op name' [...] [--last N] [--json OUT]
FETCH_SIZE and WRITE_SIZE are collected in separate passes (one counter each) over
tools/kprobe.py, which launches each probed operator N times after one warm step;
on gfx950 FETCH_SIZE reads half the bytes of a wide coalesced read, so
traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes per dispatch.  The last N
dispatches of each kernel are its probe launches.
"""
import csv
import glob
import json
import sys


def rows(d, counter):
    f = glob.glob(d + '/**/*counter_collection.csv', recursive=True)[0]
    with open(f) as fh:
        return [(int(r['Dispatch_Id']), r['Kernel_Name'], float(r['Counter_Value']))
                for r in csv.DictReader(fh) if r['Counter_Name'] == counter]


def last(rs, pat, n):
    v = sorted((i, x) for i, k, x in rs if pat in k)
    return [x for _, x in v[-n:]]


def main():
    a = sys.argv[1:]
    out_json, n = None, 20
    if '--json' in a:
        i = a.index('--json')
        out_json = a[i + 1]
        del a[i:i + 2]
    if '--last' in a:
        i = a.index('--last')
        n = int(a[i + 1])
        del a[i:i + 2]
    fr, wr = rows(a[0], 'FETCH_SIZE'), rows(a[1], 'WRITE_SIZE')
    res = {'rule': '(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes per dispatch; separate --pmc passes; '
                   'mean of the last %d dispatches of each kernel (tools/kprobe.py launches)' % n, 'ops': {}}
    for pair in a[2:]:
        pat, op = pair.split('=', 1)
        fe, wb = last(fr, pat, n), last(wr, pat, n)
        f_b = 2 * 1024 * sum(fe) / len(fe)
        w_b = 1024 * sum(wb) / len(wb)
        res['ops'][op] = dict(kernel=pat, dispatches=len(fe), fetch_bytes=f_b, write_bytes=w_b,
                              traffic_bytes=f_b + w_b)
    print(json.dumps(res, indent=1))
    if out_json:
        with open(out_json, 'w') as fh:
            json.dump(res, fh, indent=1)


if __name__ == '__main__':
    main()
