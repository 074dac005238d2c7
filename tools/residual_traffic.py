"""HBM traffic per launch of the residual kernel from two rocprofv3 PMC passes over tools/residual_bench.py
(--no-cpu): the cgr dispatches in launch order are the CONFIGS x (flux off, on) x 21 launches of the bench
(one warm + 20 timed); traffic = (2 FETCH_SIZE + WRITE_SIZE) x 1024 B per dispatch (gfx950,
MI355X_MICROARCH.md HBM section), averaged over each configuration's 20 timed launches.
usage: python tools/residual_traffic.py FETCH_DIR WRITE_DIR OUT.json"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from residual_bench import CONFIGS, stencil_sha  # noqa: E402


def rows(d, counter):
    f = glob.glob(d + '/**/*counter_collection.csv', recursive=True)[0]
    acc = {}
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if r['Counter_Name'] == counter and 'cgr_' in r['Kernel_Name']:
                k = int(r['Dispatch_Id'])
                acc[k] = acc.get(k, 0.0) + float(r['Counter_Value'])
    return [acc[k] for k in sorted(acc)]


def main():
    fdir, wdir, out = sys.argv[1:4]
    fe, wr = rows(fdir, 'FETCH_SIZE'), rows(wdir, 'WRITE_SIZE')
    per = 21
    need = len(CONFIGS) * 2 * per
    assert len(fe) == need and len(wr) == need, (len(fe), len(wr), need)
    ents = []
    k = 0
    for n, nc, N in CONFIGS:
        for flux in (False, True):
            f = 2 * 1024 * sum(fe[k + 1:k + per]) / (per - 1)
            w = 1024 * sum(wr[k + 1:k + per]) / (per - 1)
            alg = 4.0 * N * (n * n + (n + 1) * (n - 1) + 4 + (nc + 1) ** 2 + (2 * nc * nc if flux else 0))
            ents.append(dict(grid=n, nc=nc, fields=N, flux=flux, fetch_bytes=f, write_bytes=w, traffic_bytes=f + w,
                             algorithmic_bytes=alg, traffic_over_algorithmic=(f + w) / alg))
            print('%4d^2 flux %d: traffic %.1f MB, algorithmic %.1f MB, ratio %.3f' % (n, flux, (f + w) / 1e6,
                                                                                      alg / 1e6, (f + w) / alg))
            k += per
    with open(out, 'w') as fh:
        json.dump(dict(stencil_sha1=stencil_sha(), rule='(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes per dispatch, '
                       'separate --pmc passes over tools/residual_bench.py --no-cpu', entries=ents), fh, indent=1)


if __name__ == '__main__':
    main()
