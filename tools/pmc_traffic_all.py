"""Per-operator HBM traffic of the codec convolutions from two rocprofv3 PMC passes over
tools/pmc_all.py (MI355X_MICROARCH.md HBM section: separate FETCH_SIZE / WRITE_SIZE passes; on
gfx950 FETCH_SIZE counts half the bytes of a wide coalesced read, so traffic =
(2 FETCH_SIZE + WRITE_SIZE) x 1024 B per dispatch).  The conv dispatches of each pass are matched to
the manifest in launch order (the last sum(launches) conv_fwd / conv_bwd dispatches).
usage: python tools/pmc_traffic_all.py FETCH_DIR WRITE_DIR MANIFEST.json OUT.json"""
import csv
import glob
import json
import sys


def conv_rows(d, counter):
    f = glob.glob(d + '/**/*counter_collection.csv', recursive=True)[0]
    with open(f) as fh:
        rs = [(int(r['Dispatch_Id']), float(r['Counter_Value'])) for r in csv.DictReader(fh)
              if r['Counter_Name'] == counter and ('conv_fwd_kernel' in r['Kernel_Name'] or
                                                   'conv_bwd_kernel' in r['Kernel_Name'])]
    return [v for _, v in sorted(rs)]


def main():
    fdir, wdir, man, out = sys.argv[1:5]
    m = json.load(open(man))
    total = sum(x['launches'] for x in m['launches'])
    fe, wr = conv_rows(fdir, 'FETCH_SIZE')[-total:], conv_rows(wdir, 'WRITE_SIZE')[-total:]
    assert len(fe) == total and len(wr) == total, (len(fe), len(wr), total)
    res = dict(conv_hip_sha1=m['conv_hip_sha1'], config=m.get('config', 'c64'),
               rule='(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes per dispatch; separate --pmc passes over '
                    'tools/pmc_all.py; mean over each operator\'s launches', ops={})
    k = 0
    for x in m['launches']:
        n = x['launches']
        f = 2 * 1024 * sum(fe[k:k + n]) / n
        w = 1024 * sum(wr[k:k + n]) / n
        res['ops'][x['op']] = dict(fetch_bytes=f, write_bytes=w, traffic_bytes=f + w,
                                   algorithmic_bytes=x['algorithmic_bytes'],
                                   traffic_over_algorithmic=(f + w) / x['algorithmic_bytes'])
        k += n
    with open(out, 'w') as fh:
        json.dump(res, fh, indent=1)
    for op, v in res['ops'].items():
        print('%-46s traffic %9.0f B  algorithmic %9.0f B  ratio %.2f' % (op, v['traffic_bytes'],
                                                                        v['algorithmic_bytes'],
                                                                        v['traffic_over_algorithmic']))


if __name__ == '__main__':
    main()
