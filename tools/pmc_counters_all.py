"""Per-operator averages of arbitrary SQ counters from one rocprofv3 --pmc pass over tools/pmc_all.py
(conv dispatches matched to the manifest in launch order, as tools/pmc_traffic_all.py).
usage: python tools/pmc_counters_all.py PMC_DIR MANIFEST.json [COUNTER ...]"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    pdir, man = sys.argv[1:3]
    m = json.load(open(man))
    f = glob.glob(pdir + '/**/*counter_collection.csv', recursive=True)[0]
    rows = defaultdict(dict)
    names = {}
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if 'conv_fwd_kernel' in r['Kernel_Name'] or 'conv_bwd_kernel' in r['Kernel_Name']:
                d = int(r['Dispatch_Id'])
                rows[d][r['Counter_Name']] = float(r['Counter_Value'])
                names[d] = r['Kernel_Name']
    counters = sys.argv[3:] or sorted({c for v in rows.values() for c in v})
    disp = sorted(rows)
    total = sum(x['launches'] for x in m['launches'])
    disp = disp[-total:]
    assert len(disp) == total, (len(disp), total)
    k = 0
    print('%-46s' % 'op' + ''.join('%22s' % c for c in counters))
    for x in m['launches']:
        n = x['launches']
        vals = [sum(rows[d].get(c, 0.0) for d in disp[k:k + n]) / n for c in counters]
        print('%-46s' % x['op'] + ''.join('%22.0f' % v for v in vals))
        k += n


if __name__ == '__main__':
    main()
