"""Per-kernel average durations of a rocprofv3 kernel-trace database, split at the first dispatch of a
marker kernel (e.g. two workloads run back to back in one process).
usage: python tools/prof_split.py run_results.db MARKER_SUBSTRING [occurrence]"""
import collections
import sqlite3
import sys


def main():
    db, marker = sys.argv[1], sys.argv[2]
    occ = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    c = sqlite3.connect(db)
    ks = list(c.execute('select name, start, duration from kernels order by start'))
    seen, cut = 0, len(ks)
    for n, (name, _, _) in enumerate(ks):
        if marker in name:
            seen += 1
            if seen == occ:
                cut = n
                break
    for part, rows in (('part 1', ks[:cut]), ('part 2', ks[cut:])):
        agg = collections.OrderedDict()
        for name, _, dur in rows:
            short = name.replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0]
            a = agg.setdefault(short, [0, 0.0])
            a[0] += 1
            a[1] += dur / 1e3
        print('== %s (%d dispatches)' % (part, len(rows)))
        for short, (n, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
            print('%-58s %6d %11.1f %9.2f' % (short[:58], n, tot, tot / n))


if __name__ == '__main__':
    main()
