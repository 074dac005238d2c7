"""Timeline of one training step from a rocprofv3 kernel-trace database (rocpd .db).

usage: python tools/step_timeline.py <dir-or-db> [step_index_from_end]
Takes the window between two consecutive step_epilogue_kernel ends, prints every kernel
dispatch in it (queue, start offset, duration, idle gap before it on the whole device) and
the totals: busy time (union of kernel intervals) vs window length.
"""
import glob
import sqlite3
import sys


def main():
    path = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    db = path if path.endswith('.db') else glob.glob(path + '/**/*.db', recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute('select name, queue_id, start, end from kernels order by start').fetchall()
    ends = [r[3] for r in rows if 'step_epilogue' in r[0]]
    t0, t1 = ends[-back - 1], ends[-back]
    win = [r for r in rows if r[2] >= t0 and r[2] < t1]
    busy_end = t0
    busy = 0
    print('%-44s %5s %9s %8s %7s' % ('kernel', 'queue', 'start_us', 'dur_us', 'idle_us'))
    for name, q, s, e in win:
        short = name.replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0][:44]
        idle = max(0, s - busy_end)
        print('%-44s %5d %9.1f %8.1f %7.1f' % (short, q, (s - t0) / 1e3, (e - s) / 1e3, idle / 1e3))
        busy += max(0, e - max(s, busy_end))
        busy_end = max(busy_end, e)
    print('window %.1f us, busy %.1f us, idle %.1f us, %d kernels' % ((t1 - t0) / 1e3, busy / 1e3,
                                                                     (t1 - t0 - busy) / 1e3, len(win)))
    # every traced step (the window above is one of them; traced steps run longer than untraced ones)
    w = sorted((b - a) / 1e3 for a, b in zip(ends, ends[1:]))
    if w:
        print('all %d traced step windows: min %.1f us, median %.1f us, max %.1f us'
              % (len(w), w[0], w[len(w) // 2], w[-1]))


if __name__ == '__main__':
    main()
