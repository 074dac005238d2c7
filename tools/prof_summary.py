"""Summarise a rocprofv3 kernel-trace database (rocpd .db): per-kernel calls, total / average time.
rocpd 'top_kernels' durations are in microseconds."""
import glob
import sqlite3
import sys


def rows(path):
    dbs = [path] if path.endswith('.db') else glob.glob(path + '/**/*.db', recursive=True)
    c = sqlite3.connect(dbs[0])
    out = []
    for name, n, tot, avg, pct in c.execute('select name, total_calls, total_duration, average, percentage '
                                            'from top_kernels'):
        short = name.replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0]
        out.append((short, n, tot, avg, pct))
    return out


if __name__ == '__main__':
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    print('%-58s %6s %11s %9s %7s' % ('kernel', 'calls', 'total_us', 'avg_us', 'pct'))
    for short, n, tot, avg, pct in rows(sys.argv[1])[:top]:
        print('%-58s %6d %11.1f %9.2f %6.2f%%' % (short[:58], n, tot, avg, pct))
