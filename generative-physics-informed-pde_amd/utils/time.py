"""Progress timing for training drivers (the role of the reference's utils/time.py).

training.py uses exactly two things (training.py:13,401,446-448): ``Timer(N)`` created before an
N-step loop and ``timer.RRT(step=n)``, a printable estimate of the remaining run time.  This module
provides that interface plus section timing, written for this package:

* ``Timer.RRT(step)`` extrapolates linearly from the elapsed monotonic time (perf_counter) and the
  fraction of steps done; ``Timer.ETA(step)`` turns it into a wall-clock date.
* ``with timer('name'):`` adds the block's duration to a named section; ``str(timer)`` tabulates
  the sections with their share of the elapsed time (the reference divides by a constant 10, which
  is not a share; not reproduced).
* ``StopWatch`` measures a single interval.
"""
import time
from datetime import datetime, timedelta


def _fmt_days(seconds):
    seconds = max(0.0, float(seconds))
    d, rem = divmod(int(round(seconds)), 86400)
    h, rem = divmod(rem, 3600)
    m, s = divmod(rem, 60)
    return '{:d} Days, {:02d}h:{:02d}m:{:02d}s'.format(d, h, m, s)


class StopWatch(object):
    """One interval: start() ... stop(); runtime() in seconds."""

    def __init__(self, start=True):
        self._begin = None
        self._end = None
        if start:
            self.start()

    def start(self):
        self._begin = time.perf_counter()
        self._end = None

    def stop(self):
        self._end = time.perf_counter()

    def runtime(self):
        end = self._end if self._end is not None else time.perf_counter()
        return end - self._begin

    def runtime_str(self):
        return str(timedelta(seconds=self.runtime()))


class Timer(object):
    """Remaining-runtime estimate of an N-step loop and named section totals."""

    def __init__(self, NumSteps):
        if NumSteps <= 0:
            raise ValueError('NumSteps must be positive')
        self._n_total = NumSteps
        self._origin = time.perf_counter()
        self._stopped_at = None
        self._sections = {}          # name -> [seconds, entries]
        self._open = []              # stack of (name, entry time)
        self._pending = None

    # ---------------------------------------------------------------- progress
    def elapsed(self):
        end = self._stopped_at if self._stopped_at is not None else time.perf_counter()
        return end - self._origin

    def remaining_seconds(self, step):
        """Linear extrapolation: elapsed * (N - step) / step (step 0 counts as a tiny fraction)."""
        done = max(float(step), 1e-4)
        return self.elapsed() * (self._n_total - done) / done

    def RRT(self, step, verbose=False):
        s = _fmt_days(self.remaining_seconds(step))
        if verbose:
            print('Estimated Remaining runtime: ' + s)
        return s

    def ETA(self, step):
        when = datetime.now() + timedelta(seconds=self.remaining_seconds(step))
        return when.strftime('ETA: %d.%m.%Y, %H:%M:%S')

    def stop(self):
        self._stopped_at = time.perf_counter()

    # ---------------------------------------------------------------- sections
    def __call__(self, name):
        self._pending = name
        return self

    def __enter__(self):
        name = self._pending if self._pending is not None else 'default'
        self._pending = None
        self._open.append((name, time.perf_counter()))
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        name, t0 = self._open.pop()
        acc = self._sections.setdefault(name, [0.0, 0])
        acc[0] += time.perf_counter() - t0
        acc[1] += 1
        return False

    def sections(self):
        return {k: v[0] for k, v in self._sections.items()}

    def __str__(self):
        total = self.elapsed()
        rows = [('section', 'seconds', 'entries', 'share'), ('overall', '%.3f' % total, '', '1.000')]
        for name, (sec, cnt) in sorted(self._sections.items(), key=lambda kv: -kv[1][0]):
            rows.append((str(name), '%.3f' % sec, str(cnt), '%.3f' % (sec / total if total > 0 else 0.0)))
        widths = [max(len(r[i]) for r in rows) for i in range(4)]
        return '\n'.join('  '.join(c.rjust(widths[i]) if i else c.ljust(widths[i]) for i, c in enumerate(r))
                         for r in rows)
