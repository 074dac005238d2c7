"""Wall-clock helpers the training driver imports (reference utils/time.py:1-103).

``Timer(N)`` projects the remaining runtime of an N-step loop (``RRT``, ``ETA``) and
accumulates named sections (``with timer('name'):``); ``StopWatch`` measures one
interval.  The reference renders the section table with prettytable, which is not
a dependency here: ``str(timer)`` prints the same three columns as plain text.
"""
import time
from datetime import datetime, timedelta


class StopWatch(object):

    def __init__(self, start=True):
        self._t1 = None
        self._t2 = None
        if start:
            self.start()

    def start(self):
        self._t1 = time.time()

    def stop(self):
        self._t2 = time.time()

    def runtime(self):
        return self._t2 - self._t1

    def runtime_str(self):
        return str(timedelta(seconds=self.runtime()))


class Timer(object):

    def __init__(self, NumSteps):
        self._start = datetime.now()
        self._t1 = time.time()
        self._NumSteps = NumSteps
        self._stop_time = None
        self._threads = dict()
        self._thread_start_time = None
        self._active_thread = None

    def __call__(self, thread):
        if thread not in self._threads:
            self._threads[thread] = 0
        self._active_thread = thread
        self._thread_start_time = time.time()
        return self

    def _rrt(self, step):
        if step == 0:
            step = 0.0001
        fraction = step / self._NumSteps
        curr = time.time() - self._t1
        return (1 / fraction) * curr - curr

    def stop(self):
        self._stop_time = datetime.now()

    def RRT(self, step, verbose=False):
        td = timedelta(seconds=self._rrt(step))
        s = '{:d} Days, {:02d}h:{:02d}m:{:02d}s'.format(td.days, td.seconds // 3600, (td.seconds // 60) % 60,
                                                       td.seconds % 60)
        if verbose:
            print('Estimated Remaining runtime: ' + s)
        return s

    def ETA(self, step):
        eta = timedelta(seconds=self._rrt(step)) + datetime.now()
        return eta.strftime('ETA: %d.%m.%Y, %H:%M:%S')

    def __enter__(self):
        if self._active_thread is None:
            self('default')
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        self._threads[self._active_thread] += time.time() - self._thread_start_time
        self._active_thread = None

    def __str__(self):
        rows = [('Job', 'Runtime', 'Fraction'), ('Overall', str(datetime.now()), '1')]
        # the reference divides by a constant 10 (utils/time.py:94); kept
        rows += [(str(k), '%.6f' % v, '%.6f' % (v / 10)) for k, v in self._threads.items()]
        w = [max(len(r[i]) for r in rows) for i in range(3)]
        return '\n'.join(' | '.join(c.ljust(w[i]) for i, c in enumerate(r)) for r in rows)
