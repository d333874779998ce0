"""Minimal promises + ``@delayed`` (the role of ``vaex/promise.py`` / ``vaex/delayed.py``):
tasks are promises fulfilled by the executor; ``delayed`` functions run once all their
promise arguments are fulfilled.

Thread-safe: a task scheduled by one thread may be fulfilled by another thread's executor
pass (execution_test.py:79-101 counts from a thread pool), so the state change and the
callback list are guarded by one lock; callbacks run outside it."""
import threading

_LOCK = threading.RLock()


class Promise:
    def __init__(self):
        self._done = False
        self._value = None
        self._error = None
        self._callbacks = []

    @classmethod
    def fulfilled(cls, value):
        p = cls()
        p.fulfill(value)
        return p

    @property
    def isFulfilled(self):
        return self._done and self._error is None

    @property
    def isRejected(self):
        return self._done and self._error is not None

    def fulfill(self, value):
        if isinstance(value, Promise):
            value.then(self.fulfill, self.reject)
            return
        with _LOCK:
            if self._done:
                return
            self._done, self._value = True, value
            cbs, self._callbacks = self._callbacks, []
        for ok, _ in cbs:
            ok(value)

    def reject(self, error):
        with _LOCK:
            if self._done:
                return
            self._done, self._error = True, error
            cbs, self._callbacks = self._callbacks, []
        for _, bad in cbs:
            bad(error)

    def then(self, on_ok, on_error=None):
        out = Promise()

        def ok(v):
            try:
                out.fulfill(on_ok(v))
            except Exception as e:  # noqa
                out.reject(e)

        def bad(e):
            if on_error is not None:
                try:
                    out.fulfill(on_error(e))
                except Exception as e2:  # noqa
                    out.reject(e2)
            else:
                out.reject(e)

        with _LOCK:
            done = self._done
            if not done:
                self._callbacks.append((ok, bad))
        if done:
            (ok(self._value) if self._error is None else bad(self._error))
        return out

    def get(self):
        if not self._done:
            raise RuntimeError("promise not fulfilled yet: call df.execute()")
        if self._error is not None:
            raise self._error
        return self._value


def delayed(f):
    """Call ``f`` with promise arguments replaced by their values once all are fulfilled."""

    def wrapped(*args, **kwargs):
        promises = [a for a in list(args) + list(kwargs.values()) if isinstance(a, Promise)]
        result = Promise()

        fired = []

        def run(_=None):
            with _LOCK:
                if not all(p._done for p in promises) or fired:
                    return
                fired.append(True)
            for p in promises:
                if p._error is not None:
                    result.reject(p._error)
                    return
            a2 = [a._value if isinstance(a, Promise) else a for a in args]
            k2 = {k: (v._value if isinstance(v, Promise) else v) for k, v in kwargs.items()}
            try:
                result.fulfill(f(*a2, **k2))
            except Exception as e:  # noqa
                result.reject(e)

        if not promises:
            run()
        for p in promises:
            p.then(run, run)
        return result

    return wrapped
