"""Stack sampler used for slow-path profiling of server processes (utils/sampler.py)."""
import threading
import time

from alluxio_amd.utils.sampler import StackSampler


def _busy(stop):
    while not stop.is_set():
        sum(range(2000))
        time.sleep(0)


def test_sampler_sees_busy_thread():
    stop = threading.Event()
    t = threading.Thread(target=_busy, args=(stop,), daemon=True)
    t.start()
    s = StackSampler(interval_s=0.001).start()
    time.sleep(0.3)
    s.stop()
    stop.set()
    t.join()
    assert s.samples > 0
    rep = s.report()
    assert "test_sampler.py:_busy" in rep
    assert rep.startswith("samples:")
