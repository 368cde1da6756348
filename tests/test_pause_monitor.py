"""Pause monitor + sampling logger (reference JvmPauseMonitor, SamplingLogger) and their wiring
into the master / worker processes."""
import logging
import threading
import time

from alluxio_amd import metrics as msys
from alluxio_amd.utils.pause_monitor import PauseMonitor, SamplingLogger


def test_thresholds_and_counters(caplog):
    m = msys.metrics("PauseTest")
    pm = PauseMonitor(sleep_s=0.05, info_s=0.2, warn_s=1.0, metrics=m, prefix="PauseTest")
    with caplog.at_level(logging.INFO, logger="alluxio_amd.utils.pause_monitor"):
        assert pm.check(0.01) is None
        assert pm.check(0.5) == "INFO"
        assert pm.check(2.0) == "WARN"
    assert pm.info_exceeded == 1 and pm.warn_exceeded == 1
    assert abs(pm.total_extra_s - 2.51) < 1e-6
    assert m.counter("PauseTest.WarnTimeExceeded").count == 1
    assert any("Detected pause" in r.message for r in caplog.records)


def test_detects_a_gil_hog():
    pm = PauseMonitor(sleep_s=0.02, info_s=0.1, warn_s=5.0).start()
    try:
        time.sleep(0.1)
        import sys
        old = sys.getswitchinterval()
        sys.setswitchinterval(1.0)            # a busy thread keeps the GIL for a long time
        try:
            t0 = time.monotonic()
            while time.monotonic() - t0 < 0.6:
                sum(range(1000))
        finally:
            sys.setswitchinterval(old)
        time.sleep(0.1)
    finally:
        pm.stop()
    assert pm.total_extra_s > 0.1


def test_sampling_logger(caplog):
    sl = SamplingLogger(logging.getLogger("sampling-test"), 60.0)
    with caplog.at_level(logging.WARNING, logger="sampling-test"):
        assert sl.warning("slow %d", 1, key="k")
        assert not sl.warning("slow %d", 2, key="k")
        assert sl.warning("other", key="k2")
    assert sl.suppressed == 1 and len(caplog.records) == 2


def test_processes_run_monitors(tmp_path):
    from alluxio_amd.minicluster import LocalAlluxioCluster
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"},
                             work_dir=str(tmp_path)) as c:
        pm = c.master.pause_monitor
        assert pm is not None and pm.is_started()
        assert c.workers[0].pause_monitor.is_started()
    assert not pm.is_started()
