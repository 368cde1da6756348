"""Per-thread-name CPU of this process (benches): native threads name themselves (frpc-io-N,
ufs-file, s3-upload, sink-pair); Python threads show as the interpreter's name."""
import os


def thread_cpu(pid: str = "self") -> dict:
    """{thread name group: CPU seconds} for process ``pid`` (digits stripped from names)."""
    out: dict = {}
    tck = os.sysconf("SC_CLK_TCK")
    base = f"/proc/{pid}/task"
    for t in os.listdir(base):
        try:
            with open(f"{base}/{t}/stat") as f:
                s = f.read()
        except OSError:
            continue
        name = s[s.index("(") + 1:s.rindex(")")].rstrip("0123456789").rstrip("-")
        fl = s.rsplit(")", 1)[1].split()
        out[name] = out.get(name, 0.0) + (int(fl[11]) + int(fl[12])) / tck
    return out


def busy(before: dict, after: dict, seconds: float) -> dict:
    """{group: cores busy} between two thread_cpu() samples, largest first."""
    d = {k: (after.get(k, 0.0) - before.get(k, 0.0)) / max(seconds, 1e-9) for k in after}
    return {k: round(v, 2) for k, v in sorted(d.items(), key=lambda kv: -kv[1]) if v >= 0.01}


def python_thread_cpu() -> dict:
    """{Python thread name (digits stripped): CPU seconds} of this process's live Python threads,
    read from /proc by each thread's native id (which Python threads burn the interpreter)."""
    import threading
    tck = os.sysconf("SC_CLK_TCK")
    out: dict = {}
    for th in threading.enumerate():
        tid = getattr(th, "native_id", None)
        if tid is None:
            continue
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                s = f.read()
        except OSError:
            continue
        fl = s.rsplit(")", 1)[1].split()
        name = th.name.rstrip("0123456789").rstrip("-_")
        out[name] = out.get(name, 0.0) + (int(fl[11]) + int(fl[12])) / tck
    return out


def python_user_sys() -> tuple:
    """(user, system) CPU seconds summed over this process's live Python threads: user time is the
    interpreter (and the C code it calls), system time the syscalls they make -- e.g. the unlink of
    a deleted UFS file's pages, which is kernel work on a Python thread."""
    import threading
    tck = os.sysconf("SC_CLK_TCK")
    u = k = 0.0
    for th in threading.enumerate():
        tid = getattr(th, "native_id", None)
        if tid is None:
            continue
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                fl = f.read().rsplit(")", 1)[1].split()
        except OSError:
            continue
        u += int(fl[11]) / tck
        k += int(fl[12]) / tck
    return u, k


class StackSampler:
    """Samples the innermost alluxio_amd frames of every Python thread that burned CPU since the
    previous sample (per-thread ticks from /proc), every ``interval`` s: a cheap attribution of
    interpreter time in benches (it holds the GIL for each sample)."""

    def __init__(self, interval: float = 0.02, depth: int = 5):
        import threading
        self.interval, self.depth = interval, depth
        self.counts: dict = {}
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True, name="stack-sampler")

    def start(self):
        self._t.start()
        return self

    @staticmethod
    def _ticks(native_id) -> int:
        try:
            with open(f"/proc/self/task/{native_id}/stat") as f:
                fl = f.read().rsplit(")", 1)[1].split()
            return int(fl[11]) + int(fl[12])
        except OSError:
            return -1

    def _run(self):
        import sys
        import threading
        me = threading.get_ident()
        last: dict = {}
        while not self._stop.wait(self.interval):
            natives = {th.ident: th.native_id for th in threading.enumerate()}
            for tid, fr in sys._current_frames().items():
                if tid == me:
                    continue
                nid = natives.get(tid)
                ticks = self._ticks(nid) if nid is not None else -1
                busy = ticks > last.get(tid, ticks)      # burned CPU since the last sample
                last[tid] = ticks
                if not busy:
                    continue
                keys = []
                f = fr
                while f is not None and len(keys) < self.depth:
                    fn = f.f_code.co_filename
                    if "alluxio_amd" in fn:
                        keys.append(f"{fn.rsplit('alluxio_amd/', 1)[-1]}:{f.f_code.co_name}")
                    f = f.f_back
                if not keys:
                    continue
                k = " < ".join(keys)
                self.counts[k] = self.counts.get(k, 0) + 1

    def stop(self, top: int = 25) -> list:
        self._stop.set()
        self._t.join()
        return sorted(self.counts.items(), key=lambda kv: -kv[1])[:top]
