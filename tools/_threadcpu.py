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
