"""Size / time parsing and pretty-printing.

Behavioural parity with the reference's ``FormatUtils`` (core/common/src/main/java/alluxio/util/
FormatUtils.java: ``parseSpaceSize``, ``parseTimeSize``, ``getSizeFromBytes``) — the stress-bench
and configuration layers accept the same ``"128m"``, ``"4k"``, ``"30s"``, ``"1min"`` spellings.
"""
from __future__ import annotations

import re

_SIZE_UNITS = {
    "": 1, "b": 1,
    "k": 1 << 10, "kb": 1 << 10, "kib": 1 << 10,
    "m": 1 << 20, "mb": 1 << 20, "mib": 1 << 20,
    "g": 1 << 30, "gb": 1 << 30, "gib": 1 << 30,
    "t": 1 << 40, "tb": 1 << 40, "tib": 1 << 40,
    "p": 1 << 50, "pb": 1 << 50, "pib": 1 << 50,
}

_TIME_UNITS_MS = {
    "": 1, "ms": 1, "millisecond": 1, "milliseconds": 1,
    "s": 1000, "sec": 1000, "second": 1000, "seconds": 1000,
    "m": 60_000, "min": 60_000, "minute": 60_000, "minutes": 60_000,
    "h": 3_600_000, "hr": 3_600_000, "hour": 3_600_000, "hours": 3_600_000,
    "d": 86_400_000, "day": 86_400_000, "days": 86_400_000,
}

_NUM_UNIT = re.compile(r"^\s*([0-9]*\.?[0-9]+)\s*([a-zA-Z]*)\s*$")


def parse_space_size(spec) -> int:
    """Parse ``"64MB"`` / ``"4k"`` / ``"1.5g"`` / ``1024`` into a byte count."""
    if isinstance(spec, (int,)):
        return int(spec)
    m = _NUM_UNIT.match(str(spec))
    if not m:
        raise ValueError(f"invalid space size: {spec!r}")
    num, unit = m.group(1), m.group(2).lower()
    if unit not in _SIZE_UNITS:
        raise ValueError(f"invalid space unit in {spec!r}")
    return int(float(num) * _SIZE_UNITS[unit])


def parse_time_size(spec) -> int:
    """Parse ``"30s"`` / ``"1min"`` / ``"500ms"`` / ``1000`` into milliseconds."""
    if isinstance(spec, (int,)):
        return int(spec)
    m = _NUM_UNIT.match(str(spec))
    if not m:
        raise ValueError(f"invalid time size: {spec!r}")
    num, unit = m.group(1), m.group(2).lower()
    if unit not in _TIME_UNITS_MS:
        raise ValueError(f"invalid time unit in {spec!r}")
    return int(float(num) * _TIME_UNITS_MS[unit])


def bytes_to_human(n: int) -> str:
    """``1536`` -> ``"1536.00B"`` style used by the shell's ``du``/``report`` output."""
    n = float(n)
    for unit in ("B", "KB", "MB", "GB", "TB", "PB"):
        if abs(n) < 1024 or unit == "PB":
            return f"{n:.2f}{unit}"
        n /= 1024.0
    return f"{n:.2f}PB"


def ms_to_human(ms: int) -> str:
    if ms < 1000:
        return f"{ms} ms"
    s = ms / 1000.0
    if s < 60:
        return f"{s:.2f} sec"
    return f"{s / 60.0:.2f} min"


def mode_to_string(mode: int, is_dir: bool = False) -> str:
    """POSIX mode bits -> ``drwxr-xr-x`` (cf. reference ``FormatUtils.formatMode``)."""
    out = ["d" if is_dir else "-"]
    for shift in (6, 3, 0):
        bits = (mode >> shift) & 7
        out.append("r" if bits & 4 else "-")
        out.append("w" if bits & 2 else "-")
        out.append("x" if bits & 1 else "-")
    return "".join(out)
