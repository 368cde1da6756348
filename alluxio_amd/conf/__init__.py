"""Configuration: typed key registry + layered sources + path-level overrides.

Parity: InstancedConfiguration (core/common/src/main/java/alluxio/conf/InstancedConfiguration.java),
source priority DEFAULT < CLUSTER_DEFAULT < SITE_PROPERTY < SYSTEM_PROPERTY < PATH_DEFAULT <
RUNTIME < MOUNT_OPTION (Source.java:30-80), ``${key}`` substitution, ``alluxio-site.properties``
discovery (ConfigurationUtils.java:394-601), path configuration (conf/path/*.java) and the
cluster config hash exchanged with the master (ConfigHashSync).
"""
from __future__ import annotations

import enum
import hashlib
import os
import re
import threading

from ..utils.format import parse_space_size, parse_time_size
from . import keys as _keys
from .keys import K, PropertyKey, Scope, Templates  # noqa: F401

SITE_PROPERTIES = "alluxio-site.properties"


class Source(enum.IntEnum):
    DEFAULT = 0
    CLUSTER_DEFAULT = 1
    SITE_PROPERTY = 2
    SYSTEM_PROPERTY = 3
    PATH_DEFAULT = 4
    RUNTIME = 5
    MOUNT_OPTION = 6


_SUBST = re.compile(r"\$\{([^}]+)\}")


def _keyname(key) -> str:
    return key.name if isinstance(key, PropertyKey) else str(key)


def site_properties_path() -> str:
    """Where ``bootstrapConf`` writes / the first site-properties location searched."""
    d = os.environ.get("ALLUXIO_CONF_DIR") or os.path.expanduser("~/.alluxio")
    return os.path.join(d, SITE_PROPERTIES)


class Configuration:
    def __init__(self, props: dict | None = None, load_site: bool = False):
        self._lock = threading.RLock()
        self._values: dict[str, tuple[str, Source]] = {}
        if load_site:
            self._load_site_properties()
            self._load_env()
        if props:
            for k, v in props.items():
                self.set(k, v, Source.RUNTIME)

    # --- sources -------------------------------------------------------------------------------
    def _load_site_properties(self) -> None:
        dirs = [os.environ.get("ALLUXIO_CONF_DIR"), os.path.expanduser("~/.alluxio"), "/etc/alluxio"]
        for d in dirs:
            if not d:
                continue
            p = os.path.join(d, SITE_PROPERTIES)
            if os.path.isfile(p):
                self.merge(load_properties_file(p), Source.SITE_PROPERTY)
                return

    def _load_env(self) -> None:
        # ALLUXIO_JAVA_OPTS-style "-Dkey=value" and explicit ALLUXIO_PROP_<key> overrides.
        opts = os.environ.get("ALLUXIO_OPTS", "")
        for tok in opts.split():
            if tok.startswith("-D") and "=" in tok:
                k, v = tok[2:].split("=", 1)
                self.set(k, v, Source.SYSTEM_PROPERTY)

    def merge(self, props: dict, source: Source = Source.RUNTIME) -> None:
        for k, v in props.items():
            self.set(k, v, source)

    # --- accessors -----------------------------------------------------------------------------
    def set(self, key, value, source: Source = Source.RUNTIME) -> None:
        name = _keys.get(_keyname(key)).name
        with self._lock:
            cur = self._values.get(name)
            if cur is None or cur[1] <= source:
                self._values[name] = (str(value) if value is not None else None, source)

    def unset(self, key) -> None:
        with self._lock:
            self._values.pop(_keys.get(_keyname(key)).name, None)

    def is_set(self, key) -> bool:
        name = _keys.get(_keyname(key)).name
        with self._lock:
            if name in self._values and self._values[name][0] is not None:
                return True
        return _keys.get(name).default is not None

    def is_set_by_user(self, key) -> bool:
        with self._lock:
            return _keys.get(_keyname(key)).name in self._values

    def source(self, key) -> Source:
        with self._lock:
            v = self._values.get(_keys.get(_keyname(key)).name)
        return v[1] if v else Source.DEFAULT

    def get_raw(self, key):
        pk = _keys.get(_keyname(key))
        with self._lock:
            v = self._values.get(pk.name)
        return v[0] if v is not None else pk.default

    def get(self, key, default=None) -> str:
        raw = self.get_raw(key)
        if raw is None:
            if default is not None:
                return str(default)
            raise KeyError(f"configuration key {_keyname(key)} is not set")
        return self._substitute(raw, depth=0)

    def _substitute(self, value: str, depth: int) -> str:
        if depth > 16 or "${" not in value:
            return value

        def repl(m):
            inner = m.group(1)
            env = os.environ.get(inner)
            if inner.startswith("env.") or (env is not None and not inner.startswith("alluxio.")):
                return os.environ.get(inner.removeprefix("env."), "")
            raw = self.get_raw(inner)
            if raw is None and inner == "alluxio.home":
                raw = os.environ.get("ALLUXIO_HOME", "/tmp/alluxio_amd")
            return self._substitute(raw or "", depth + 1)
        return _SUBST.sub(repl, value)

    def get_int(self, key, default=None) -> int:
        return int(float(self.get(key, default)))

    def get_float(self, key, default=None) -> float:
        return float(self.get(key, default))

    def get_bool(self, key, default=None) -> bool:
        v = self.get(key, default)
        return str(v).strip().lower() in ("true", "1", "yes", "on")

    def get_bytes(self, key, default=None) -> int:
        return parse_space_size(self.get(key, default))

    def get_ms(self, key, default=None) -> int:
        return parse_time_size(self.get(key, default))

    def get_list(self, key, sep: str = ",", default=None) -> list[str]:
        v = self.get(key, default)
        return [s.strip() for s in v.split(sep) if s.strip()]

    def get_enum(self, key, enum_cls, default=None):
        return enum_cls[self.get(key, default).strip().upper()]

    def get_class_name(self, key, default=None) -> str:
        return self.get(key, default).strip()

    def to_map(self, include_defaults: bool = False) -> dict[str, str]:
        out = {}
        if include_defaults:
            for k in _keys.all_keys():
                if k.default is not None:
                    out[k.name] = k.default
        with self._lock:
            for k, (v, _) in self._values.items():
                if v is not None:
                    out[k] = v
        return out

    def copy(self) -> "Configuration":
        c = Configuration()
        with self._lock:
            c._values = dict(self._values)
        return c

    def hash(self) -> str:
        """Stable hash of the non-default values (reference cluster config hash)."""
        items = sorted(self.to_map().items())
        return hashlib.md5("\n".join(f"{k}={v}" for k, v in items).encode()).hexdigest()

    def validate(self) -> list[str]:
        """Return names of set keys that are unknown (reference ``validate()`` warnings)."""
        with self._lock:
            return [k for k in self._values if not _keys.is_valid(k)]

    # tier helpers ----------------------------------------------------------------------------
    def tier_levels(self) -> int:
        return self.get_int("alluxio.worker.tieredstore.levels")

    def tier_key(self, template, level: int) -> PropertyKey:
        return template.format(level)


def load_properties_file(path: str) -> dict[str, str]:
    """Java ``.properties`` subset: ``key=value`` / ``key: value`` / ``#`` comments / ``\\`` joins."""
    props: dict[str, str] = {}
    with open(path, encoding="utf-8") as f:
        pending = ""
        for raw in f:
            line = raw.rstrip("\n")
            if pending:
                line = pending + line.lstrip()
                pending = ""
            s = line.strip()
            if not s or s[0] in "#!":
                continue
            if s.endswith("\\"):
                pending = s[:-1]
                continue
            m = re.match(r"([^=:\s]+)\s*[=:\s]\s*(.*)$", s)
            if m:
                props[m.group(1)] = m.group(2)
    return props


class PathConfiguration:
    """Path-prefix scoped overrides (reference conf/path/PrefixPathConfiguration.java)."""

    def __init__(self, path_props: dict[str, dict[str, str]] | None = None):
        self._lock = threading.RLock()
        self._props: dict[str, dict[str, str]] = dict(path_props or {})

    def set(self, path: str, props: dict[str, str]) -> None:
        with self._lock:
            self._props.setdefault(path, {}).update(props)

    def remove(self, path: str, keys=None) -> None:
        with self._lock:
            if keys is None:
                self._props.pop(path, None)
            else:
                d = self._props.get(path, {})
                for k in keys:
                    d.pop(k, None)
                if not d:
                    self._props.pop(path, None)

    def get_all(self) -> dict[str, dict[str, str]]:
        with self._lock:
            return {k: dict(v) for k, v in self._props.items()}

    def resolve(self, conf: Configuration, path: str) -> Configuration:
        """Configuration for ``path``: longest-prefix-last overlay at PATH_DEFAULT priority."""
        with self._lock:
            matches = sorted((p for p in self._props
                              if path == p or path.startswith(p.rstrip("/") + "/") or p == "/"),
                             key=len)
            out = conf.copy()
            for p in matches:
                for k, v in self._props[p].items():
                    out.set(k, v, Source.PATH_DEFAULT)
        return out

    def hash(self) -> str:
        with self._lock:
            s = repr(sorted((p, sorted(d.items())) for p, d in self._props.items()))
        return hashlib.md5(s.encode()).hexdigest()


_GLOBAL = None
_GLOBAL_LOCK = threading.Lock()


def global_conf() -> Configuration:
    """Process-wide configuration (site properties + env), like ``ServerConfiguration``."""
    global _GLOBAL
    with _GLOBAL_LOCK:
        if _GLOBAL is None:
            _GLOBAL = Configuration(load_site=True)
        return _GLOBAL


def reset_global() -> None:
    global _GLOBAL
    with _GLOBAL_LOCK:
        _GLOBAL = None
