"""Users, groups, authentication and permission checking.

Parity: core/common/src/main/java/alluxio/security/{user,login,group}/ (login user from the OS or
``alluxio.security.login.username``; group mapping via the OS / a static map),
authentication/AuthType (NOSASL | SIMPLE | CUSTOM) and the master's DefaultPermissionChecker
(core/server/master/.../file/DefaultPermissionChecker.java: traverse = EXECUTE on every ancestor,
owner/superuser/supergroup shortcuts).
"""
from __future__ import annotations

import contextvars
import enum
import getpass
import grp
import os
import pwd
import threading
import time

from ..utils.exceptions import AccessControlException
from .acl import AccessControlList, Bits  # noqa: F401


class AuthType(enum.Enum):
    NOSASL = "NOSASL"
    SIMPLE = "SIMPLE"
    CUSTOM = "CUSTOM"


_current_user: contextvars.ContextVar[str | None] = contextvars.ContextVar("alluxio_user", default=None)


def login_user(conf=None) -> str:
    if conf is not None:
        u = conf.get_raw("alluxio.security.login.username")
        if u:
            return u
    return os.environ.get("ALLUXIO_USER") or getpass.getuser()


def current_user() -> str | None:
    return _current_user.get()


class as_user:
    """``with as_user('alice'): ...`` — sets the authenticated RPC user for this context."""

    def __init__(self, user: str | None):
        self.user = user

    def __enter__(self):
        self._tok = _current_user.set(self.user)
        return self

    def __exit__(self, *exc):
        _current_user.reset(self._tok)


class GroupMapping:
    """Unix shell-style group lookup with a TTL cache (CachedGroupMapping,
    ``alluxio.security.group.mapping.cache.timeout``, 1min): group lookups scan the whole group
    database, and every namespace mutation asks for the caller's primary group."""

    cache_ttl_s = 60.0
    _cache: dict = {}
    _cache_lock = threading.Lock()

    def groups(self, user: str) -> list[str]:
        now = time.monotonic()
        key = (type(self), user)
        hit = GroupMapping._cache.get(key)
        if hit is not None and now - hit[0] < self.cache_ttl_s:
            return list(hit[1])
        out = self._lookup(user)
        with GroupMapping._cache_lock:
            GroupMapping._cache[key] = (now, tuple(out))
        return out

    def _lookup(self, user: str) -> list[str]:
        out = []
        try:
            pw = pwd.getpwnam(user)
            out.append(grp.getgrgid(pw.pw_gid).gr_name)
        except KeyError:
            pass
        try:
            for g in grp.getgrall():
                if user in g.gr_mem and g.gr_name not in out:
                    out.append(g.gr_name)
        except Exception:  # noqa: BLE001
            pass
        return out


class StaticGroupMapping(GroupMapping):
    def __init__(self, mapping: dict[str, list[str]]):
        self.mapping = mapping

    def groups(self, user: str) -> list[str]:
        return list(self.mapping.get(user, []))


def primary_group(user: str, mapping: GroupMapping | None = None) -> str:
    g = (mapping or GroupMapping()).groups(user)
    return g[0] if g else user


class PermissionChecker:
    def __init__(self, enabled: bool = True, superuser: str | None = None, supergroup: str = "supergroup",
                 group_mapping: GroupMapping | None = None):
        self.enabled = enabled
        self.superuser = superuser or getpass.getuser()
        self.supergroup = supergroup
        self.groups = group_mapping or GroupMapping()

    def _is_privileged(self, user, groups) -> bool:
        return user == self.superuser or self.supergroup in groups

    def check(self, user: str | None, inodes: list, bits: int, path: str = "") -> None:
        """``inodes`` = resolved chain root..target (target may be missing for creates)."""
        if not self.enabled or user is None:
            return
        groups = self.groups.groups(user)
        if self._is_privileged(user, groups):
            return
        for anc in inodes[:-1]:
            if not self._allowed(anc, user, groups, Bits.EXECUTE):
                raise AccessControlException(f"Permission denied: user={user}, access=--x, path={path}: "
                                             f"failed at {anc.name or '/'}")
        if inodes and not self._allowed(inodes[-1], user, groups, bits):
            p = ("r" if bits & 4 else "-") + ("w" if bits & 2 else "-") + ("x" if bits & 1 else "-")
            raise AccessControlException(f"Permission denied: user={user}, access={p}, path={path}")

    def check_owner(self, user: str | None, inode, path: str = "") -> None:
        if not self.enabled or user is None:
            return
        groups = self.groups.groups(user)
        if self._is_privileged(user, groups) or inode.owner == user:
            return
        raise AccessControlException(f"Permission denied: user={user} is not the owner of {path}")

    def check_superuser(self, user: str | None) -> None:
        if not self.enabled or user is None:
            return
        if not self._is_privileged(user, self.groups.groups(user)):
            raise AccessControlException(f"Permission denied: user={user} is not a superuser")

    @staticmethod
    def _allowed(inode, user, groups, bits) -> bool:
        if inode.acl is not None and inode.acl.is_extended:
            acl = inode.acl
            acl.owner, acl.group, acl.mode = inode.owner, inode.group, (acl.mode & 0o777) | 0
            perm = AccessControlList(inode.owner, inode.group, inode.mode)
            perm.named_users, perm.named_groups, perm.mask = acl.named_users, acl.named_groups, acl.mask
            return (perm.permission(user, groups) & bits) == bits
        if user == inode.owner:
            allowed = (inode.mode >> 6) & 7
        elif inode.group in groups:
            allowed = (inode.mode >> 3) & 7
        else:
            allowed = inode.mode & 7
        return (allowed & bits) == bits
