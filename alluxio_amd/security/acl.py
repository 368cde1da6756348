"""POSIX mode bits and ACLs.

Parity: core/base/src/main/java/alluxio/security/authorization/{Mode,AclEntry,AccessControlList,
DefaultAccessControlList}.java — owner/group/other bits, named user/group entries, mask,
default ACLs inherited by children, ``checkPermission`` evaluation order (owner -> named user
-> owning/named groups (masked) -> other).
"""
from __future__ import annotations

import enum

from ..proto import pb


class Bits(enum.IntFlag):
    NONE = 0
    EXECUTE = 1
    WRITE = 2
    READ = 4
    ALL = 7


def bits_from_proto(v: int) -> int:
    # alluxio.grpc.Bits enum: NONE=1 EXECUTE=2 WRITE=3 WRITE_EXECUTE=4 READ=5 READ_EXECUTE=6 READ_WRITE=7 ALL=8
    return max(0, v - 1)


def bits_to_proto(b: int) -> int:
    return int(b) + 1


def mode_from_pmode(pm) -> int:
    return (bits_from_proto(pm.ownerBits) << 6) | (bits_from_proto(pm.groupBits) << 3) | \
        bits_from_proto(pm.otherBits)


def mode_to_pmode(mode: int):
    return pb.grpc.PMode(ownerBits=bits_to_proto((mode >> 6) & 7), groupBits=bits_to_proto((mode >> 3) & 7),
                         otherBits=bits_to_proto(mode & 7))


def apply_umask(mode: int, umask: int) -> int:
    return mode & ~umask & 0o777


def parse_umask(s: str) -> int:
    return int(str(s), 8)


class AclEntryType(enum.IntEnum):
    OWNER = 0
    NAMED_USER = 1
    OWNING_GROUP = 2
    NAMED_GROUP = 3
    MASK = 4
    OTHER = 5


class AclEntry:
    __slots__ = ("type", "subject", "actions", "is_default")

    def __init__(self, type: AclEntryType, subject: str, actions: int, is_default: bool = False):
        self.type, self.subject, self.actions, self.is_default = type, subject, actions, is_default

    @staticmethod
    def parse(s: str) -> "AclEntry":
        """``[default:]user:alice:rwx`` / ``group::r-x`` / ``mask::rw-`` / ``other::---``."""
        parts = s.strip().split(":")
        is_default = False
        if parts[0] == "default":
            is_default = True
            parts = parts[1:]
        kind, subject, perm = parts[0], parts[1] if len(parts) > 1 else "", parts[2] if len(parts) > 2 else ""
        bits = (Bits.READ if "r" in perm else 0) | (Bits.WRITE if "w" in perm else 0) | \
            (Bits.EXECUTE if "x" in perm else 0)
        t = {"user": AclEntryType.NAMED_USER if subject else AclEntryType.OWNER,
             "group": AclEntryType.NAMED_GROUP if subject else AclEntryType.OWNING_GROUP,
             "mask": AclEntryType.MASK, "other": AclEntryType.OTHER}[kind]
        return AclEntry(t, subject, int(bits), is_default)

    def to_cli(self) -> str:
        kind = {AclEntryType.OWNER: "user", AclEntryType.NAMED_USER: "user",
                AclEntryType.OWNING_GROUP: "group", AclEntryType.NAMED_GROUP: "group",
                AclEntryType.MASK: "mask", AclEntryType.OTHER: "other"}[self.type]
        p = ("r" if self.actions & 4 else "-") + ("w" if self.actions & 2 else "-") + ("x" if self.actions & 1 else "-")
        return ("default:" if self.is_default else "") + f"{kind}:{self.subject}:{p}"

    def to_proto(self):
        acts = [a for a, b in ((0, 4), (1, 2), (2, 1)) if self.actions & b]
        return pb.shared.AclEntry(type=int(self.type), subject=self.subject, actions=acts,
                                  isDefault=self.is_default)

    @staticmethod
    def from_proto(p) -> "AclEntry":
        bits = 0
        for a in p.actions:
            bits |= {0: 4, 1: 2, 2: 1}[a]
        return AclEntry(AclEntryType(p.type), p.subject, bits, p.isDefault)

    def to_pacl_entry(self):
        acts = [a for a, b in ((0, 4), (1, 2), (2, 1)) if self.actions & b]
        return pb.file.PAclEntry(type=int(self.type), subject=self.subject, actions=acts, isDefault=self.is_default)

    @staticmethod
    def from_pacl_entry(p) -> "AclEntry":
        bits = 0
        for a in p.actions:
            bits |= {0: 4, 1: 2, 2: 1}[a]
        return AclEntry(AclEntryType(p.type), p.subject, bits, p.isDefault)


class AccessControlList:
    def __init__(self, owner: str = "", group: str = "", mode: int = 0o755, is_default: bool = False):
        self.owner = owner
        self.group = group
        self.mode = mode
        self.named_users: dict[str, int] = {}
        self.named_groups: dict[str, int] = {}
        self.mask: int | None = None
        self.is_default = is_default

    @property
    def is_extended(self) -> bool:
        return bool(self.named_users or self.named_groups)

    def entries(self) -> list[AclEntry]:
        d = self.is_default
        out = [AclEntry(AclEntryType.OWNER, "", (self.mode >> 6) & 7, d)]
        out += [AclEntry(AclEntryType.NAMED_USER, u, a, d) for u, a in sorted(self.named_users.items())]
        out.append(AclEntry(AclEntryType.OWNING_GROUP, "", (self.mode >> 3) & 7, d))
        out += [AclEntry(AclEntryType.NAMED_GROUP, g, a, d) for g, a in sorted(self.named_groups.items())]
        if self.is_extended:
            out.append(AclEntry(AclEntryType.MASK, "", self.effective_mask(), d))
        out.append(AclEntry(AclEntryType.OTHER, "", self.mode & 7, d))
        return out

    def effective_mask(self) -> int:
        if self.mask is not None:
            return self.mask
        m = (self.mode >> 3) & 7
        for a in list(self.named_users.values()) + list(self.named_groups.values()):
            m |= a
        return m

    def set_entry(self, e: AclEntry) -> None:
        if e.type == AclEntryType.OWNER:
            self.mode = (self.mode & 0o077) | (e.actions << 6)
        elif e.type == AclEntryType.OWNING_GROUP:
            self.mode = (self.mode & 0o707) | (e.actions << 3)
        elif e.type == AclEntryType.OTHER:
            self.mode = (self.mode & 0o770) | e.actions
        elif e.type == AclEntryType.NAMED_USER:
            self.named_users[e.subject] = e.actions
        elif e.type == AclEntryType.NAMED_GROUP:
            self.named_groups[e.subject] = e.actions
        elif e.type == AclEntryType.MASK:
            self.mask = e.actions

    def remove_entry(self, e: AclEntry) -> None:
        if e.type == AclEntryType.NAMED_USER:
            self.named_users.pop(e.subject, None)
        elif e.type == AclEntryType.NAMED_GROUP:
            self.named_groups.pop(e.subject, None)
        elif e.type == AclEntryType.MASK:
            self.mask = None

    def clear_extended(self) -> None:
        self.named_users.clear()
        self.named_groups.clear()
        self.mask = None

    def permission(self, user: str, groups: list[str]) -> int:
        """Allowed bits for ``user`` (POSIX ACL evaluation order)."""
        if user == self.owner:
            return (self.mode >> 6) & 7
        mask = self.effective_mask() if self.is_extended else 7
        if user in self.named_users:
            return self.named_users[user] & mask
        matched = False
        allowed = 0
        if self.group in groups:
            matched = True
            allowed |= (self.mode >> 3) & 7
        for g in groups:
            if g in self.named_groups:
                matched = True
                allowed |= self.named_groups[g]
        if matched:
            return allowed & mask
        return self.mode & 7

    def to_proto(self):
        def named(d):
            out = []
            for name, a in sorted(d.items()):
                acts = [x for x, b in ((0, 4), (1, 2), (2, 1)) if a & b]
                out.append(pb.shared.NamedAclActions(name=name, actions=pb.shared.AclActions(actions=acts)))
            return out
        p = pb.shared.AccessControlList(owningUser=self.owner, owningGroup=self.group,
                                        userActions=named(self.named_users),
                                        groupActions=named(self.named_groups),
                                        isDefault=self.is_default, isEmpty=not self.is_extended)
        if self.mask is not None:
            p.maskActions.CopyFrom(pb.shared.AclActions(actions=[x for x, b in ((0, 4), (1, 2), (2, 1))
                                                                 if self.mask & b]))
        oth = self.mode & 7
        p.otherActions.CopyFrom(pb.shared.AclActions(actions=[x for x, b in ((0, 4), (1, 2), (2, 1)) if oth & b]))
        return p

    @staticmethod
    def from_proto(p) -> "AccessControlList":
        def bits(acts):
            v = 0
            for a in acts.actions:
                v |= {0: 4, 1: 2, 2: 1}[a]
            return v
        a = AccessControlList(p.owningUser, p.owningGroup, 0, p.isDefault)
        for n in p.userActions:
            a.named_users[n.name] = bits(n.actions)
        for n in p.groupActions:
            a.named_groups[n.name] = bits(n.actions)
        if p.HasField("maskActions"):
            a.mask = bits(p.maskActions)
        a.mode = bits(p.otherActions) if p.HasField("otherActions") else 0
        return a

    def to_pacl(self, mode: int):
        return pb.file.PAcl(owner=self.owner, owningGroup=self.group, mode=mode,
                            entries=[e.to_pacl_entry() for e in self.entries()],
                            isDefault=self.is_default, isDefaultEmpty=not self.is_extended)
