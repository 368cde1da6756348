"""Inodes (files and directories) and their journal/wire encodings.

Parity: core/server/master/src/main/java/alluxio/master/file/meta/MutableInode{,File,Directory}.java
(fields, ``toJournalEntry``, ``fromJournalEntry``, ``updateFromEntry``) and the ``FileInfo``
generation in DefaultFileSystemMaster.getFileInfoInternal (DefaultFileSystemMaster.java:818-891).
"""
from __future__ import annotations

import time

from ..proto import pb
from ..utils import ids

NO_TTL = -1
UNKNOWN_SIZE = -1

PERSISTED = "PERSISTED"
NOT_PERSISTED = "NOT_PERSISTED"
TO_BE_PERSISTED = "TO_BE_PERSISTED"
LOST = "LOST"


# enum name <-> number of PTtlAction (dict lookups: descriptor ``values_by_*`` are slow per call)
_PTTL_NUM = {v.name: v.number for v in pb.journal.PTtlAction.values}
_PTTL_NAME = {v.number: v.name for v in pb.journal.PTtlAction.values}


def now_ms() -> int:
    return int(time.time() * 1000)


class Inode:
    is_directory = False

    def __init__(self, id: int, parent_id: int, name: str, owner: str = "", group: str = "",
                 mode: int = 0o755, creation_ms: int | None = None):
        self.id = id
        self.parent_id = parent_id
        self.name = name
        self.owner = owner
        self.group = group
        self.mode = mode
        self.creation_time_ms = creation_ms if creation_ms is not None else now_ms()
        self.last_modification_time_ms = self.creation_time_ms
        self.last_access_time_ms = self.creation_time_ms
        self.persistence_state = NOT_PERSISTED
        self.pinned = False
        self.ttl = NO_TTL
        self.ttl_action = "DELETE"
        self.ufs_fingerprint = ""
        self.xattr: dict[str, bytes] = {}
        self.medium_types: list[str] = []
        self.acl = None           # alluxio_amd.security.acl.AccessControlList | None
        self.deleted = False

    @property
    def is_file(self) -> bool:
        return not self.is_directory

    @property
    def is_persisted(self) -> bool:
        return self.persistence_state == PERSISTED

    def update_from(self, e) -> None:
        """Apply an UpdateInodeEntry (reference MutableInode.updateFromEntry)."""
        if e.HasField("parent_id"):
            self.parent_id = e.parent_id
        if e.HasField("name"):
            self.name = e.name
        if e.HasField("persistence_state"):
            self.persistence_state = e.persistence_state
        if e.HasField("pinned"):
            self.pinned = e.pinned
        if e.HasField("creation_time_ms"):
            self.creation_time_ms = e.creation_time_ms
        if e.HasField("last_modification_time_ms"):
            if e.overwrite_modification_time:
                self.last_modification_time_ms = e.last_modification_time_ms
            else:
                self.last_modification_time_ms = max(self.last_modification_time_ms,
                                                     e.last_modification_time_ms)
        if e.HasField("last_access_time_ms"):
            if e.overwrite_access_time:
                self.last_access_time_ms = e.last_access_time_ms
            else:
                self.last_access_time_ms = max(self.last_access_time_ms, e.last_access_time_ms)
        if e.HasField("owner"):
            self.owner = e.owner
        if e.HasField("group"):
            self.group = e.group
        if e.HasField("mode"):
            self.mode = e.mode
        if e.HasField("ttl"):
            self.ttl = e.ttl
        if e.HasField("ttlAction"):
            self.ttl_action = _PTTL_NAME[e.ttlAction]
        if e.HasField("ufs_fingerprint"):
            self.ufs_fingerprint = e.ufs_fingerprint
        if e.medium_type:
            self.medium_types = list(e.medium_type)
        if e.xAttr:
            self.xattr.update(dict(e.xAttr))


class InodeDirectory(Inode):
    is_directory = True

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.mount_point = False
        self.direct_children_loaded = False
        self.default_acl = None

    def to_entry(self, path: str = ""):
        e = pb.journal.InodeDirectoryEntry(
            id=self.id, parent_id=self.parent_id, name=self.name,
            persistence_state=self.persistence_state, pinned=self.pinned,
            creation_time_ms=self.creation_time_ms,
            last_modification_time_ms=self.last_modification_time_ms, owner=self.owner,
            group=self.group, mode=self.mode, mount_point=self.mount_point,
            direct_children_loaded=self.direct_children_loaded, ttl=self.ttl,
            ttlAction=_PTTL_NUM[self.ttl_action],
            last_access_time_ms=self.last_access_time_ms, medium_type=self.medium_types)
        if path:
            e.path = path
        for k, v in self.xattr.items():
            e.xAttr[k] = v
        if self.acl is not None:
            e.acl.CopyFrom(self.acl.to_proto())
        if self.default_acl is not None:
            e.defaultAcl.CopyFrom(self.default_acl.to_proto())
        return pb.journal.JournalEntry(inode_directory=e)

    @staticmethod
    def from_entry(e) -> "InodeDirectory":
        d = InodeDirectory(e.id, e.parent_id, e.name, e.owner, e.group, e.mode, e.creation_time_ms)
        d.persistence_state = e.persistence_state or NOT_PERSISTED
        d.pinned = e.pinned
        d.last_modification_time_ms = e.last_modification_time_ms
        d.last_access_time_ms = e.last_access_time_ms or e.last_modification_time_ms
        d.mount_point = e.mount_point
        d.direct_children_loaded = e.direct_children_loaded
        d.ttl = e.ttl if e.HasField("ttl") else NO_TTL
        d.ttl_action = _PTTL_NAME[e.ttlAction]
        d.xattr = dict(e.xAttr)
        d.medium_types = list(e.medium_type)
        if e.HasField("acl"):
            from ..security.acl import AccessControlList
            d.acl = AccessControlList.from_proto(e.acl)
        if e.HasField("defaultAcl"):
            from ..security.acl import AccessControlList
            d.default_acl = AccessControlList.from_proto(e.defaultAcl)
        return d


class InodeFile(Inode):
    def __init__(self, *a, block_size: int = 64 << 20, **kw):
        super().__init__(*a, **kw)
        self.block_size_bytes = block_size
        self.length = 0
        self.completed = False
        self.cacheable = True
        self.block_ids: list[int] = []
        self.replication_min = 0
        self.replication_max = -1
        self.replication_durable = 1
        self.persist_job_id = -1
        self.temp_ufs_path = ""
        self.should_persist_time = 0
        self._next_seq = 0

    @property
    def block_container_id(self) -> int:
        return ids.get_container_id(self.id)

    def new_block_id(self) -> int:
        bid = ids.create_block_id(self.block_container_id, self._next_seq)
        self._next_seq += 1
        return bid

    def to_entry(self, path: str = ""):
        e = pb.journal.InodeFileEntry(
            id=self.id, parent_id=self.parent_id, name=self.name,
            persistence_state=self.persistence_state, pinned=self.pinned,
            creation_time_ms=self.creation_time_ms,
            last_modification_time_ms=self.last_modification_time_ms,
            block_size_bytes=self.block_size_bytes, length=self.length, completed=self.completed,
            cacheable=self.cacheable, blocks=self.block_ids, ttl=self.ttl, owner=self.owner,
            group=self.group, mode=self.mode,
            ttlAction=_PTTL_NUM[self.ttl_action],
            ufs_fingerprint=self.ufs_fingerprint, replication_max=self.replication_max,
            replication_min=self.replication_min, persist_job_id=self.persist_job_id,
            temp_ufs_path=self.temp_ufs_path, replication_durable=self.replication_durable,
            medium_type=self.medium_types, should_persist_time=self.should_persist_time,
            last_access_time_ms=self.last_access_time_ms)
        if path:
            e.path = path
        for k, v in self.xattr.items():
            e.xAttr[k] = v
        if self.acl is not None:
            e.acl.CopyFrom(self.acl.to_proto())
        return pb.journal.JournalEntry(inode_file=e)

    @staticmethod
    def from_entry(e) -> "InodeFile":
        f = InodeFile(e.id, e.parent_id, e.name, e.owner, e.group, e.mode, e.creation_time_ms,
                      block_size=e.block_size_bytes)
        f.persistence_state = e.persistence_state or NOT_PERSISTED
        f.pinned = e.pinned
        f.last_modification_time_ms = e.last_modification_time_ms
        f.last_access_time_ms = e.last_access_time_ms or e.last_modification_time_ms
        f.length = e.length
        f.completed = e.completed
        f.cacheable = e.cacheable
        f.block_ids = list(e.blocks)
        f._next_seq = len(f.block_ids)
        f.ttl = e.ttl if e.HasField("ttl") else NO_TTL
        f.ttl_action = _PTTL_NAME[e.ttlAction]
        f.ufs_fingerprint = e.ufs_fingerprint
        f.replication_max = e.replication_max if e.HasField("replication_max") else -1
        f.replication_min = e.replication_min
        f.replication_durable = e.replication_durable if e.HasField("replication_durable") else 1
        f.persist_job_id = e.persist_job_id if e.HasField("persist_job_id") else -1
        f.temp_ufs_path = e.temp_ufs_path
        f.should_persist_time = e.should_persist_time
        f.xattr = dict(e.xAttr)
        f.medium_types = list(e.medium_type)
        if e.HasField("acl"):
            from ..security.acl import AccessControlList
            f.acl = AccessControlList.from_proto(e.acl)
        return f

    def update_file_from(self, e) -> None:
        """Apply an UpdateInodeFileEntry."""
        if e.HasField("block_size_bytes"):
            self.block_size_bytes = e.block_size_bytes
        if e.HasField("length"):
            self.length = e.length
        if e.HasField("completed"):
            self.completed = e.completed
        if e.HasField("cacheable"):
            self.cacheable = e.cacheable
        if e.set_blocks:
            self.block_ids = list(e.set_blocks)
            self._next_seq = max(self._next_seq, len(self.block_ids))
        if e.HasField("replication_max"):
            self.replication_max = e.replication_max
        if e.HasField("replication_min"):
            self.replication_min = e.replication_min
        if e.HasField("persist_job_id"):
            self.persist_job_id = e.persist_job_id
        if e.HasField("temp_ufs_path"):
            self.temp_ufs_path = e.temp_ufs_path


# ---- InodeMeta.Inode (checkpoint / metastore encoding) ----------------------------------------
# Reference MutableInode.toProtoBuilder (MutableInode.java:657-677), MutableInodeFile.toProto
# (:504-517) / fromProto (:523-550), MutableInodeDirectory.toProto (:278-285) / fromProto
# (:291-313).  Owner/group/mode travel inside ``access_acl`` (ProtoUtils.toProto(AccessControlList),
# ProtoUtils.java:93-125): the owning user's and group's actions are the NamedAclActions whose name
# is "" (AccessControlList.OWNING_USER_KEY / OWNING_GROUP_KEY), the other bits are otherActions.
def _actions(bits: int):
    return pb.shared.AclActions(actions=[a for a, b in ((0, 4), (1, 2), (2, 1)) if bits & b])


def _bits(acts) -> int:
    v = 0
    for a in acts.actions:
        v |= {0: 4, 1: 2, 2: 1}[a]
    return v


def acl_to_proto(owner: str, group: str, mode: int, acl=None, is_default: bool = False, empty: bool = False):
    p = pb.shared.AccessControlList(owningUser=owner, owningGroup=group, isDefault=is_default, isEmpty=empty)
    p.userActions.add(name="", actions=_actions((mode >> 6) & 7))
    p.groupActions.add(name="", actions=_actions((mode >> 3) & 7))
    p.otherActions.CopyFrom(_actions(mode & 7))
    if acl is not None and acl.is_extended:
        for u, a in sorted(acl.named_users.items()):
            p.userActions.add(name=u, actions=_actions(a))
        for g, a in sorted(acl.named_groups.items()):
            p.groupActions.add(name=g, actions=_actions(a))
        p.maskActions.CopyFrom(_actions(acl.effective_mask()))
    return p


def acl_from_proto(p):
    """(owner, group, mode, extended AccessControlList | None, is_empty)."""
    from ..security.acl import AccessControlList
    mode = _bits(p.otherActions) if p.HasField("otherActions") else 0
    ext = AccessControlList(p.owningUser, p.owningGroup, 0, p.isDefault)
    for n in p.userActions:
        if n.name == "":
            mode |= _bits(n.actions) << 6
        else:
            ext.named_users[n.name] = _bits(n.actions)
    for n in p.groupActions:
        if n.name == "":
            mode |= _bits(n.actions) << 3
        else:
            ext.named_groups[n.name] = _bits(n.actions)
    if p.HasField("maskActions") and ext.is_extended:
        ext.mask = _bits(p.maskActions)
    ext.mode = mode
    return p.owningUser, p.owningGroup, mode, (ext if ext.is_extended else None), p.isEmpty


_TTL_ACTION = {"DELETE": 0, "FREE": 1}
_TTL_ACTION_BACK = {0: "DELETE", 1: "FREE"}


def inode_to_proto(n: Inode, child_count: int = 0):
    p = pb.metastore.Inode(
        id=n.id, creation_time_ms=n.creation_time_ms, is_directory=n.is_directory, ttl=n.ttl,
        ttl_action=_TTL_ACTION.get(n.ttl_action, 0), last_modified_ms=n.last_modification_time_ms,
        last_accessed_ms=n.last_access_time_ms, name=n.name, parent_id=n.parent_id,
        persistence_state=n.persistence_state, is_pinned=n.pinned,
        access_acl=acl_to_proto(n.owner, n.group, n.mode, n.acl), ufs_fingerprint=n.ufs_fingerprint,
        medium_type=n.medium_types)
    for k, v in n.xattr.items():
        p.xAttr[k] = v
    if n.is_directory:
        p.is_mount_point = n.mount_point
        p.has_direct_children_loaded = n.direct_children_loaded
        p.child_count = child_count
        d = n.default_acl
        if d is None:     # DefaultAccessControlList(accessAcl): the access ACL's base, empty
            p.default_acl.CopyFrom(acl_to_proto(n.owner, n.group, n.mode, None, True, True))
        else:
            p.default_acl.CopyFrom(acl_to_proto(d.owner or n.owner, d.group or n.group, d.mode, d, True,
                                                not d.is_extended and d.mode == 0))
    else:
        p.block_size_bytes = n.block_size_bytes
        p.blocks.extend(n.block_ids)
        p.is_cacheable = n.cacheable
        p.is_completed = n.completed
        p.length = n.length
        p.replication_durable = n.replication_durable
        p.replication_max = n.replication_max
        p.replication_min = n.replication_min
        p.persist_job_id = n.persist_job_id
        p.persist_job_temp_ufs_path = n.temp_ufs_path
        if n.should_persist_time:
            p.should_persist_time = n.should_persist_time
    return p


def inode_from_proto(p) -> Inode:
    owner, group, mode, ext, _empty = acl_from_proto(p.access_acl)
    if p.is_directory:
        n = InodeDirectory(p.id, p.parent_id, p.name, owner, group, mode, p.creation_time_ms)
        n.mount_point = p.is_mount_point
        n.direct_children_loaded = p.has_direct_children_loaded
        if p.HasField("default_acl") and not p.default_acl.isEmpty:
            _o, _g, dmode, dext, _e = acl_from_proto(p.default_acl)
            from ..security.acl import AccessControlList
            d = dext or AccessControlList(owner, group, dmode, True)
            d.mode, d.is_default = dmode, True
            n.default_acl = d
    else:
        n = InodeFile(p.id, p.parent_id, p.name, owner, group, mode, p.creation_time_ms,
                      block_size=p.block_size_bytes)
        n.block_ids = list(p.blocks)
        n._next_seq = len(n.block_ids)
        n.cacheable = p.is_cacheable
        n.completed = p.is_completed
        n.length = p.length
        n.replication_durable = p.replication_durable if p.HasField("replication_durable") else 1
        n.replication_max = p.replication_max if p.HasField("replication_max") else -1
        n.replication_min = p.replication_min
        n.persist_job_id = p.persist_job_id if p.HasField("persist_job_id") else -1
        n.temp_ufs_path = p.persist_job_temp_ufs_path
        n.should_persist_time = p.should_persist_time
    n.last_modification_time_ms = p.last_modified_ms
    n.last_access_time_ms = p.last_accessed_ms or p.last_modified_ms
    n.ttl = p.ttl if p.HasField("ttl") else NO_TTL
    n.ttl_action = _TTL_ACTION_BACK.get(p.ttl_action, "DELETE")
    n.persistence_state = p.persistence_state or NOT_PERSISTED
    n.pinned = p.is_pinned
    n.ufs_fingerprint = p.ufs_fingerprint
    n.medium_types = list(p.medium_type)
    n.xattr = dict(p.xAttr)
    if ext is not None:
        ext.mode = mode
        n.acl = ext
    return n

