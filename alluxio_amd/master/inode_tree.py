"""Inode tree: the namespace, its id generators and journal application.

Parity: core/server/master/src/main/java/alluxio/master/file/meta/InodeTree.java (root
initialisation ``initializeRoot`` :233, ``lockInodePath`` :375-436, ``createPath`` :670),
InodeTreePersistentState.java (every mutation is a journal entry applied through one code path,
for both live RPCs and replay), InodeDirectoryIdGenerator (directory ids = container id ||
sequence, containers drawn from the block master), TtlBucketList (TTL expiry buckets).

Concurrency: a tree-wide reader/writer lock.  Lookups (``getStatus``/``listStatus`` — the
metadata hot path) share it; mutations are serialised.  With CPython's GIL a finer-grained
per-inode lock scheme would add overhead without adding parallelism.
"""
from __future__ import annotations

import bisect
import threading

from ..proto import pb
from ..utils import ids
from ..utils.exceptions import (FileAlreadyExistsException, FileDoesNotExistException,
                                InvalidPathException)
from ..utils.locks import RWLock
from ..utils.uri import normalize_path, path_components
from .inode import NO_TTL, Inode, InodeDirectory, InodeFile, now_ms


class DirectoryIdGenerator:
    def __init__(self, container_source):
        self._source = container_source  # callable -> new container id
        self.container_id = -1
        self.sequence = ids.MAX_SEQUENCE_NUMBER + 1  # force a new container on first use
        self._lock = threading.Lock()

    def next_id(self) -> tuple[int, object | None]:
        """Returns (id, journal entry or None) — entry records a new container/sequence."""
        with self._lock:
            entry = None
            if self.sequence > ids.MAX_SEQUENCE_NUMBER - 1:
                self.container_id = self._source()
                self.sequence = 0
            did = ids.create_block_id(self.container_id, self.sequence)
            self.sequence += 1
            entry = pb.journal.JournalEntry(inode_directory_id_generator=pb.journal.InodeDirectoryIdGeneratorEntry(
                container_id=self.container_id, sequence_number=self.sequence))
            return did, entry

    def apply(self, e) -> None:
        with self._lock:
            self.container_id = e.container_id
            self.sequence = e.sequence_number


class TtlBuckets:
    """Inodes grouped by expiry interval (reference TtlBucketList: interval = check period)."""

    def __init__(self, interval_ms: int = 3_600_000):
        self.interval = max(1, interval_ms)
        self._buckets: dict[int, set[int]] = {}
        self._starts: list[int] = []
        self._of: dict[int, int] = {}     # inode id -> its bucket start
        self._lock = threading.Lock()

    def _start(self, expiry_ms: int) -> int:
        return expiry_ms - expiry_ms % self.interval

    def insert(self, inode: Inode) -> None:
        if inode.ttl == NO_TTL:
            return
        s = self._start(inode.creation_time_ms + inode.ttl)
        with self._lock:
            if s not in self._buckets:
                self._buckets[s] = set()
                bisect.insort(self._starts, s)
            self._buckets[s].add(inode.id)
            self._of[inode.id] = s

    def remove(self, inode: Inode) -> None:
        if inode.id not in self._of:      # GIL-atomic probe: most inodes have no TTL
            return
        with self._lock:
            s = self._of.pop(inode.id, None)
            b = self._buckets.get(s) if s is not None else None
            if b is not None:
                b.discard(inode.id)
                if not b:
                    del self._buckets[s]
                    self._starts.remove(s)

    def expired(self, now: int) -> list[int]:
        with self._lock:
            out = []
            for s in self._starts:
                if s + self.interval > now:
                    break
                out.extend(self._buckets[s])
            return out

    def clear(self) -> None:
        with self._lock:
            self._buckets.clear()
            self._starts.clear()
            self._of.clear()


class InodeTree:
    ROOT_NAME = ""

    def __init__(self, container_source, ttl_interval_ms: int = 3_600_000, store=None):
        from .metastore import HeapInodeStore
        self.lock = RWLock()
        self.inodes = store if store is not None else HeapInodeStore()   # InodeStore SPI (HEAP / ROCKS)
        self.children: dict[int, dict[str, int]] = {}
        self.root: InodeDirectory | None = None
        self.dir_ids = DirectoryIdGenerator(container_source)
        self.ttl_buckets = TtlBuckets(ttl_interval_ms)
        self.pinned_ids: set[int] = set()
        self.to_be_persisted: set[int] = set()
        self.replication_limited: set[int] = set()
        # bumped by every applied mutation: versions cached FileInfo replies (FileSystemMaster)
        self.epoch = 0
        self.epoch_listeners: list = []   # called after every bump (native reply cache)

    def _bump_epoch(self) -> None:
        self.epoch += 1
        for cb in self.epoch_listeners:
            cb()

    # ---- state ------------------------------------------------------------------------------
    def reset(self) -> None:
        self._bump_epoch()
        self.inodes.clear()
        self.children.clear()
        self.root = None
        self.ttl_buckets.clear()
        self.pinned_ids.clear()
        self.to_be_persisted.clear()
        self.replication_limited.clear()

    def _add(self, inode: Inode) -> None:
        self.inodes[inode.id] = inode
        if inode.is_directory:
            self.children.setdefault(inode.id, {})
        if inode.parent_id >= 0 and inode.parent_id in self.children and inode.name != self.ROOT_NAME:
            self.children[inode.parent_id][inode.name] = inode.id
        if inode.parent_id == -1 or (inode.is_directory and inode.name == self.ROOT_NAME and self.root is None):
            self.root = inode  # type: ignore[assignment]
        self._index(inode)

    def _index(self, inode: Inode) -> None:
        if inode.is_file and inode.replication_min > 0:
            inode.pinned = True           # a file that must keep copies is pinned (applyCreateInode)
        if inode.pinned:
            self.pinned_ids.add(inode.id)
        else:
            self.pinned_ids.discard(inode.id)
        self.ttl_buckets.remove(inode)
        self.ttl_buckets.insert(inode)
        if inode.is_file:
            if inode.persistence_state == "TO_BE_PERSISTED":
                self.to_be_persisted.add(inode.id)
            else:
                self.to_be_persisted.discard(inode.id)
            if inode.replication_max >= 0:      # InodeTreePersistentState: max != REPLICATION_MAX_INFINITY
                self.replication_limited.add(inode.id)
            else:
                self.replication_limited.discard(inode.id)

    def _remove(self, inode: Inode) -> None:
        self.inodes.pop(inode.id, None)
        kids = self.children.get(inode.parent_id)
        if kids is not None and kids.get(inode.name) == inode.id:
            del kids[inode.name]
        self.children.pop(inode.id, None)
        self.pinned_ids.discard(inode.id)
        self.to_be_persisted.discard(inode.id)
        self.replication_limited.discard(inode.id)
        self.ttl_buckets.remove(inode)
        inode.deleted = True

    # ---- journal application (single code path for replay and live ops) ---------------------
    def apply(self, e) -> bool:
        self.inodes.begin()
        try:
            return self._apply(e)
        finally:
            self._bump_epoch()
            self.inodes.end()

    def _apply(self, e) -> bool:
        # one C-level ListFields() instead of a HasField probe per entry type
        for fd, val in e.ListFields():
            h = _APPLY.get(fd.name)
            if h is not None:
                h(self, val)
                return True
        return False

    def _ap_inode_directory(self, v) -> None:
        self._add(InodeDirectory.from_entry(v))

    def _ap_inode_file(self, v) -> None:
        self._add(InodeFile.from_entry(v))

    def _ap_dir_ids(self, v) -> None:
        self.dir_ids.apply(v)

    def _ap_update_inode(self, u) -> None:
        inode = self.inodes.get(u.id)
        if inode is None:
            return
        old_parent, old_name = inode.parent_id, inode.name
        inode.update_from(u)
        if u.HasField("pinned") and inode.is_file:
            # InodeTreePersistentState.applyUpdateInode: pinning a file pins it to the listed media
            # (none listed = any medium) and raises replicationMin 0 -> 1; unpinning drops it to 0
            if u.pinned:
                inode.medium_types = list(u.medium_type)
                if inode.replication_min == 0:
                    inode.replication_min = 1
                    if inode.replication_max == 0:
                        inode.replication_max = -1
            else:
                inode.replication_min = 0
        if inode.parent_id != old_parent or inode.name != old_name:
            kids = self.children.get(old_parent)
            if kids is not None and kids.get(old_name) == inode.id:
                del kids[old_name]
            self.children.setdefault(inode.parent_id, {})[inode.name] = inode.id
        self._index(inode)

    def _ap_update_inode_directory(self, u) -> None:
        d = self.inodes.get(u.id)
        if d is not None and d.is_directory:
            if u.HasField("mount_point"):
                d.mount_point = u.mount_point
            if u.HasField("direct_children_loaded"):
                d.direct_children_loaded = u.direct_children_loaded
            if u.HasField("defaultAcl"):
                from ..security.acl import AccessControlList
                d.default_acl = AccessControlList.from_proto(u.defaultAcl)

    def _ap_update_inode_file(self, u) -> None:
        f = self.inodes.get(u.id)
        if f is not None and f.is_file:
            f.update_file_from(u)
            self._index(f)

    def _ap_delete_file(self, v) -> None:
        inode = self.inodes.get(v.id)
        if inode is not None:
            self._remove(inode)

    def _ap_rename(self, r) -> None:
        inode = self.inodes.get(r.id)
        if inode is None:
            return
        new_parent, new_name = r.new_parent_id, r.new_name
        if r.HasField("dst_path") and not r.HasField("new_parent_id"):
            # 1.x entries name the destination by path; resolve it against the tree as
            # replayed so far (InodeTreePersistentState.rewriteDeprecatedRenameEntry)
            parent_path, _, new_name = r.dst_path.rstrip("/").rpartition("/")
            new_parent = self.get(parent_path or "/").id
        kids = self.children.get(inode.parent_id)
        if kids is not None and kids.get(inode.name) == inode.id:
            del kids[inode.name]
        inode.parent_id = new_parent
        inode.name = new_name
        self.children.setdefault(new_parent, {})[new_name] = inode.id
        inode.last_modification_time_ms = r.op_time_ms or inode.last_modification_time_ms

    def _ap_set_acl(self, s) -> None:
        inode = self.inodes.get(s.id)
        if inode is not None:
            self._apply_set_acl(inode, s)

    def _ap_last_mod(self, v) -> None:
        inode = self.inodes.get(v.id)
        if inode is not None:
            inode.last_modification_time_ms = v.last_modification_time_ms

    def _ap_persist_directory(self, v) -> None:
        inode = self.inodes.get(v.id)
        if inode is not None:
            inode.persistence_state = "PERSISTED"

    def _ap_set_attribute(self, s) -> None:
        inode = self.inodes.get(s.id)
        if inode is None:
            return
        if s.HasField("pinned"):
            inode.pinned = s.pinned
        if s.HasField("ttl"):
            inode.ttl = s.ttl
        if s.HasField("persisted") and s.persisted:
            inode.persistence_state = "PERSISTED"
        if s.HasField("owner"):
            inode.owner = s.owner
        if s.HasField("group"):
            inode.group = s.group
        if s.HasField("permission"):
            inode.mode = s.permission
        self._index(inode)

    def _ap_complete_file(self, c) -> None:   # legacy form
        f = self.inodes.get(c.id)
        if f is not None and f.is_file:
            f.block_ids = list(c.block_ids)
            f.length = c.length
            f.completed = True
            f.last_modification_time_ms = c.op_time_ms

    def _ap_async_persist(self, v) -> None:
        f = self.inodes.get(v.file_id)
        if f is not None:
            f.persistence_state = "TO_BE_PERSISTED"
            self._index(f)

    @staticmethod
    def _apply_set_acl(inode: Inode, s) -> None:
        from ..security.acl import AccessControlList, AclEntry, AclEntryType
        entries = [AclEntry.from_proto(x) for x in s.entries]
        action = pb.journal.PSetAclAction.values_by_number[s.action].name
        acl = inode.acl or AccessControlList(inode.owner, inode.group, inode.mode)
        acl.mode = inode.mode
        dacl = getattr(inode, "default_acl", None)
        if action == "REMOVE_ALL":
            acl.clear_extended()
        elif action == "REMOVE_DEFAULT":
            if inode.is_directory:
                inode.default_acl = None
        for e in entries:
            target_default = e.is_default and inode.is_directory
            if target_default:
                if dacl is None:
                    dacl = AccessControlList(inode.owner, inode.group, inode.mode, is_default=True)
                    inode.default_acl = dacl
                tgt = dacl
            else:
                tgt = acl
            if action in ("REPLACE", "MODIFY"):
                tgt.set_entry(e)
            elif action == "REMOVE":
                tgt.remove_entry(e)
        if action == "REPLACE":
            keep_u = {e.subject for e in entries if e.type == AclEntryType.NAMED_USER and not e.is_default}
            keep_g = {e.subject for e in entries if e.type == AclEntryType.NAMED_GROUP and not e.is_default}
            acl.named_users = {k: v for k, v in acl.named_users.items() if k in keep_u}
            acl.named_groups = {k: v for k, v in acl.named_groups.items() if k in keep_g}
        inode.mode = acl.mode
        inode.acl = acl if acl.is_extended else None

    # ---- lookups ----------------------------------------------------------------------------
    def resolve(self, path: str) -> tuple[list[Inode], list[str]]:
        """Return (existing inode chain from root, remaining missing components)."""
        comps = path_components(path)
        chain: list[Inode] = [self.root]
        cur = self.root
        for i, c in enumerate(comps):
            if not cur.is_directory:
                raise InvalidPathException(f"{path}: {cur.name} is a file")
            cid = self.children.get(cur.id, {}).get(c)
            if cid is None:
                return chain, comps[i:]
            cur = self.inodes[cid]
            chain.append(cur)
        return chain, []

    def get(self, path: str) -> Inode:
        chain, missing = self.resolve(path)
        if missing:
            raise FileDoesNotExistException(f"Path \"{normalize_path(path)}\" does not exist.")
        return chain[-1]

    def get_or_none(self, path: str) -> Inode | None:
        try:
            chain, missing = self.resolve(path)
        except InvalidPathException:
            return None
        return None if missing else chain[-1]

    def exists(self, path: str) -> bool:
        return self.get_or_none(path) is not None

    def path_of(self, inode: Inode) -> str:
        parts = []
        cur = inode
        while cur is not None and cur.id != self.root.id:
            parts.append(cur.name)
            cur = self.inodes.get(cur.parent_id)
            if cur is None:
                raise FileDoesNotExistException(f"inode {inode.id} is detached")
        return "/" + "/".join(reversed(parts))

    def list_children(self, inode: Inode) -> list[Inode]:
        kids = self.children.get(inode.id, {})
        return [self.inodes[k] for _, k in sorted(kids.items())]

    def descendants(self, inode: Inode) -> list[Inode]:
        """Post-order (children before parent) list of all descendants, excluding ``inode``."""
        out = []
        stack = [(inode, False)]
        while stack:
            n, visited = stack.pop()
            if visited:
                if n is not inode:
                    out.append(n)
                continue
            stack.append((n, True))
            if n.is_directory:
                for c in self.list_children(n):
                    stack.append((c, False))
        return out

    # ---- entry builders (live path) ---------------------------------------------------------
    def new_directory_entries(self, parent: Inode, name: str, owner: str, group: str, mode: int,
                              persisted: bool, mount_point: bool = False, ttl: int = NO_TTL,
                              ttl_action: str = "DELETE"):
        did, gen_entry = self.dir_ids.next_id()
        d = InodeDirectory(did, parent.id if parent else -1, name, owner, group, mode, now_ms())
        d.persistence_state = "PERSISTED" if persisted else "NOT_PERSISTED"
        d.mount_point = mount_point
        d.ttl, d.ttl_action = ttl, ttl_action
        if parent is not None and getattr(parent, "default_acl", None) is not None:
            d.default_acl = parent.default_acl
        return [gen_entry, d.to_entry()]

    def new_file_entry(self, parent: Inode, name: str, file_id: int, owner: str, group: str, mode: int,
                       block_size: int, persisted_state: str, ttl: int = NO_TTL, ttl_action: str = "DELETE",
                       replication_min: int = 0, replication_max: int = -1, replication_durable: int = 1,
                       cacheable: bool = True):
        f = InodeFile(file_id, parent.id, name, owner, group, mode, now_ms(), block_size=block_size)
        f.persistence_state = persisted_state
        f.ttl, f.ttl_action = ttl, ttl_action
        f.replication_min, f.replication_max = replication_min, replication_max
        f.replication_durable = replication_durable
        f.cacheable = cacheable
        return f.to_entry()

    def check_no_conflict(self, parent: Inode, name: str) -> None:
        if name in self.children.get(parent.id, {}):
            raise FileAlreadyExistsException(f"{name} already exists under {self.path_of(parent)}")


# JournalEntry field -> InodeTree handler (the namespace entry types InodeTree.apply owns)
_APPLY = {
    "inode_directory": InodeTree._ap_inode_directory,
    "inode_file": InodeTree._ap_inode_file,
    "inode_directory_id_generator": InodeTree._ap_dir_ids,
    "update_inode": InodeTree._ap_update_inode,
    "update_inode_directory": InodeTree._ap_update_inode_directory,
    "update_inode_file": InodeTree._ap_update_inode_file,
    "delete_file": InodeTree._ap_delete_file,
    "rename": InodeTree._ap_rename,
    "set_acl": InodeTree._ap_set_acl,
    "inode_last_modification_time": InodeTree._ap_last_mod,
    "persist_directory": InodeTree._ap_persist_directory,
    "set_attribute": InodeTree._ap_set_attribute,
    "complete_file": InodeTree._ap_complete_file,
    "async_persist_request": InodeTree._ap_async_persist,
}
