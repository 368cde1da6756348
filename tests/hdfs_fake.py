"""A one-process mini HDFS (NameNode + DataNodes) serving the Hadoop wire protocols that
``alluxio_amd.underfs.hadoop_rpc`` speaks: Hadoop IPC v9 ClientNamenodeProtocol calls and
DataTransferProtocol READ_BLOCK / WRITE_BLOCK with CRC32C packets and pipeline forwarding.

It is the test double for the HDFS UFS (the reference tests its HDFS UFS against MiniDFSCluster;
no JVM here).  Semantics follow FSNamesystem where the UFS contract observes them: create with
overwrite/createParent, FileAlreadyExistsException, mkdirs with createParent, non-recursive
delete of a non-empty directory -> PathIsNotEmptyDirectoryException, rename returning false when
the destination exists or the source is missing, paged getListing (``ls_limit`` entries a page).
"""
from __future__ import annotations

import threading
import time

from alluxio_amd.proxy.hdfs_gateway import DataTransferServer, IpcServer
from alluxio_amd.proxy.hdfs_gateway import RpcError as _Remote
from alluxio_amd.underfs import hadoop_rpc as H

common, hdfs = H.common, H.hdfs


def _fnf(p):
    return _Remote("java.io.FileNotFoundException", f"File does not exist: {p}")


class Node:
    def __init__(self, is_dir, mode, owner, group, block_size=0, replication=0):
        self.is_dir, self.mode, self.owner, self.group = is_dir, mode, owner, group
        self.mtime = int(time.time() * 1000)
        self.blocks: list = []          # ExtendedBlockProto (numBytes committed)
        self.block_size, self.replication = block_size, replication
        self.complete = is_dir
        self.file_id = 0
        self.acl: list = []             # extended + default AclEntryProto (HDFS AclFeature)


class MiniDfs:
    def __init__(self, num_datanodes=1, ls_limit=1000, owner="hdfs", group="supergroup"):
        self.lock = threading.RLock()
        self.ns: dict[str, Node] = {"/": Node(True, 0o755, owner, group)}
        self.ls_limit = ls_limit
        self.next_block = 1 << 30
        self.next_file_id = 16386
        self.pool_id = "BP-1-127.0.0.1-1"
        self.datanodes = [_DataNode(self, i) for i in range(num_datanodes)]
        self.namenode = IpcServer(self.handle)
        self.port = self.namenode.port
        self.calls: list[str] = []
        self.edits: list = []           # inotify: EventBatchProto per edit, txid = index + 1

    def _event(self, etype, msg):
        b = hdfs.EventBatchProto(txid=len(self.edits) + 1)
        b.events.add(type=etype, contents=msg.SerializeToString())
        self.edits.append(b)

    def stop(self):
        self.namenode.stop()
        for d in self.datanodes:
            d.stop()

    # ---- namespace helpers ------------------------------------------------------------------
    @staticmethod
    def _norm(p):
        p = "/" + p.strip("/")
        return p

    @staticmethod
    def _parent(p):
        return p.rsplit("/", 1)[0] or "/"

    def _children(self, p):
        pre = p.rstrip("/") + "/"
        return sorted(k for k in self.ns if k.startswith(pre) and "/" not in k[len(pre):] and k != "/")

    def _status(self, p, n: Node, name: bytes):
        st = hdfs.HdfsFileStatusProto(fileType=H.FILE_IS_DIR if n.is_dir else H.FILE_IS_FILE, path=name,
                                      length=0 if n.is_dir else sum(b.numBytes for b in n.blocks),
                                      owner=n.owner, group=n.group, modification_time=n.mtime,
                                      access_time=n.mtime, block_replication=n.replication,
                                      blocksize=n.block_size, fileId=n.file_id,
                                      childrenNum=len(self._children(p)) if n.is_dir else 0)
        st.permission.perm = n.mode
        return st

    def _mkdirs(self, p, mode, owner):
        parts = [x for x in p.split("/") if x]
        cur = ""
        for x in parts:
            cur += "/" + x
            n = self.ns.get(cur)
            if n is None:
                self.ns[cur] = Node(True, mode, owner, "supergroup")
            elif not n.is_dir:
                raise _Remote("org.apache.hadoop.fs.ParentNotDirectoryException", f"{cur} is not a directory")

    def _located(self, eb, offset, dns):
        lb = hdfs.LocatedBlockProto(offset=offset, corrupt=False)
        lb.b.CopyFrom(eb)
        lb.blockToken.CopyFrom(common.TokenProto(identifier=b"", password=b"", kind="", service=""))
        for dn in dns:
            lb.locs.add().CopyFrom(dn.info())
        return lb

    # ---- ClientProtocol -----------------------------------------------------------------------
    def handle(self, method, req_bytes, user):
        self.calls.append(method)
        with self.lock:
            fn = getattr(self, "rpc_" + method, None)
            if fn is None:
                raise _Remote("org.apache.hadoop.ipc.RpcNoSuchMethodException", f"Unknown method {method}")
            return fn(req_bytes, user)

    def rpc_getFileInfo(self, b, user):
        r = hdfs.GetFileInfoRequestProto.FromString(b)
        p = self._norm(r.src)
        out = hdfs.GetFileInfoResponseProto()
        n = self.ns.get(p)
        if n is not None:
            out.fs.CopyFrom(self._status(p, n, b""))
        return out

    def rpc_getListing(self, b, user):
        r = hdfs.GetListingRequestProto.FromString(b)
        p = self._norm(r.src)
        out = hdfs.GetListingResponseProto()
        n = self.ns.get(p)
        if n is None:
            return out
        if not n.is_dir:
            out.dirList.partialListing.add().CopyFrom(self._status(p, n, b""))
            out.dirList.remainingEntries = 0
            return out
        names = [c.rsplit("/", 1)[1] for c in self._children(p)]
        after = r.startAfter.decode()
        names = [x for x in names if x > after]
        page, rest = names[:self.ls_limit], names[self.ls_limit:]
        for x in page:
            c = p.rstrip("/") + "/" + x
            out.dirList.partialListing.add().CopyFrom(self._status(c, self.ns[c], x.encode()))
        out.dirList.remainingEntries = len(rest)
        return out

    def rpc_mkdirs(self, b, user):
        r = hdfs.MkdirsRequestProto.FromString(b)
        p = self._norm(r.src)
        n = self.ns.get(p)
        if n is not None:
            if not n.is_dir:
                raise _Remote("org.apache.hadoop.fs.FileAlreadyExistsException", f"{p} is a file")
            return hdfs.MkdirsResponseProto(result=True)
        par = self.ns.get(self._parent(p))
        if par is None and not r.createParent:
            raise _fnf(self._parent(p))
        if par is not None and not par.is_dir:
            raise _Remote("org.apache.hadoop.fs.ParentNotDirectoryException", f"{self._parent(p)}")
        self._mkdirs(p, r.masked.perm, user)
        self._event(0, hdfs.CreateEventProto(type=1, path=p, ctime=0, ownerName=user, groupName="supergroup",
                                             perms=r.masked))
        return hdfs.MkdirsResponseProto(result=True)

    def _subtree(self, p):
        pre = p.rstrip("/") + "/"
        return [k for k in self.ns if k == p or k.startswith(pre)]

    def rpc_delete(self, b, user):
        r = hdfs.DeleteRequestProto.FromString(b)
        p = self._norm(r.src)
        n = self.ns.get(p)
        if n is None or p == "/":
            return hdfs.DeleteResponseProto(result=False)
        if n.is_dir and not r.recursive and self._children(p):
            raise _Remote("org.apache.hadoop.fs.PathIsNotEmptyDirectoryException", f"{p} is non empty")
        for k in self._subtree(p):
            for eb in self.ns[k].blocks:
                for dn in self.datanodes:
                    dn.blocks.pop(eb.blockId, None)
            del self.ns[k]
        self._event(5, hdfs.UnlinkEventProto(path=p, timestamp=0))
        return hdfs.DeleteResponseProto(result=True)

    def rpc_rename(self, b, user):
        r = hdfs.RenameRequestProto.FromString(b)
        src, dst = self._norm(r.src), self._norm(r.dst)
        if src not in self.ns or dst in self.ns or self._parent(dst) not in self.ns \
                or dst.startswith(src.rstrip("/") + "/"):
            return hdfs.RenameResponseProto(result=False)
        for k in sorted(self._subtree(src)):
            self.ns[dst + k[len(src):]] = self.ns.pop(k)
        self._event(3, hdfs.RenameEventProto(srcPath=src, destPath=dst, timestamp=0))
        return hdfs.RenameResponseProto(result=True)

    def rpc_create(self, b, user):
        r = hdfs.CreateRequestProto.FromString(b)
        p = self._norm(r.src)
        n = self.ns.get(p)
        if n is not None:
            if n.is_dir:
                raise _Remote("org.apache.hadoop.fs.FileAlreadyExistsException", f"{p} already exists as a directory")
            if not r.createFlag & H.CREATE_FLAG_OVERWRITE:
                raise _Remote("org.apache.hadoop.fs.FileAlreadyExistsException", f"{p} for client already exists")
        par = self.ns.get(self._parent(p))
        if par is None:
            if not r.createParent:
                raise _fnf(self._parent(p))
            self._mkdirs(self._parent(p), 0o755, user)
        elif not par.is_dir:
            raise _Remote("org.apache.hadoop.fs.ParentNotDirectoryException", self._parent(p))
        node = Node(False, r.masked.perm, user, "supergroup", r.blockSize, r.replication)
        node.file_id = self.next_file_id
        self.next_file_id += 1
        self.ns[p] = node
        self._event(0, hdfs.CreateEventProto(type=0, path=p, ctime=0, ownerName=user, groupName="supergroup",
                                             perms=r.masked, overwrite=bool(r.createFlag & 2)))
        return hdfs.CreateResponseProto(fs=self._status(p, node, b""))

    def _file(self, src, file_id):
        p = self._norm(src)
        n = self.ns.get(p)
        if n is None or n.is_dir or (file_id and n.file_id != file_id):
            raise _Remote("org.apache.hadoop.hdfs.server.namenode.LeaseExpiredException", f"No lease on {p}")
        return n

    def _commit(self, n, eb):
        for i, x in enumerate(n.blocks):
            if x.blockId == eb.blockId:
                n.blocks[i].numBytes = eb.numBytes
                return

    def rpc_addBlock(self, b, user):
        r = hdfs.AddBlockRequestProto.FromString(b)
        n = self._file(r.src, r.fileId)
        if r.HasField("previous"):
            self._commit(n, r.previous)
        eb = hdfs.ExtendedBlockProto(poolId=self.pool_id, blockId=self.next_block, generationStamp=1001, numBytes=0)
        self.next_block += 1
        offset = sum(x.numBytes for x in n.blocks)
        n.blocks.append(eb)
        k = max(1, min(n.replication or 1, len(self.datanodes)))
        return hdfs.AddBlockResponseProto(block=self._located(eb, offset, self.datanodes[:k]))

    def rpc_abandonBlock(self, b, user):
        r = hdfs.AbandonBlockRequestProto.FromString(b)
        n = self._file(r.src, r.fileId)
        n.blocks = [x for x in n.blocks if x.blockId != r.b.blockId]
        return hdfs.AbandonBlockResponseProto()

    def rpc_complete(self, b, user):
        r = hdfs.CompleteRequestProto.FromString(b)
        n = self._file(r.src, r.fileId)
        if r.HasField("last"):
            self._commit(n, r.last)
        for eb in n.blocks:                       # every replica must have reported the block
            if any(dn.blocks.get(eb.blockId) is None or len(dn.blocks[eb.blockId]) != eb.numBytes
                   for dn in self.datanodes[:max(1, min(n.replication or 1, len(self.datanodes)))]):
                return hdfs.CompleteResponseProto(result=False)
        n.complete = True
        n.mtime = int(time.time() * 1000)
        self._event(1, hdfs.CloseEventProto(path=self._norm(r.src), fileSize=sum(x.numBytes for x in n.blocks),
                                            timestamp=n.mtime))
        return hdfs.CompleteResponseProto(result=True)

    def rpc_getBlockLocations(self, b, user):
        r = hdfs.GetBlockLocationsRequestProto.FromString(b)
        p = self._norm(r.src)
        n = self.ns.get(p)
        if n is None or n.is_dir:
            raise _fnf(p)
        out = hdfs.GetBlockLocationsResponseProto()
        lbs = out.locations
        lbs.fileLength = sum(x.numBytes for x in n.blocks)
        lbs.underConstruction = not n.complete
        lbs.isLastBlockComplete = n.complete
        off = 0
        for eb in n.blocks:
            if off + eb.numBytes > r.offset and off < r.offset + r.length:
                dns = [dn for dn in self.datanodes if eb.blockId in dn.blocks]
                lbs.blocks.add().CopyFrom(self._located(eb, off, dns))
            off += eb.numBytes
        return out

    def rpc_setPermission(self, b, user):
        r = hdfs.SetPermissionRequestProto.FromString(b)
        n = self.ns.get(self._norm(r.src))
        if n is None:
            raise _fnf(r.src)
        n.mode = r.permission.perm
        self._event(4, hdfs.MetadataUpdateEventProto(path=self._norm(r.src), type=2))
        return hdfs.SetPermissionResponseProto()

    def rpc_setOwner(self, b, user):
        r = hdfs.SetOwnerRequestProto.FromString(b)
        n = self.ns.get(self._norm(r.src))
        if n is None:
            raise _fnf(r.src)
        if r.HasField("username"):
            n.owner = r.username
        if r.HasField("groupname"):
            n.group = r.groupname
        return hdfs.SetOwnerResponseProto()

    def rpc_getFsStats(self, b, user):
        used = sum(len(v) for dn in self.datanodes for v in dn.blocks.values())
        return hdfs.GetFsStatsResponseProto(capacity=1 << 40, used=used, remaining=(1 << 40) - used,
                                            under_replicated=0, corrupt_blocks=0, missing_blocks=0)

    def rpc_getAclStatus(self, b, user):
        r = hdfs.GetAclStatusRequestProto.FromString(b)
        n = self.ns.get(self._norm(r.src))
        if n is None:
            raise _fnf(r.src)
        out = hdfs.GetAclStatusResponseProto()
        st = out.result
        st.owner, st.group, st.sticky = n.owner, n.group, False
        st.permission.perm = n.mode
        st.entries.extend(n.acl)
        return out

    def rpc_setAcl(self, b, user):
        """Full replacement: base entries set the permission bits (the mask, when present, takes
        the group bits); named, unnamed-group-with-mask and default entries are kept as the ACL."""
        r = hdfs.SetAclRequestProto.FromString(b)
        n = self.ns.get(self._norm(r.src))
        if n is None:
            raise _fnf(r.src)
        keep, mode, mask = [], n.mode, None
        access = [e for e in r.aclSpec if e.scope == 0]
        extended = any(e.HasField("name") and e.name for e in access)
        for e in r.aclSpec:
            if e.scope == 1:
                keep.append(e)
                continue
            if e.type == 0 and not e.name:
                mode = (mode & 0o7077) | (e.permissions << 6)
            elif e.type == 3:
                mode = (mode & 0o7770) | e.permissions
            elif e.type == 2:
                mask = e.permissions
            elif e.type == 1 and not e.name:
                if extended:
                    keep.append(e)
                else:
                    mode = (mode & 0o7707) | (e.permissions << 3)
            else:
                keep.append(e)
        if extended and mask is not None:
            mode = (mode & 0o7707) | (mask << 3)
        n.mode, n.acl = mode, keep
        self._event(4, hdfs.MetadataUpdateEventProto(path=self._norm(r.src), type=5))
        return hdfs.SetAclResponseProto()

    def rpc_getCurrentEditLogTxid(self, b, user):
        return hdfs.GetCurrentEditLogTxidResponseProto(txid=len(self.edits))

    def rpc_getEditsFromTxid(self, b, user):
        r = hdfs.GetEditsFromTxidRequestProto.FromString(b)
        out = hdfs.GetEditsFromTxidResponseProto()
        el = out.eventsList
        batches = self.edits[max(0, r.txid - 1):max(0, r.txid - 1) + 50]   # a bounded page per call
        el.batch.extend(batches)
        el.firstTxid = batches[0].txid if batches else r.txid
        el.lastTxid = batches[-1].txid if batches else r.txid - 1
        el.syncTxid = len(self.edits)
        return out

    def rpc_getServerDefaults(self, b, user):
        d = hdfs.FsServerDefaultsProto(blockSize=128 << 20, bytesPerChecksum=512, writePacketSize=65536,
                                       replication=3, fileBufferSize=4096, checksumType=H.CHECKSUM_CRC32C)
        return hdfs.GetServerDefaultsResponseProto(serverDefaults=d)

    def rpc_renewLease(self, b, user):
        return hdfs.RenewLeaseResponseProto()


class _Sink:
    def __init__(self, dn, bid):
        self.dn, self.bid, self.buf = dn, bid, bytearray()

    def write(self, data):
        self.buf += data

    def commit(self, n):
        self.dn.blocks[self.bid] = bytes(self.buf)        # finalized replica (blockReceived)


class _Reader:
    def __init__(self, data, off):
        self.data, self.off = data, off

    def read(self, n):
        b = self.data[self.off:self.off + n]
        self.off += len(b)
        return b


class _DataNode:
    """One DataNode: the shared DataTransferServer over an in-memory replica map."""

    def __init__(self, dfs: MiniDfs, idx: int):
        self.dfs, self.idx = dfs, idx
        self.blocks: dict[int, bytes] = {}
        self.fail_reads = False
        self.server = DataTransferServer(self._open_read, self._open_write)
        self.port = self.server.port

    @property
    def truncate_reads(self):
        return self.server.fault_truncate

    @truncate_reads.setter
    def truncate_reads(self, v):
        self.server.fault_truncate = v

    @property
    def corrupt_reads(self):
        return self.server.fault_flip_bits

    @corrupt_reads.setter
    def corrupt_reads(self, v):
        self.server.fault_flip_bits = v

    def _open_read(self, bid, offset, length):
        data = self.blocks.get(bid)
        if data is None or self.fail_reads or offset + length > len(data):
            raise IOError(f"block {bid} unavailable")
        return _Reader(data, offset)

    def _open_write(self, op):
        return _Sink(self, op.header.baseHeader.block.blockId)

    def info(self):
        d = self.server.info("127.0.0.1")
        d.id.hostName = "localhost"
        d.id.datanodeUuid = f"dn-{self.idx}"
        return d

    def stop(self):
        self.server.stop()
