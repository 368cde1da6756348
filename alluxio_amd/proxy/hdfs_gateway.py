"""HDFS-protocol gateway: unmodified Hadoop clients reach the Alluxio namespace as ``hdfs://``.

The reference ships ``alluxio.hadoop.FileSystem`` (core/client/hdfs/src/main/java/alluxio/hadoop/
AbstractFileSystem.java: create :152, initialize :447-460, open :622-629, plus getFileStatus /
listStatus / mkdirs / rename / delete / setOwner / setPermission) so that Spark, Presto and Hive
can read ``alluxio://``.  That class needs a JVM on the compute side.  This gateway instead speaks
the two wire protocols every Hadoop client already has built in, so ``hdfs://gateway:port/`` works
with no Alluxio jar at all:

* a **NameNode** endpoint (Hadoop IPC v9, ``ClientProtocol``) whose calls map onto the Alluxio
  FileSystem API: getFileInfo/getListing (paged)/mkdirs/delete/rename/create/addBlock/complete/
  abandonBlock/getBlockLocations/setPermission/setOwner/getFsStats/getServerDefaults/
  getContentSummary/renewLease/fsync;
* a **DataNode** endpoint (DataTransferProtocol v28): READ_BLOCK streams the Alluxio block's bytes
  (an HDFS block here IS an Alluxio block: same id, same length) in CRC32C-checksummed packets;
  WRITE_BLOCK appends the packets of each block, in order, to the file's Alluxio out stream, which
  ``complete`` closes.

``IpcServer`` and ``DataTransferServer`` are the protocol halves, reusable with any backend (the
test-suite's mini HDFS uses them over an in-memory namespace).  Wire details are shared with the
client in :mod:`alluxio_amd.underfs.hadoop_rpc`.  Java-client interop is parity unpinned (no JVM
here); the native Hadoop client runs the UFS contract through it in ``tests/test_hdfs_gateway.py``.
"""
from __future__ import annotations

import collections
import logging
import posixpath
import socket
import socketserver
import struct
import threading
import time

from ..underfs import hadoop_rpc as H
from ..utils.exceptions import (AlreadyExistsException, DirectoryNotEmptyException, NotFoundException,
                                PermissionDeniedException)

LOG = logging.getLogger(__name__)
common, hdfs = H.common, H.hdfs


class RpcError(Exception):
    """A Java exception to return to the caller (RpcResponseHeaderProto status ERROR)."""

    def __init__(self, cls: str, msg: str):
        super().__init__(msg)
        self.cls, self.msg = cls, msg


def file_not_found(path: str) -> RpcError:
    return RpcError("java.io.FileNotFoundException", f"File does not exist: {path}")


class _TcpServer(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True


class _Service:
    def __init__(self, host: str, port: int, handler_cls):
        self.server = _TcpServer((host, port), handler_cls)
        self.server.owner = self
        self.port = self.server.server_address[1]
        threading.Thread(target=self.server.serve_forever, kwargs={"poll_interval": 0.05}, daemon=True,
                         name=type(self).__name__).start()

    def stop(self) -> None:
        self.server.shutdown()
        self.server.server_close()


# ---- NameNode (Hadoop IPC v9) -----------------------------------------------------------------------
MAX_IPC_FRAME = 64 << 20     # Hadoop's ipc.maximum.data.length default


class IpcServer(_Service):
    """Serves ``ClientProtocol`` calls: ``dispatch(method, request_bytes, user)`` returns the
    response message or raises :class:`RpcError`."""

    def __init__(self, dispatch, host: str = "127.0.0.1", port: int = 0):
        self.dispatch = dispatch
        super().__init__(host, port, _IpcHandler)


def _send_frame(sock, *msgs) -> None:
    payload = b"".join(H.delimited(m) for m in msgs)
    sock.sendall(struct.pack(">I", len(payload)) + payload)


class _IpcHandler(socketserver.BaseRequestHandler):
    def handle(self):
        s, srv = self.request, self.server.owner
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        try:
            pre = bytes(H.recv_exact(s, 7))
            if pre[:4] != b"hrpc" or pre[4] != H.IPC_VERSION or pre[6] != H.AUTH_NONE:
                return                      # only SIMPLE auth (no SASL) is served
            user = "hadoop"
            while True:
                (n,) = struct.unpack(">I", bytes(H.recv_exact(s, 4)))
                if n > MAX_IPC_FRAME:           # ipc.maximum.data.length: refuse, do not allocate
                    LOG.warning("hdfs gateway: %d-byte RPC frame from %s exceeds %d; closing", n,
                                self.client_address, MAX_IPC_FRAME)
                    return
                frame = H.recv_exact(s, n)
                rh, pos = H.parse_delimited(frame, 0, common.RpcRequestHeaderProto)
                if rh.callId == H.CONNECTION_CONTEXT_CALL_ID:
                    ctx, _ = H.parse_delimited(frame, pos, common.IpcConnectionContextProto)
                    user = ctx.userInfo.effectiveUser or user
                    continue
                if rh.callId < 0:               # ping / SASL negotiation: nothing to answer
                    continue
                req_hdr, pos = H.parse_delimited(frame, pos, common.RequestHeaderProto)
                body = _delimited_body(frame, pos)
                resp = common.RpcResponseHeaderProto(callId=rh.callId, status=0, serverIpcVersionNum=H.IPC_VERSION,
                                                     clientId=rh.clientId)
                try:
                    out = srv.dispatch(req_hdr.methodName, body, user)
                    _send_frame(s, resp, out)
                except RpcError as e:
                    resp.status = 1
                    resp.exceptionClassName, resp.errorMsg = e.cls, e.msg
                    _send_frame(s, resp)
                except Exception as e:  # noqa: BLE001 - every failure becomes an IOException
                    LOG.debug("hdfs gateway call %s failed", req_hdr.methodName, exc_info=True)
                    resp.status = 1
                    resp.exceptionClassName, resp.errorMsg = "java.io.IOException", str(e)[:500]
                    _send_frame(s, resp)
        except (ConnectionError, OSError):
            return


def _delimited_body(frame, pos: int) -> bytes:
    shift = ln = 0
    while True:
        c = frame[pos]
        pos += 1
        ln |= (c & 0x7F) << shift
        if not c & 0x80:
            break
        shift += 7
    return bytes(frame[pos:pos + ln])


# ---- DataNode (DataTransferProtocol v28) --------------------------------------------------------------
class DataTransferServer(_Service):
    """READ_BLOCK / WRITE_BLOCK.  ``open_read(block_id, offset, length)`` returns an object with
    ``read(n) -> bytes`` and optional ``close()`` (raise to refuse); ``open_write(op)`` returns a
    sink with ``write(memoryview)`` and ``commit(num_bytes)``.  Pipelines (``targets``) are
    forwarded to the next DataNode, acks merged, as BlockReceiver/PacketResponder do."""

    def __init__(self, open_read, open_write, host: str = "127.0.0.1", port: int = 0):
        self.open_read, self.open_write = open_read, open_write
        self.fault_flip_bits = False    # fault injection: corrupt sent data AFTER checksumming it
        self.fault_truncate = False     # fault injection: end the block after its first packet
        self.packet_bytes = 1 << 20     # data bytes per packet of the native sender
        super().__init__(host, port, _DataHandler)
        self.host = host
        self.uuid = f"alluxio-dn-{self.port}"

    def info(self, host: str | None = None):
        d = hdfs.DatanodeInfoProto(capacity=1 << 50)
        h = host or self.host
        d.id.CopyFrom(hdfs.DatanodeIDProto(ipAddr=h, hostName=h, datanodeUuid=self.uuid, xferPort=self.port,
                                           infoPort=0, ipcPort=0))
        return d


class _DataHandler(socketserver.BaseRequestHandler):
    def handle(self):
        s, srv = self.request, self.server.owner
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        try:
            ver, op = struct.unpack(">HB", bytes(H.recv_exact(s, 3)))
            if ver != H.DATA_TRANSFER_VERSION:
                return
            if op == H.OP_READ_BLOCK:
                self._read(s, srv, H.recv_delimited(s, hdfs.OpReadBlockProto))
            elif op == H.OP_WRITE_BLOCK:
                self._write(s, srv, H.recv_delimited(s, hdfs.OpWriteBlockProto))
            else:
                s.sendall(H.delimited(hdfs.BlockOpResponseProto(status=7, message=f"op {op} unsupported")))
        except (ConnectionError, OSError):
            return

    @staticmethod
    def _read(s, srv, op):
        bid = op.header.baseHeader.block.blockId
        bpc = H.BYTES_PER_CHECKSUM
        start = op.offset - op.offset % bpc           # chunk-aligned, as BlockSender does
        try:
            src = srv.open_read(bid, start, op.offset + op.len - start)
        except Exception as e:  # noqa: BLE001
            s.sendall(H.delimited(hdfs.BlockOpResponseProto(status=H.ST_ERROR, message=str(e)[:300])))
            return
        try:
            resp = hdfs.BlockOpResponseProto(status=H.ST_SUCCESS)
            resp.readOpChecksumInfo.checksum.type = H.CHECKSUM_CRC32C
            resp.readOpChecksumInfo.checksum.bytesPerChecksum = bpc
            resp.readOpChecksumInfo.chunkOffset = start
            s.sendall(H.delimited(resp))
            native = getattr(src, "native_source", None)
            ns = native() if native is not None else None
            if ns is not None:
                # packets built and sent in C++ (csrc/hdfs_packets.cpp): source chunk -> CRC32C
                # per 512 B -> one writev per 1 MiB packet, GIL released
                from ..ops.native import lib
                bsrc, soff = ns
                try:
                    lib().dn_send_block(s.fileno(), bsrc, soff, op.offset + op.len - start, bpc,
                                        srv.packet_bytes, 60_000, srv.fault_flip_bits, srv.fault_truncate)
                except Exception:  # noqa: BLE001 - a reader that stops early closes its socket
                    LOG.debug("hdfs gateway: read of block %d ended by the client", bid, exc_info=True)
                return
            seq, off, end = 0, start, op.offset + op.len
            while off < end:
                data = src.read(min(H.PACKET_DATA, end - off))
                if not data:
                    break
                if srv.fault_flip_bits:
                    sums = H._crc_chunks(data, bpc)
                    hdr = hdfs.PacketHeaderProto(offsetInBlock=off, seqno=seq, lastPacketInBlock=False,
                                                 dataLen=len(data)).SerializeToString()
                    s.sendall(struct.pack(">IH", 4 + len(sums) + len(data), len(hdr)) + hdr + sums +
                              bytes([data[0] ^ 1]) + bytes(data[1:]))
                else:
                    H.write_packet(s, off, seq, data, False)
                off += len(data)
                seq += 1
                if srv.fault_truncate:
                    break
            H.write_packet(s, off, seq, b"", True)
        finally:
            close = getattr(src, "close", None)
            if close is not None:
                close()
        try:
            H.recv_delimited(s, hdfs.ClientReadStatusProto)
        except (ConnectionError, OSError):
            pass

    @staticmethod
    def _write(s, srv, op):
        downstream = None
        if len(op.targets):
            nxt = op.targets[0]
            downstream = socket.create_connection((nxt.id.ipAddr, nxt.id.xferPort), timeout=60)
            fwd = hdfs.OpWriteBlockProto()
            fwd.CopyFrom(op)
            del fwd.targets[0]
            downstream.sendall(struct.pack(">HB", H.DATA_TRANSFER_VERSION, H.OP_WRITE_BLOCK) + H.delimited(fwd))
            r = H.recv_delimited(downstream, hdfs.BlockOpResponseProto)
            if r.status != H.ST_SUCCESS:
                s.sendall(H.delimited(hdfs.BlockOpResponseProto(status=H.ST_ERROR, firstBadLink=nxt.id.ipAddr)))
                downstream.close()
                return
        try:
            sink = srv.open_write(op)
        except Exception as e:  # noqa: BLE001
            s.sendall(H.delimited(hdfs.BlockOpResponseProto(status=H.ST_ERROR, message=str(e)[:300])))
            return
        s.sendall(H.delimited(hdfs.BlockOpResponseProto(status=H.ST_SUCCESS)))
        bpc = op.requestedChecksum.bytesPerChecksum or H.BYTES_PER_CHECKSUM
        received = 0
        status = H.ST_SUCCESS
        try:
            received, status = _DataHandler._receive(s, sink, downstream, bpc)
        except BaseException:
            abort = getattr(sink, "abort", None)
            if abort is not None:
                abort()               # a block cut off mid-stream must not complete silently
            raise
        finally:
            if downstream is not None:
                downstream.close()
        if status == H.ST_SUCCESS:
            sink.commit(received)
        else:
            abort = getattr(sink, "abort", None)
            if abort is not None:
                abort()

    @staticmethod
    def _receive(s, sink, downstream, bpc):
        if downstream is None:
            rx = None
            try:
                from ..ops.native import lib
                rx = lib().DnPacketReceiver(s.fileno(), bpc, 60_000)
            except Exception:  # noqa: BLE001 - no native extension: the Python packet loop
                rx = None
            if rx is not None:
                return _DataHandler._receive_native(rx, sink)
        received, status = 0, H.ST_SUCCESS
        while True:
            plen, hlen = struct.unpack(">IH", bytes(H.recv_exact(s, 6)))
            hraw = bytes(H.recv_exact(s, hlen))
            body = H.recv_exact(s, plen - 4)
            hdr = hdfs.PacketHeaderProto.FromString(hraw)
            data = body[len(body) - hdr.dataLen:]
            if hdr.dataLen and H._crc_chunks(data, bpc) != bytes(body[:len(body) - hdr.dataLen]):
                status = H.ST_ERROR_CHECKSUM
            elif hdr.offsetInBlock != received:
                status = H.ST_ERROR
            if downstream is not None:
                downstream.sendall(struct.pack(">IH", plen, hlen) + hraw + bytes(body))
            if status == H.ST_SUCCESS and hdr.dataLen:
                try:
                    sink.write(data)
                except Exception:  # noqa: BLE001
                    LOG.debug("hdfs gateway block write failed", exc_info=True)
                    status = H.ST_ERROR
                received += hdr.dataLen
            replies = [status]
            if downstream is not None:
                replies += list(H.recv_delimited(downstream, hdfs.PipelineAckProto).reply)
            ack = hdfs.PipelineAckProto(seqno=hdr.seqno)
            ack.reply.extend(replies)
            s.sendall(H.delimited(ack))
            if hdr.lastPacketInBlock or status != H.ST_SUCCESS:
                return received, status


    _RX_BATCH = 4 << 20

    @staticmethod
    def _receive_native(rx, sink):
        """Packets parsed and CRC-verified in C++ straight into a batch buffer
        (csrc/hdfs_packets.cpp DnPacketReceiver); the batch goes to the sink, then every packet of it
        is acked -- an ack still means the bytes reached the Alluxio out stream."""
        buf = bytearray(_DataHandler._RX_BATCH + (17 << 20))
        mv = memoryview(buf)
        while True:
            n, last, status = rx.receive(buf, _DataHandler._RX_BATCH)
            if status == H.ST_SUCCESS and n:
                try:
                    sink.write(mv[:n])
                except Exception:  # noqa: BLE001
                    LOG.debug("hdfs gateway block write failed", exc_info=True)
                    status = H.ST_ERROR
            rx.ack(status)
            if last or status != H.ST_SUCCESS:
                return rx.received, status


# ---- the Alluxio-backed gateway -------------------------------------------------------------------------
_BLOCK_POOL = "BP-alluxio-amd"
_LS_LIMIT = 1000


def _remote(e: Exception, path: str) -> RpcError:
    if isinstance(e, NotFoundException):
        return file_not_found(path)
    if isinstance(e, AlreadyExistsException):
        return RpcError("org.apache.hadoop.fs.FileAlreadyExistsException", f"{path} already exists")
    if isinstance(e, PermissionDeniedException):
        return RpcError("org.apache.hadoop.security.AccessControlException", str(e))
    if isinstance(e, DirectoryNotEmptyException):
        return RpcError("org.apache.hadoop.fs.PathIsNotEmptyDirectoryException", f"{path} is non empty")
    return RpcError("java.io.IOException", str(e)[:500])


class _OpenFile:
    def __init__(self, path, stream, file_id, block_size):
        self.path, self.stream, self.file_id, self.block_size = path, stream, file_id, block_size
        self.lock = threading.Lock()
        self.blocks: list = []       # ExtendedBlockProto of the blocks handed out by addBlock
        self.written = 0
        self.broken = False          # a block stream failed after bytes reached the out stream


class _BlockSink:
    def __init__(self, of: _OpenFile):
        self.of = of

    def write(self, data) -> None:
        with self.of.lock:
            self.of.stream.write(data)          # copied into the cache (and UFS) before it returns
            self.of.written += len(data)

    def commit(self, n: int) -> None:
        pass

    def abort(self) -> None:
        # bytes of the failed block may already be in the Alluxio out stream, which cannot take
        # them back: fail the file at complete() instead of publishing a corrupt one
        self.of.broken = True


class _RangeReader:
    def __init__(self, stream, offset: int, length: int):
        self.stream, self.left, self.start = stream, length, offset
        stream.seek(offset)

    def native_source(self):
        """(native BlockSource, offset in it) for the DataNode's C++ packet sender when the range
        lies in one Alluxio block (a gateway block is one), else None."""
        f = self.stream
        if getattr(f, "_nat", None) is None or self.left <= 0:
            return None
        idx = self.start // f.block_size
        if (self.start + self.left - 1) // f.block_size != idx:
            return None
        return f._open_native(idx, False), self.start - idx * f.block_size

    def read(self, n: int) -> bytes:
        if self.left <= 0:
            return b""
        b = self.stream.read(min(n, self.left))
        self.left -= len(b)
        return b

    def close(self) -> None:
        self.stream.close()


class HdfsGateway:
    """NameNode + DataNode endpoints over an Alluxio :class:`FileSystem` client."""

    def __init__(self, fs, host: str = "127.0.0.1", rpc_port: int = 0, data_port: int = 0,
                 advertised_host: str | None = None, write_type: str = "CACHE_THROUGH", impersonate: bool = True):
        self._default_fs, self.write_type = fs, write_type
        # NameNode calls run as the Hadoop caller (IpcConnectionContext effectiveUser): one client
        # per user, so the master authorizes -- and records as owner -- that user, not the proxy's
        self.impersonate = impersonate
        self._tls = threading.local()
        self._user_fs: "collections.OrderedDict[str, object]" = collections.OrderedDict()
        self._user_fs_cap = 64
        self.adv = advertised_host or host
        self.lock = threading.Lock()
        self.open_files: dict[str, _OpenFile] = {}
        self.write_blocks: dict[int, _OpenFile] = {}
        # block id -> (path, file offset, length), filled by getBlockLocations; LRU-bounded
        self.read_blocks: "collections.OrderedDict[int, tuple[str, int, int]]" = collections.OrderedDict()
        self.read_blocks_cap = 1 << 20
        self.next_block = 1 << 40
        self.data = DataTransferServer(self._open_read, self._open_write, host, data_port)
        self.rpc = IpcServer(self._dispatch, host, rpc_port)
        self.calls: dict[str, int] = {}

    @property
    def port(self) -> int:
        return self.rpc.port

    @property
    def fs(self):
        """The client of the current NameNode call's user (the proxy's own outside a call)."""
        return getattr(self._tls, "fs", None) or self._default_fs

    def _fs_for(self, user: str):
        base = self._default_fs
        if not self.impersonate or not user or user == base.ctx.user:
            return base
        with self.lock:
            fs = self._user_fs.get(user)
            if fs is not None:
                self._user_fs.move_to_end(user)
                return fs
        from ..client.file_system import FileSystem
        from ..client.context import FileSystemContext
        ctx = FileSystemContext(base.ctx.conf, ",".join(base.ctx.master_addresses), user)
        fs = FileSystem(context=ctx)
        with self.lock:
            self._user_fs[user] = fs
            while len(self._user_fs) > self._user_fs_cap:
                _u, old = self._user_fs.popitem(last=False)
                try:
                    old.close()
                except Exception:  # noqa: BLE001
                    pass
        return fs

    def stop(self) -> None:
        self.rpc.stop()
        self.data.stop()
        with self.lock:
            users, self._user_fs = list(self._user_fs.values()), collections.OrderedDict()
        for fs in users:
            try:
                fs.close()
            except Exception:  # noqa: BLE001
                pass
        with self.lock:
            files, self.open_files = list(self.open_files.values()), {}
        for of in files:
            try:
                of.stream.close()
            except Exception:  # noqa: BLE001
                pass

    # ---- dispatch -----------------------------------------------------------------------------------
    def _dispatch(self, method: str, body: bytes, user: str):
        self.calls[method] = self.calls.get(method, 0) + 1
        fn = getattr(self, "rpc_" + method, None)
        if fn is None:
            raise RpcError("org.apache.hadoop.ipc.RpcNoSuchMethodException", f"Unknown method {method} called on "
                           f"{H.CLIENT_PROTOCOL} protocol.")
        self._tls.fs = self._fs_for(user)
        try:
            return fn(body, user)
        finally:
            self._tls.fs = None

    def _status(self, st, name: bytes):
        info = st.info
        out = hdfs.HdfsFileStatusProto(fileType=H.FILE_IS_DIR if info.folder else H.FILE_IS_FILE, path=name,
                                       length=0 if info.folder else info.length, owner=info.owner,
                                       group=info.group, modification_time=info.lastModificationTimeMs,
                                       access_time=info.lastAccessTimeMs or info.lastModificationTimeMs,
                                       block_replication=0 if info.folder else max(1, info.replicationMin or 1),
                                       blocksize=0 if info.folder else info.blockSizeBytes, fileId=info.fileId,
                                       childrenNum=0)
        out.permission.perm = info.mode & 0o7777
        return out

    @staticmethod
    def _norm(p: str) -> str:
        return "/" + p.strip("/") if p.strip("/") else "/"

    # ---- ClientProtocol -----------------------------------------------------------------------------
    def rpc_getFileInfo(self, b, user):
        p = self._norm(hdfs.GetFileInfoRequestProto.FromString(b).src)
        out = hdfs.GetFileInfoResponseProto()
        try:
            out.fs.CopyFrom(self._status(self.fs.get_status(p), b""))
        except NotFoundException:
            pass
        except Exception as e:  # noqa: BLE001
            raise _remote(e, p) from None
        return out

    def rpc_getListing(self, b, user):
        r = hdfs.GetListingRequestProto.FromString(b)
        p = self._norm(r.src)
        out = hdfs.GetListingResponseProto()
        try:
            st = self.fs.get_status(p)
            if not st.info.folder:
                out.dirList.partialListing.add().CopyFrom(self._status(st, b""))
                out.dirList.remainingEntries = 0
                return out
            items = sorted(self.fs.list_status(p), key=lambda x: x.name)
        except NotFoundException:
            return out
        except Exception as e:  # noqa: BLE001
            raise _remote(e, p) from None
        after = r.startAfter.decode()
        items = [x for x in items if x.name > after]
        for x in items[:_LS_LIMIT]:
            out.dirList.partialListing.add().CopyFrom(self._status(x, x.name.encode()))
        out.dirList.remainingEntries = max(0, len(items) - _LS_LIMIT)
        return out

    def rpc_mkdirs(self, b, user):
        r = hdfs.MkdirsRequestProto.FromString(b)
        p = self._norm(r.src)
        try:
            if not r.createParent and not self.fs.exists(posixpath.dirname(p) or "/"):
                raise file_not_found(posixpath.dirname(p))
            self.fs.create_directory(p, recursive=True, allow_exists=True, mode=r.masked.perm & 0o7777)
        except RpcError:
            raise
        except Exception as e:  # noqa: BLE001
            raise _remote(e, p) from None
        return hdfs.MkdirsResponseProto(result=True)

    def rpc_delete(self, b, user):
        r = hdfs.DeleteRequestProto.FromString(b)
        p = self._norm(r.src)
        if p == "/":
            return hdfs.DeleteResponseProto(result=False)
        try:
            self.fs.delete(p, recursive=r.recursive)
        except NotFoundException:
            return hdfs.DeleteResponseProto(result=False)
        except Exception as e:  # noqa: BLE001
            raise _remote(e, p) from None
        return hdfs.DeleteResponseProto(result=True)

    def rpc_rename(self, b, user):
        r = hdfs.RenameRequestProto.FromString(b)
        try:
            self.fs.rename(self._norm(r.src), self._norm(r.dst))
        except Exception:  # noqa: BLE001 - HDFS rename reports failure as false
            return hdfs.RenameResponseProto(result=False)
        return hdfs.RenameResponseProto(result=True)

    def rpc_create(self, b, user):
        r = hdfs.CreateRequestProto.FromString(b)
        p = self._norm(r.src)
        try:
            if self.fs.exists(p):
                if self.fs.get_status(p).info.folder or not r.createFlag & H.CREATE_FLAG_OVERWRITE:
                    raise RpcError("org.apache.hadoop.fs.FileAlreadyExistsException", f"{p} already exists")
                self.fs.delete(p)
            parent = posixpath.dirname(p) or "/"
            if not r.createParent and not self.fs.exists(parent):
                raise file_not_found(parent)
            stream = self.fs.create_file(p, block_size=r.blockSize or None, recursive=True,
                                         mode=r.masked.perm & 0o7777, write_type=self.write_type)
            st = self.fs.get_status(p)
        except RpcError:
            raise
        except Exception as e:  # noqa: BLE001
            raise _remote(e, p) from None
        with self.lock:
            self.open_files[p] = _OpenFile(p, stream, st.info.fileId, st.info.blockSizeBytes)
        return hdfs.CreateResponseProto(fs=self._status(st, b""))

    def _open(self, src: str) -> _OpenFile:
        of = self.open_files.get(self._norm(src))
        if of is None:
            raise RpcError("org.apache.hadoop.hdfs.server.namenode.LeaseExpiredException",
                           f"No lease on {src}: file is not open for writing")
        return of

    def rpc_addBlock(self, b, user):
        r = hdfs.AddBlockRequestProto.FromString(b)
        with self.lock:
            of = self._open(r.src)
            bid = self.next_block
            self.next_block += 1
            eb = hdfs.ExtendedBlockProto(poolId=_BLOCK_POOL, blockId=bid, generationStamp=1, numBytes=0)
            of.blocks.append(eb)
            self.write_blocks[bid] = of
        lb = hdfs.LocatedBlockProto(offset=of.written, corrupt=False)
        lb.b.CopyFrom(eb)
        lb.blockToken.CopyFrom(common.TokenProto(identifier=b"", password=b"", kind="", service=""))
        lb.locs.add().CopyFrom(self.data.info(self.adv))
        return hdfs.AddBlockResponseProto(block=lb)

    def rpc_abandonBlock(self, b, user):
        r = hdfs.AbandonBlockRequestProto.FromString(b)
        with self.lock:
            self.write_blocks.pop(r.b.blockId, None)
        return hdfs.AbandonBlockResponseProto()

    def rpc_complete(self, b, user):
        r = hdfs.CompleteRequestProto.FromString(b)
        p = self._norm(r.src)
        with self.lock:
            of = self.open_files.pop(p, None)
            if of is not None:
                for eb in of.blocks:
                    self.write_blocks.pop(eb.blockId, None)
        if of is None:
            # a retried complete of a file already closed succeeds, as FSNamesystem allows
            if self.fs.exists(p):
                return hdfs.CompleteResponseProto(result=True)
            raise file_not_found(p)
        if of.broken:
            try:
                of.stream.cancel() if hasattr(of.stream, "cancel") else of.stream.close()
                self.fs.delete(p)
            except Exception:  # noqa: BLE001
                LOG.debug("cleanup of failed gateway write %s", p, exc_info=True)
            raise RpcError("java.io.IOException", f"a block of {p} failed mid-stream; the file was discarded")
        try:
            with of.lock:
                of.stream.close()
        except Exception as e:  # noqa: BLE001
            raise _remote(e, p) from None
        return hdfs.CompleteResponseProto(result=True)

    def rpc_fsync(self, b, user):
        return hdfs.FsyncResponseProto()

    def rpc_getBlockLocations(self, b, user):
        r = hdfs.GetBlockLocationsRequestProto.FromString(b)
        p = self._norm(r.src)
        try:
            st = self.fs.get_status(p)
        except Exception as e:  # noqa: BLE001
            raise _remote(e, p) from None
        if st.info.folder:
            raise file_not_found(p)
        out = hdfs.GetBlockLocationsResponseProto()
        lbs = out.locations
        lbs.fileLength, lbs.underConstruction = st.info.length, not st.info.completed
        lbs.isLastBlockComplete = st.info.completed
        off = 0
        for fbi in st.info.fileBlockInfos:
            bi = fbi.blockInfo
            if bi.length and off + bi.length > r.offset and off < r.offset + r.length:
                lb = lbs.blocks.add(offset=off, corrupt=False)
                lb.b.CopyFrom(hdfs.ExtendedBlockProto(poolId=_BLOCK_POOL, blockId=bi.blockId, generationStamp=1,
                                                      numBytes=bi.length))
                lb.blockToken.CopyFrom(common.TokenProto(identifier=b"", password=b"", kind="", service=""))
                lb.locs.add().CopyFrom(self.data.info(self.adv))
                with self.lock:
                    self.read_blocks[bi.blockId] = (p, off, bi.length)
                    self.read_blocks.move_to_end(bi.blockId)
                    while len(self.read_blocks) > self.read_blocks_cap:
                        self.read_blocks.popitem(last=False)
            off += bi.length
        return out

    def rpc_setPermission(self, b, user):
        r = hdfs.SetPermissionRequestProto.FromString(b)
        try:
            self.fs.set_attribute(self._norm(r.src), mode=r.permission.perm & 0o7777)
        except Exception as e:  # noqa: BLE001
            raise _remote(e, r.src) from None
        return hdfs.SetPermissionResponseProto()

    def rpc_setOwner(self, b, user):
        r = hdfs.SetOwnerRequestProto.FromString(b)
        try:
            self.fs.set_attribute(self._norm(r.src), owner=r.username if r.HasField("username") else None,
                                  group=r.groupname if r.HasField("groupname") else None)
        except Exception as e:  # noqa: BLE001
            raise _remote(e, r.src) from None
        return hdfs.SetOwnerResponseProto()

    def rpc_getFsStats(self, b, user):
        total, used = self.fs.capacity()
        return hdfs.GetFsStatsResponseProto(capacity=total, used=used, remaining=max(0, total - used),
                                            under_replicated=0, corrupt_blocks=0, missing_blocks=0)

    def rpc_getServerDefaults(self, b, user):
        d = hdfs.FsServerDefaultsProto(blockSize=64 << 20, bytesPerChecksum=H.BYTES_PER_CHECKSUM,
                                       writePacketSize=H.PACKET_DATA, replication=1, fileBufferSize=4096,
                                       encryptDataTransfer=False, trashInterval=0, checksumType=H.CHECKSUM_CRC32C)
        return hdfs.GetServerDefaultsResponseProto(serverDefaults=d)

    def rpc_getContentSummary(self, b, user):
        p = self._norm(hdfs.GetContentSummaryRequestProto.FromString(b).path)
        try:
            st = self.fs.get_status(p)
            items = self.fs.list_status(p, recursive=True) if st.info.folder else [st]
        except Exception as e:  # noqa: BLE001
            raise _remote(e, p) from None
        files = [x for x in items if not x.info.folder]
        n_dirs = (1 if st.info.folder else 0) + sum(1 for x in items if x.info.folder)
        length = sum(x.info.length for x in files)
        none = (1 << 64) - 1     # uint64 on the wire; a Java long reads it as -1 (no quota)
        cs = hdfs.ContentSummaryProto(length=length, fileCount=len(files), directoryCount=n_dirs, quota=none,
                                      spaceConsumed=length, spaceQuota=none)
        return hdfs.GetContentSummaryResponseProto(summary=cs)

    def rpc_renewLease(self, b, user):
        return hdfs.RenewLeaseResponseProto()

    # ---- DataNode backend -----------------------------------------------------------------------------
    def _open_read(self, block_id: int, offset: int, length: int):
        with self.lock:
            loc = self.read_blocks.get(block_id)
        if loc is None:
            raise IOError(f"block {block_id} is not known to this gateway (getBlockLocations first)")
        path, foff, blen = loc
        if offset + length > blen:
            raise IOError(f"read past the end of block {block_id}")
        return _RangeReader(self.fs.open_file(path), foff + offset, length)

    def _open_write(self, op):
        bid = op.header.baseHeader.block.blockId
        with self.lock:
            of = self.write_blocks.get(bid)
        if of is None:
            raise IOError(f"block {bid} was not allocated by addBlock")
        return _BlockSink(of)


def serve(fs, host: str, rpc_port: int, data_port: int, advertised_host: str | None = None) -> HdfsGateway:
    g = HdfsGateway(fs, host, rpc_port, data_port, advertised_host)
    LOG.info("HDFS gateway: NameNode on %s:%d, DataNode on %s:%d", host, g.rpc.port, host, g.data.port)
    return g


def _wait_forever():  # pragma: no cover - CLI helper
    while True:
        time.sleep(3600)
