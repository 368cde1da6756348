"""Native framed-RPC transport for unary calls (see ``csrc/frame_rpc.h``).

Server side: :class:`NativeRpcFrontend` serves every unary method of an :class:`RpcServer`'s
servicers through ``_C.FrameRpcServer``: C++ I/O threads decode frames and queue them per *lane*;
Python dispatcher threads take a batch per GIL acquisition, run the same servicer method the gRPC
handler would (same user binding, gate, error -> status mapping) and send the serialized reply.
Read-only metadata methods use the ``fast`` lane (few threads, large batches: nothing in them
blocks); the namespace mutations of the client hot path use the ``mutation`` lane (few threads,
batches: with the flush deferred they do not block either — many threads contending for the GIL
cost more than they overlap); everything else (UFS-bound, job, worker-sync calls) uses the
``blocking`` lane (many threads, one request each).  A mutation does not park its thread until
its journal entries are durable: the handler runs under :class:`journal.system.deferred_flush` and
the reply is sent from the journal's flush callback, so one flush batch answers every mutation it
carries (group commit) while the dispatcher threads go on decoding and applying requests.

Replies of ``GetStatus`` / ``ListStatus`` calls that never sync with the UFS are also kept in the
server's native reply cache, keyed by (method, user, request bytes) and versioned by the master's
metadata epoch (bumped inside every namespace / block-location / mount-table change): a repeat call
is answered on the C++ I/O thread without entering Python.

Client side: :class:`NativeChannelCore` wraps ``_C.FrameRpcClient`` (connection pool, GIL released
for the whole call).  :class:`alluxio_amd.rpc.Channel` switches its unary methods to it once the
server advertised a native port (``getServiceVersion`` -> ``nativeRpcPort``).
"""
from __future__ import annotations

import atexit
import logging
import os
import threading
import time
import weakref

from ..journal.system import deferred_flush
from ..proto import SERVICES
from ..utils import exceptions as ex
from ..utils import optiming as _OPT

LOG = logging.getLogger(__name__)

# methods that never block on a journal flush, UFS call or lock wait beyond the namespace lock
FAST_METHODS = frozenset({
    "GetStatus", "ListStatus", "Exists", "CheckAccess", "GetMountTable", "GetFilePath", "GetSyncPathList",
    "getServiceVersion", "GetBlockInfo", "GetWorkerInfoList", "GetCapacityBytes", "GetUsedBytes",
    "GetBlockMasterInfo", "GetConfiguration", "GetMasterInfo", "GetStateLockHolders", "GetPinnedFileIds",
    "GetUfsInfo", "GetFileInfo",
})
# read-only methods whose replies the native cache may keep (see _cacheable)
CACHEABLE_METHODS = frozenset({"GetStatus", "ListStatus"})
# namespace mutations of the client hot path: CPU-only apart from the (deferred) journal flush
MUTATION_METHODS = frozenset({
    "CreateFile", "CompleteFile", "Remove", "Rename", "CreateDirectory", "SetAttribute",
    "GetNewBlockIdForFile",
})
FS_SERVICE = "alluxio.grpc.file.FileSystemMasterClientService"
SASL_SERVICE = "alluxio.grpc.sasl.SaslAuthenticationService"
# services a gRPC caller reaches without an authenticated channel (rpc._UNAUTH_SERVICES)
UNAUTH_SERVICES = frozenset({SASL_SERVICE, "alluxio.grpc.version.ServiceVersionClientService"})
LANE_FAST, LANE_BLOCKING, LANE_MUTATION, LANE_STREAM = 0, 1, 2, 3
AUTH_PATH = "@auth"
_LIVE: "weakref.WeakSet[NativeRpcFrontend]" = weakref.WeakSet()


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NULL = _NullCtx()


@atexit.register
def _stop_all() -> None:
    # dispatcher threads sit in C++ with the GIL released: stop them before the interpreter
    # finalizes (a daemon thread re-entering a finalized interpreter aborts the process)
    for fe in list(_LIVE):
        try:
            fe.stop()
        except Exception:  # noqa: BLE001
            pass


def _cacheable(req) -> bool:
    """The reply depends only on metadata state and the caller: no UFS sync is requested."""
    o = req.options
    if o.HasField("loadMetadataType") and o.loadMetadataType == 2:   # ALWAYS
        return False
    c = o.commonOptions if o.HasField("commonOptions") else None
    return c is None or not c.HasField("syncIntervalMs") or c.syncIntervalMs < 0
# services whose server-streaming methods are served natively (bounded metadata replies)
STREAM_SERVICES = frozenset({"alluxio.grpc.file.FileSystemMasterClientService"})


class _Ctx:
    """ServicerContext stand-in (the servicers only read metadata / abort)."""

    def __init__(self, user, internal: bool = False):
        self._md = (("alluxio-user", user),) if user else ()
        # posted by a native stream of this server (NativeStream::on_end), not sent by a client
        self.internal = internal

    def invocation_metadata(self):
        return self._md

    def is_active(self):
        return True

    def abort(self, code, details):
        raise ex.AlluxioStatusException.from_status(code.value[0] if hasattr(code, "value") else code, details)

    def set_code(self, code):
        pass

    def set_details(self, details):
        pass

    def peer(self):
        return "native"


def auth_payload(auth) -> bytes:
    """Handshake payload for ``Channel.auth`` = (type, user, password) or None (NOSASL)."""
    if auth is None:
        return b"NOSASL\0\0"
    t, user, password = auth
    return f"{t}\0{user or ''}\0{password or ''}".encode()


class NativeRpcFrontend:
    """``services``: serve only these services (default: every servicer of ``rpc_server``).
    ``bridge_services``: their client-/bidi-streaming and data-streaming methods are served too,
    bridged call by call to the Python servicer (kind 2: request messages pulled with
    ``stream_recv``, responses pushed with ``stream_send``, one pool thread per live call) -- the
    worker's data port serves the whole BlockWorker service this way, with ReadBlock answered in
    C++ whenever the block is in the store (csrc/data_server.cpp)."""

    def __init__(self, rpc_server, host: str, port: int = 0, fast_threads: int = 2, blocking_threads: int = 32,
                 io_threads: int = 2, batch: int = 64, mutation_threads: int = 2, mutation_batch: int = 16,
                 reply_cache: bool = True, epoch_source=None, services=None, bridge_services=(),
                 stream_threads: int = 128):
        from ..ops.native import lib
        self.rpc = rpc_server
        self.methods = [(AUTH_PATH, None, None)]
        lanes = [0]
        kinds = [0]
        servicers = dict(rpc_server._servicers)
        if services is not None:
            servicers = {k: v for k, v in servicers.items() if k in services}
        if rpc_server.authenticator is not None:
            servicers[SASL_SERVICE] = rpc_server.authenticator   # as RpcServer.start installs it
        bridge_services = frozenset(bridge_services)
        for svc, servicer in servicers.items():
            for name, spec in SERVICES[svc].items():
                # unary requests; a server-streaming reply of a metadata service travels as one
                # frame of length-prefixed messages.  The SASL handshake (one client message, one
                # reply) serves gRPC connections.  Streaming calls of a bridged service (data
                # streams) get the kind-2 bridge.
                if not hasattr(servicer, name):
                    continue
                kind = 1 if spec.server_streaming else 0
                if svc in bridge_services and (spec.client_streaming or spec.server_streaming):
                    kind = 2
                elif spec.client_streaming and svc != SASL_SERVICE:
                    continue
                elif spec.server_streaming and svc not in STREAM_SERVICES and svc != SASL_SERVICE:
                    continue
                self.methods.append((spec.path, spec, getattr(servicer, name)))
                kinds.append(kind)
                lanes.append(LANE_STREAM if kind == 2 else
                             LANE_FAST if name in FAST_METHODS or svc == SASL_SERVICE else
                             LANE_MUTATION if name in MUTATION_METHODS and svc == FS_SERVICE else LANE_BLOCKING)
        self.server = lib().FrameRpcServer(host, port, [m[0] for m in self.methods], lanes, io_threads)
        for i, k in enumerate(kinds):
            if k:
                self.server.set_method_kind(i, k)
        self.kinds = kinds
        self.stream_threads = max(1, stream_threads)
        self._stream_exec = None
        self._auth_hooked = False
        auth = rpc_server.authenticator
        if auth is not None and bridge_services:
            # calls answered in C++ (ReadBlock) check the caller's channel-id against the channels
            # the SASL service authenticated (mirrored from the Python authenticator)
            lib().set_require_channel_auth(self.server, True)
            auth.add_listener(self._on_channel)
            self._auth_hooked = True
        self.fast_threads, self.blocking_threads, self.batch = fast_threads, blocking_threads, batch
        self.mutation_threads, self.mutation_batch = max(1, mutation_threads), max(1, mutation_batch)
        self.lanes = lanes
        # reply cache: needs a master that reports its metadata changes (epoch_source =
        # FileSystemMaster.add_epoch_listener)
        self.cacheable = [False] * len(self.methods)
        if reply_cache and epoch_source is not None:
            epoch_source(self.server.bump_epoch)
            for i, (path, spec, _fn) in enumerate(self.methods):
                if spec is not None and spec.name in CACHEABLE_METHODS:
                    self.cacheable[i] = True
                    self.server.set_cacheable(i, True)
        self._threads: list[threading.Thread] = []
        self._running = False
        self.port = None
        self._after_init = threading.Lock()
        self.spilled = 0

    def method_index(self, path: str) -> int:
        for i, (p, _spec, _fn) in enumerate(self.methods):
            if p == path:
                return i
        raise KeyError(path)

    def _on_channel(self, cid: str, user: str | None) -> None:
        from ..ops.native import lib
        if user is None:
            lib().revoke_channel(self.server, cid)
        else:
            lib().allow_channel(self.server, cid, user)

    def start(self) -> int:
        self.server.start()
        self.port = self.server.port
        self._running = True
        _LIVE.add(self)
        lanes = [(LANE_FAST, self.fast_threads, self.batch), (LANE_BLOCKING, self.blocking_threads, 1),
                 (LANE_MUTATION, self.mutation_threads, self.mutation_batch)]
        if any(k == 2 for k in self.kinds):
            import concurrent.futures as cf
            self._stream_exec = cf.ThreadPoolExecutor(self.stream_threads, thread_name_prefix="native-stream")
            lanes.append((LANE_STREAM, 1, 64))
        for lane, n, batch in lanes:
            for i in range(n):
                t = threading.Thread(target=self._loop, args=(lane, batch), daemon=True,
                                     name=f"native-rpc-{lane}-{i}")
                t.start()
                self._threads.append(t)
        return self.port

    def stop(self) -> None:
        if not self._running:
            return
        self._running = False
        if self._auth_hooked:
            self.rpc.authenticator.remove_listener(self._on_channel)
            self._auth_hooked = False
        self.server.stop()
        for t in self._threads:
            t.join(timeout=2)
        self._threads = []
        for name in ("_spill_exec", "_after_exec", "_stream_exec"):
            pool = getattr(self, name, None)
            if pool is not None:
                pool.shutdown(wait=False)
                setattr(self, name, None)

    # ---- dispatch -------------------------------------------------------------------------------
    def _auth(self, token, payload: bytes):
        parts = payload.split(b"\0")
        atype, user, password = (p.decode() for p in (parts + [b"", b"", b""])[:3])
        if user and user[0] < " ":
            # "\x01..." / "\x02..." caller strings are how the server marks gRPC-connection and
            # internal (native-stream) requests: a client name may not start like one
            raise ex.UnauthenticatedException("invalid user name")
        auth = self.rpc.authenticator
        if auth is not None:
            if atype.upper() != auth.auth_type:
                raise ex.UnauthenticatedException(f"client uses {atype} authentication, server expects "
                                                  f"{auth.auth_type}")
            auth.provider.authenticate(user, password)
        self.server.set_user(token, user)

    def _grpc_user(self, spec, user: str):
        """The caller of a gRPC-connection request (user = "\\x01" channel-id "\\0" alluxio-user),
        resolved as the gRPC handlers do (rpc._Handler._enter): NOSASL trusts the alluxio-user
        header, otherwise the user is the one the channel authenticated as."""
        cid, _, auser = user[1:].partition("\0")
        auth = self.rpc.authenticator
        if auth is None:
            return auser or None
        if spec.service in UNAUTH_SERVICES:
            return None
        return auth.user_for(cid or None)

    def _one(self, token, midx, user, payload, nonblocking: bool = False, carried: dict | None = None):
        """Run one request; returns the reply tuple, or None when the reply is deferred until
        the journal entries the handler appended are durable (sent by the flush callback), or
        when the request moved to the spill pool.

        ``nonblocking`` (fast and mutation lanes): a handler that would wait on a namespace path
        lock or start UFS I/O raises ``WouldBlock`` before applying anything; the request is then
        re-run on the spill pool (``alluxio.master.native.rpc.blocking.threads`` threads) so the
        lanes keep serving other paths (reference: a slow UFS stalls only its own RPC thread)."""
        from ..master.inode_lock import WouldBlock, nonblocking_lane
        from ..security import as_user
        from ..utils import optiming
        t_start = time.perf_counter() if optiming.ENABLED else 0.0
        c_start = time.thread_time() if optiming.ENABLED else 0.0
        pending = None
        after = None
        cache_ep = None
        key_user = user
        try:
            if midx == 0:
                self._auth(token, payload)
                return (token, 0, "", b"")
            path, spec, fn = self.methods[midx]
            key_user = user     # the reply cache is keyed by the connection's caller string
            internal = bool(user) and user[0] == "\x02"
            if internal:
                user = user[1:]
            if user and user[0] == "\x01":
                user = self._grpc_user(spec, user)
            elif self.rpc.authenticator is not None and not user:
                raise ex.UnauthenticatedException("native channel is not authenticated")
            self.rpc.check(spec)
            req = spec.request.FromString(payload)
            cache_ep = self.server.epoch() if self.cacheable[midx] and _cacheable(req) else None
            with as_user(user or None), deferred_flush() as d, (nonblocking_lane() if nonblocking else _NULL):
                pending = d.pending
                after = d.after
                if carried:
                    pending.update(carried)
                if spec.server_streaming:
                    parts = []
                    for m in fn(iter([req]) if spec.client_streaming else req, _Ctx(user)):
                        b = m.SerializeToString()
                        parts.append(len(b).to_bytes(4, "little"))
                        parts.append(b)
                    body = b"".join(parts)
                else:
                    body = fn(req, _Ctx(user, internal)).SerializeToString()
            if cache_ep is not None and not pending:
                self.server.cache_put(midx, key_user, payload, body, cache_ep)
            reply = (token, 0, "", body)
        except WouldBlock:
            self.spilled += 1
            self._spill_pool().submit(self._spilled, token, midx, user, payload, dict(pending or {}))
            return None
        except Exception as e:  # noqa: BLE001
            se = ex.wrap(e)
            if not isinstance(e, ex.AlluxioStatusException):
                LOG.debug("native rpc %s failed", self.methods[midx][0], exc_info=True)
            reply = (token, int(se.status), se.message or str(se), b"")
            if cache_ep is not None and not pending and isinstance(e, ex.NotFoundException):
                # "does not exist" of a ONCE lookup: as stable as the UFS absent-path cache
                # behind it (a create, load, sync change or remount bumps the epoch)
                self.server.cache_put(midx, key_user, payload, b"", cache_ep, reply[1], reply[2])
        if optiming.ENABLED and midx:
            optiming.add("handler:" + self.methods[midx][0].rsplit("/", 1)[-1], time.perf_counter() - t_start)
            optiming.add("cpu_one:" + self.methods[midx][0].rsplit("/", 1)[-1], time.thread_time() - c_start)
        if pending:
            self._defer(pending, reply, after, self.methods[midx][0].rsplit("/", 1)[-1] if optiming.ENABLED else "")
            return None
        return reply

    def _run_after(self, after: list, reply) -> None:
        """after_durable callbacks of a flushed RPC, then its reply (off the journal flush
        thread: a callback may append + flush journal entries itself)."""
        for cb in after:
            try:
                cb()
            except Exception:  # noqa: BLE001
                LOG.exception("post-journal callback failed")
        self.server.respond_many([reply])

    def _defer(self, pending: dict, reply, after: list | None = None, name: str = "") -> None:
        """Send ``reply`` once every journal writer in ``pending`` flushed past its counter
        (after running the RPC's after_durable callbacks; on a failed flush they never run)."""
        if len(pending) == 1 and not after:
            (w, counter), = pending.items()
            rwf = getattr(w, "reply_when_flushed", None)
            if rwf is not None:          # common case: batched reply from the flush thread
                rwf(counter, self.server, reply)
                return
        left = [len(pending)]
        err = [None]
        lock = threading.Lock()
        srv = self.server
        t_defer = time.perf_counter() if name else 0.0

        def done(e):
            with lock:
                if e is not None and err[0] is None:
                    err[0] = e
                left[0] -= 1
                last = left[0] == 0
            if not last:
                return
            if name:
                from ..utils import optiming
                optiming.add("journal_wait:" + name, time.perf_counter() - t_defer)
            if err[0] is None:
                if after:
                    self._after_pool().submit(self._run_after, list(after), reply)
                else:
                    srv.respond_many([reply])
            else:
                se = ex.wrap(err[0])
                srv.respond_many([(reply[0], int(se.status), se.message or str(se), b"")])

        for w, counter in pending.items():
            w.flush_async(counter, done)

    def _spilled(self, token, midx, user, payload, carried) -> None:
        reply = self._one(token, midx, user, payload, nonblocking=False, carried=carried)
        if reply is not None:
            self.server.respond_many([reply])

    def _spill_pool(self):
        pool = getattr(self, "_spill_exec", None)
        if pool is None:
            import concurrent.futures as cf
            with self._after_init:
                pool = getattr(self, "_spill_exec", None)
                if pool is None:
                    pool = self._spill_exec = cf.ThreadPoolExecutor(
                        max(4, self.blocking_threads), thread_name_prefix="native-rpc-spill")
        return pool

    def _after_pool(self):
        pool = getattr(self, "_after_exec", None)
        if pool is None:
            import concurrent.futures as cf
            with self._after_init:
                pool = getattr(self, "_after_exec", None)
                if pool is None:
                    pool = self._after_exec = cf.ThreadPoolExecutor(2, thread_name_prefix="rpc-after-durable")
        return pool

    # ---- kind-2 bridge: one pool thread runs a streaming call of the Python servicer ------------
    def _run_stream(self, token, midx, user, payload) -> None:
        from ..ops.native import lib
        from ..security import as_user
        from . import marshal
        C = lib()
        srv = self.server
        _path, spec, fn = self.methods[midx]
        des = marshal.marshallers(spec, True)[1]
        it = None
        try:
            if user and user[0] == "\x01":
                user = self._grpc_user(spec, user)
            elif self.rpc.authenticator is not None and not user:
                raise ex.UnauthenticatedException("native channel is not authenticated")
            self.rpc.check(spec)
            first = des(payload)

            def requests():
                yield first
                while True:
                    rc, data = C.stream_recv(srv, token, 1000)
                    if rc == 0:
                        yield des(data)
                    elif rc == 1:
                        return
                    elif rc == 2:
                        raise ex.CancelledException("call cancelled by the client")
                    elif not self._running:
                        raise ex.UnavailableException("server stopping")

            with as_user(user or None):
                arg = requests() if spec.client_streaming else first
                if spec.server_streaming:
                    it = fn(arg, _Ctx(user))
                    for m in it:
                        if not C.stream_send(srv, token, m.SerializeToString(), 60_000):
                            return          # cancelled: the generator is closed below
                else:
                    r = fn(arg, _Ctx(user))
                    if not C.stream_send(srv, token, r.SerializeToString(), 60_000):
                        return
            C.stream_finish(srv, token, 0, "")
        except Exception as e:  # noqa: BLE001
            se = ex.wrap(e)
            if not isinstance(e, ex.AlluxioStatusException):
                LOG.debug("native stream %s failed", self.methods[midx][0], exc_info=True)
            C.stream_finish(srv, token, int(se.status), se.message or str(se))
        finally:
            if it is not None and hasattr(it, "close"):
                try:
                    it.close()
                except Exception:  # noqa: BLE001
                    pass
            C.stream_finish(srv, token, 1, "call ended")   # no-op once finished

    def _loop(self, lane: int, batch: int) -> None:
        prof_path = os.environ.get("ALLUXIO_LANE_PROFILE")
        if prof_path:                  # per-lane-thread cProfile (diagnostics: where handler time goes)
            import cProfile
            pr = cProfile.Profile()
            out = f"{prof_path}.lane{lane}.{threading.get_ident()}"
            nxt = [time.monotonic() + 2.0]

            def tick():                # dump every 2 s from this thread (the master is SIGTERMed)
                if time.monotonic() >= nxt[0]:
                    pr.dump_stats(out)
                    pr.enable()
                    nxt[0] = time.monotonic() + 2.0
            pr.enable()
            try:
                self._loop_inner(lane, batch, tick)
            finally:
                pr.disable()
                pr.dump_stats(out)
            return
        self._loop_inner(lane, batch)

    def _loop_inner(self, lane: int, batch: int, tick=None) -> None:
        srv = self.server
        metrics = self.rpc.metrics
        while self._running:
            try:
                reqs = srv.poll(lane, batch, 100)
            except Exception:  # noqa: BLE001 - server stopped
                if not self._running:
                    return
                time.sleep(0.01)
                continue
            if not reqs:
                continue
            if lane == LANE_STREAM:
                for r in reqs:
                    self._stream_exec.submit(self._run_stream, *r)
                continue
            t0 = time.perf_counter()
            c0 = time.thread_time() if tick is not None or _OPT.ENABLED else 0.0
            nb = lane != LANE_BLOCKING
            out = [o for o in (self._one(*r, nonblocking=nb) for r in reqs) if o is not None]
            if out:
                srv.respond_many(out)
            if _OPT.ENABLED:
                _OPT.add(f"cpu_batch:lane{lane}", time.thread_time() - c0)
                _OPT.add(f"batch_size:lane{lane}", len(reqs) * 1e-6)     # reported in "us" = count
            if metrics is not None:
                metrics.counter("NativeRpcCalls").inc(len(reqs))
                metrics.timer("NativeRpcBatch").update(time.perf_counter() - t0)
            if tick is not None:
                tick()


class NativeChannelCore:
    """Client half: one pooled native connection set to ``host:port``."""

    def __init__(self, host: str, port: int, auth, timeout_ms: int = 60_000):
        from ..ops.native import lib
        self.client = lib().FrameRpcClient(host, port, auth_payload(auth), timeout_ms)
        self.address = f"{host}:{port}"

    def method(self, spec):
        return _NativeMethod(self, spec)

    def close(self) -> None:
        self.client.close()


class _NativeMethod:
    __slots__ = ("core", "spec", "path", "des", "stream")

    def __init__(self, core: NativeChannelCore, spec):
        self.core = core
        self.spec = spec
        self.path = spec.path
        self.des = spec.response.FromString
        self.stream = spec.server_streaming

    def __call__(self, request, timeout=None, metadata=None):
        try:
            status, msg, payload = self.core.client.call(self.path, request.SerializeToString(),
                                                         int(timeout * 1000) if timeout else 0)
        except RuntimeError as e:
            raise ex.UnavailableException(str(e)) from None
        if status:
            raise ex.AlluxioStatusException.from_status(status, msg)
        if self.stream:
            out, pos, n = [], 0, len(payload)
            while pos < n:
                ln = int.from_bytes(payload[pos:pos + 4], "little")
                out.append(self.des(payload[pos + 4:pos + 4 + ln]))
                pos += 4 + ln
            return out
        return self.des(payload)
