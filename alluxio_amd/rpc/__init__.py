"""RPC plumbing: servers, channels and generic stubs for every proto service.

Parity: core/common/src/main/java/alluxio/grpc/{GrpcServerBuilder,GrpcChannelBuilder,
GrpcConnectionPool}.java and RpcUtils.call (core/server/common/.../RpcUtils.java:51-106 —
exception -> status mapping + per-RPC metrics).

Two transports share one code path:
* ``grpc``  — real gRPC over TCP (wire compatible with the reference's Java clients);
* ``local`` — same-process dispatch to the registered servicer, used by the minicluster and by
  a client co-located with its master/worker (no serialisation, identical semantics).
A servicer is any object whose methods are named like the RPCs and take ``(request, context)``;
client-streaming methods receive an iterator, server-streaming methods yield responses.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from concurrent import futures

import grpc

from ..proto import SERVICES
from ..utils import exceptions as ex
from . import marshal

LOG = logging.getLogger(__name__)


def _native_stream_services():
    from .native import STREAM_SERVICES
    return STREAM_SERVICES


class _LocalRegistry(dict):
    """service full name -> servicer, plus liveness/gate shared with the owning RpcServer."""

    def __init__(self, servicers, server):
        super().__init__(servicers)
        self.server = server


_LOCAL: dict[str, _LocalRegistry] = {}   # address -> registry
_LOCAL_LOCK = threading.Lock()

MAX_MESSAGE = 100 << 20

# services a client reaches through the master's native framed-RPC front end when offered
NATIVE_SERVICES = frozenset({
    "alluxio.grpc.file.FileSystemMasterClientService",
    "alluxio.grpc.block.BlockMasterClientService",
    "alluxio.grpc.meta.MetaMasterClientService",
})


class RpcContext:
    """Minimal ServicerContext stand-in for the local transport."""

    def __init__(self, metadata=None):
        self._metadata = metadata or ()
        self.cancelled = False

    def invocation_metadata(self):
        return self._metadata

    def is_active(self):
        return not self.cancelled

    def abort(self, code, details):
        raise ex.AlluxioStatusException.from_status(code.value[0] if hasattr(code, "value") else code, details)

    def set_code(self, code):
        pass

    def set_details(self, details):
        pass

    def peer(self):
        return "local"


def _status_of(e: BaseException) -> tuple[grpc.StatusCode, str]:
    se = ex.wrap(e)
    code = {s.value[0]: s for s in grpc.StatusCode}[int(se.status)]
    return code, se.message or str(se)


def _metadata(context, key: str) -> str | None:
    try:
        for k, v in context.invocation_metadata() or ():
            if k == key:
                return v
    except Exception:  # noqa: BLE001
        return None
    return None


def _user_from_metadata(context) -> str | None:
    return _metadata(context, "alluxio-user")


_UNAUTH_SERVICES = ("alluxio.grpc.sasl.SaslAuthenticationService", "alluxio.grpc.version.ServiceVersionClientService")


class _Handler:
    """Wraps servicer methods: user propagation, error mapping, metrics."""

    def __init__(self, servicer, spec, metrics=None, gate=None, authenticator=None):
        self.servicer = servicer
        self.spec = spec
        self.fn = getattr(servicer, spec.name)
        self.metrics = metrics
        self.gate = gate
        self.auth = authenticator

    def _enter(self, context):
        from ..security import as_user
        if self.auth is None:
            return as_user(_user_from_metadata(context))
        if self.spec.service in _UNAUTH_SERVICES:
            return as_user(None)
        # the user comes from the authenticated channel, never from a per-call claim
        return as_user(self.auth.user_for(_metadata(context, "channel-id")))

    def unary(self, request, context):
        t0 = time.perf_counter()
        try:
            if self.gate is not None:
                self.gate(self.spec)
            with self._enter(context):
                return self.fn(request, context)
        except ex.AlluxioStatusException as e:
            code, msg = _status_of(e)
            context.abort(code, msg)
        except Exception as e:  # noqa: BLE001
            LOG.debug("rpc %s failed", self.spec.path, exc_info=True)
            code, msg = _status_of(e)
            context.abort(code, msg)
        finally:
            if self.metrics is not None:
                self.metrics.timer(self.spec.name).update(time.perf_counter() - t0)

    def stream(self, request_or_iter, context):
        try:
            if self.gate is not None:
                self.gate(self.spec)
            with self._enter(context):
                yield from self.fn(request_or_iter, context)
        except ex.AlluxioStatusException as e:
            code, msg = _status_of(e)
            context.abort(code, msg)
        except Exception as e:  # noqa: BLE001
            LOG.debug("rpc %s failed", self.spec.path, exc_info=True)
            code, msg = _status_of(e)
            context.abort(code, msg)


class RpcServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, max_workers: int = 64, metrics=None,
                 enable_grpc: bool = True, conf=None, domain_socket: str | None = None):
        self.host = host
        # gRPC over a Unix domain socket next to TCP (AlluxioWorkerProcess domain-socket data server)
        self.domain_socket = domain_socket
        # SASL channel authentication (None = NOSASL: trust the alluxio-user header)
        self.authenticator = None
        if conf is not None:
            from ..security.authentication import ServerAuthenticator
            self.authenticator = ServerAuthenticator.from_conf(conf)
        self.port = port
        self.max_workers = max_workers
        self.metrics = metrics
        self.enable_grpc = enable_grpc
        self._servicers: dict[str, object] = {}
        # zero-copy data frames for ReadBlock/WriteBlock (alluxio.worker.network.zerocopy.enabled)
        self.zero_copy = conf is None or conf.get_bool("alluxio.worker.network.zerocopy.enabled", "true")
        self._server = None
        self.address = None
        self.alive = False
        # gate(spec) raises (e.g. UnavailableException on an HA standby) to refuse an RPC
        self.gate = None

    def check(self, spec) -> None:
        if not self.alive:
            raise ex.UnavailableException(f"server {self.address} is not serving")
        if self.gate is not None:
            self.gate(spec)

    def add_servicer(self, service_full_name: str, servicer) -> None:
        if service_full_name not in SERVICES:
            raise KeyError(f"unknown service {service_full_name}")
        self._servicers[service_full_name] = servicer

    def start(self) -> str:
        if self.authenticator is not None:
            self._servicers["alluxio.grpc.sasl.SaslAuthenticationService"] = self.authenticator
        if self.enable_grpc:
            self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=self.max_workers,
                                                                  thread_name_prefix="rpc"),
                                       options=[("grpc.max_receive_message_length", MAX_MESSAGE),
                                                ("grpc.max_send_message_length", MAX_MESSAGE),
                                                ("grpc.so_reuseport", 0)])
            for svc, servicer in self._servicers.items():
                handlers = {}
                for name, spec in SERVICES[svc].items():
                    if not hasattr(servicer, name):
                        continue
                    h = _Handler(servicer, spec, self.metrics, self.check, self.authenticator)
                    _, des, ser, _ = marshal.marshallers(spec, self.zero_copy)
                    if spec.client_streaming and spec.server_streaming:
                        handlers[name] = grpc.stream_stream_rpc_method_handler(h.stream, des, ser)
                    elif spec.client_streaming:
                        handlers[name] = grpc.stream_unary_rpc_method_handler(h.unary, des, ser)
                    elif spec.server_streaming:
                        handlers[name] = grpc.unary_stream_rpc_method_handler(h.stream, des, ser)
                    else:
                        handlers[name] = grpc.unary_unary_rpc_method_handler(h.unary, des, ser)
                self._server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(svc, handlers),))
            bound = self._server.add_insecure_port(f"{self.host}:{self.port}")
            if bound == 0:
                raise OSError(f"cannot bind {self.host}:{self.port}")
            self.port = bound
            if self.domain_socket:
                import os
                os.makedirs(os.path.dirname(self.domain_socket) or ".", exist_ok=True)
                if os.path.exists(self.domain_socket):
                    os.remove(self.domain_socket)
                if not self._server.add_insecure_port(f"unix:{self.domain_socket}"):
                    raise OSError(f"cannot bind unix:{self.domain_socket}")
            self._server.start()
        elif self.port == 0:
            self.port = _alloc_local_port()
        self.address = f"{self.host}:{self.port}"
        self.alive = True
        with _LOCAL_LOCK:
            _LOCAL[self.address] = _LocalRegistry(self._servicers, self)
        return self.address

    def stop(self, grace: float = 0.5) -> None:
        self.alive = False
        with _LOCAL_LOCK:
            if self.address is not None:
                _LOCAL.pop(self.address, None)
        if self._server is not None:
            self._server.stop(grace).wait(5)
            self._server = None


_port_counter = [40000]
_DOMAIN_SOCKETS: dict[str, str] = {}


def register_domain_socket(address: str, path: str) -> None:
    """Route new gRPC channels for ``address`` over the worker's Unix domain socket."""
    with _LOCAL_LOCK:
        _DOMAIN_SOCKETS[address] = path


def unregister_domain_socket(address: str, path: str | None = None) -> None:
    with _LOCAL_LOCK:
        if path is None or _DOMAIN_SOCKETS.get(address) == path:
            _DOMAIN_SOCKETS.pop(address, None)


def domain_socket_for(address: str) -> str | None:
    with _LOCAL_LOCK:
        return _DOMAIN_SOCKETS.get(address)


def _alloc_local_port() -> int:
    with _LOCAL_LOCK:
        _port_counter[0] += 1
        return _port_counter[0]


class _LocalMethod:
    def __init__(self, servicer, spec, user, server=None):
        self.fn = getattr(servicer, spec.name)
        self.spec = spec
        self.user = user
        self.server = server

    def __call__(self, request, timeout=None, metadata=None):
        from ..security import as_user
        if self.server is not None:
            self.server.check(self.spec)
        ctx = RpcContext(metadata)
        with as_user(self.user):
            if self.spec.server_streaming:
                return [marshal.materialize(r) for r in self.fn(request, ctx)]
            return marshal.materialize(self.fn(request, ctx))


class _GrpcMethod:
    def __init__(self, callable_, spec, metadata):
        self.c = callable_
        self.spec = spec
        self.metadata = metadata

    def __call__(self, request, timeout=None, metadata=None):
        try:
            r = self.c(request, timeout=timeout, metadata=self.metadata)
            if self.spec.server_streaming:
                return list(r)
            return r
        except grpc.RpcError as e:
            raise ex.AlluxioStatusException.from_status(e.code().value[0], e.details() or str(e)) from None


class Stub:
    """``Stub(channel, 'alluxio.grpc.file.FileSystemMasterClientService').GetStatus(req)``."""

    def __init__(self, channel: "Channel", service: str):
        self._channel = channel
        self._service = service
        for name, spec in SERVICES[service].items():
            setattr(self, name, channel.method(service, spec))


class Channel:
    def __init__(self, address: str, user: str | None = None, force_grpc: bool = False, auth="default",
                 zero_copy: bool = True, native: bool = True):
        self.address = address
        self.user = user
        # unary master calls over the native framed-RPC front end when the server offers one
        self.native = native
        self._native = None
        self._native_probed = False
        if auth == "default":      # SIMPLE as the login user (servers without SASL are tolerated)
            from ..security import login_user
            auth = ("SIMPLE", user or login_user(), "")
        self.auth = auth            # (type, user, password) or None (NOSASL)
        self.channel_id = None
        # alluxio.user.streaming.zerocopy.enabled: frame-aware codecs on the block data streams
        self.zero_copy = zero_copy
        with _LOCAL_LOCK:
            local = None if force_grpc else _LOCAL.get(address)
        self.local = local
        self._grpc = None
        self._lock = threading.Lock()
        self._stubs: dict[str, Stub] = {}

    @property
    def is_local(self) -> bool:
        return self.local is not None

    def _channel(self):
        with self._lock:
            if self._grpc is None:
                target = self.address
                with _LOCAL_LOCK:
                    uds = _DOMAIN_SOCKETS.get(self.address)
                    if uds and not os.path.exists(uds):
                        # the worker that listened there is gone (its port may now be someone
                        # else's, e.g. a new master): forget the route
                        del _DOMAIN_SOCKETS[self.address]
                        uds = None
                if uds:
                    target = f"unix:{uds}"
                self._grpc = grpc.insecure_channel(target, options=[
                    ("grpc.max_receive_message_length", MAX_MESSAGE),
                    ("grpc.max_send_message_length", MAX_MESSAGE)])
                if self.auth is not None:
                    try:
                        self._authenticate(self._grpc)
                    except BaseException:
                        # not authenticated (server starting, standby, ...): the next call
                        # reconnects and authenticates again instead of going out without a channel id
                        self._grpc.close()
                        self._grpc = None
                        raise
            return self._grpc

    def _authenticate(self, ch) -> None:
        """SASL PLAIN handshake once per channel (ChannelAuthenticator.authenticate)."""
        import uuid
        from ..proto import pb
        from ..security.authentication import SCHEMES, plain_payload
        atype, user, password = self.auth
        cid = str(uuid.uuid4())
        spec = SERVICES["alluxio.grpc.sasl.SaslAuthenticationService"]["authenticate"]
        call = ch.stream_stream(spec.path, spec.request.SerializeToString, spec.response.FromString)
        msg = pb.sasl.SaslMessage(messageType=0, message=plain_payload(user or self.user or "", password),
                                  clientId=cid, channelRef=cid, authenticationScheme=SCHEMES[atype])
        try:
            for resp in call(iter([msg]), timeout=30):
                if resp.messageType == 1:
                    self.channel_id = cid
                break
        except grpc.RpcError as e:
            if e.code() == grpc.StatusCode.UNIMPLEMENTED:
                return  # NOSASL server: no channel authentication
            raise ex.AlluxioStatusException.from_status(e.code().value[0], e.details() or str(e)) from None
        if self.channel_id is None:
            raise ex.UnauthenticatedException(f"authentication with {self.address} failed")

    def _md(self):
        md = []
        if self.user:
            md.append(("alluxio-user", self.user))
        if self.channel_id:
            md.append(("channel-id", self.channel_id))
        return tuple(md) or None

    def _native_core(self):
        """Native framed-RPC connection to this server when it advertises one (probed once over
        gRPC with getServiceVersion; see rpc/native.py), else None."""
        if not self.native:
            return None
        with self._lock:
            # a server without a native port is re-probed after a while (it may enable one)
            if self._native_probed and (self._native is not None or time.time() < self._native_probed):
                return self._native
            self._native_probed = time.time() + 30.0
        core = None
        try:
            from ..proto import pb
            spec = SERVICES["alluxio.grpc.version.ServiceVersionClientService"]["getServiceVersion"]
            c = self._channel().unary_unary(spec.path, spec.request.SerializeToString, spec.response.FromString)
            r = c(pb.version.GetServiceVersionPRequest(), timeout=10, metadata=self._md())
            if r.nativeRpcPort:
                from .native import NativeChannelCore
                core = NativeChannelCore(self.address.rsplit(":", 1)[0], r.nativeRpcPort, self.auth)
        except Exception:  # noqa: BLE001 - no native front end: gRPC only
            LOG.debug("native rpc probe of %s failed", self.address, exc_info=True)
        with self._lock:
            self._native = core
        return core

    def method(self, service, spec):
        if self.local is not None:
            servicer = self.local.get(service)
            if servicer is None or not hasattr(servicer, spec.name):
                def missing(*a, **kw):
                    raise ex.UnimplementedException(f"{spec.path} not served at {self.address}")
                return missing
            return _LocalMethod(servicer, spec, self.user, getattr(self.local, "server", None))
        if not spec.client_streaming and service in NATIVE_SERVICES and \
                (not spec.server_streaming or service in _native_stream_services()):
            core = self._native_core()
            if core is not None:
                return core.method(spec)
        ch = self._channel()
        ser, des = spec.request.SerializeToString, spec.response.FromString
        if spec.client_streaming and spec.server_streaming:
            c = ch.stream_stream(spec.path, ser, des)
        elif spec.client_streaming:
            c = ch.stream_unary(spec.path, ser, des)
        elif spec.server_streaming:
            c = ch.unary_stream(spec.path, ser, des)
        else:
            c = ch.unary_unary(spec.path, ser, des)
        return _GrpcMethod(c, spec, self._md())

    def stub(self, service: str) -> Stub:
        # stubs are immutable bundles of bound methods: build one per service, not per call
        st = self._stubs.get(service)
        if st is None:
            st = self._stubs[service] = Stub(self, service)
        return st

    def raw_stream(self, service: str, method: str):
        """Direct access to a streaming callable (for flow-controlled data streams)."""
        spec = SERVICES[service][method]
        if self.local is not None:
            servicer = self.local[service]
            fn = getattr(servicer, method)
            server = getattr(self.local, "server", None)

            def call(it):
                if server is not None:
                    server.check(spec)
                return fn(it, RpcContext())
            return call
        ch = self._channel()
        ser, _, _, des = marshal.marshallers(spec, self.zero_copy)
        c = ch.stream_stream(spec.path, ser, des)
        md = self._md()
        return lambda it: c(it, metadata=md)

    def close(self) -> None:
        with self._lock:
            self._stubs = {}
            if self._native is not None:
                self._native.close()
                self._native = None
            self._native_probed = False
            if self._grpc is not None:
                self._grpc.close()
                self._grpc = None


class ChannelPool:
    """One channel per (address, user) (reference GrpcConnectionPool keyed by address)."""

    def __init__(self, conf=None):
        self._lock = threading.Lock()
        self._chans: dict[tuple, Channel] = {}
        self.conf = conf

    def get(self, address: str, user: str | None = None) -> Channel:
        key = (address, user)
        c = self._chans.get(key)       # lock-free hit: every RPC comes through here
        if c is not None:
            return c
        with self._lock:
            c = self._chans.get(key)
            if c is None:
                from ..security.authentication import client_auth_from_conf
                force = self.conf is not None and not self.conf.get_bool(
                    "alluxio.user.network.inprocess.transport.enabled", "true")
                zc = self.conf is None or self.conf.get_bool("alluxio.user.streaming.zerocopy.enabled", "true")
                nat = self.conf is None or self.conf.get_bool("alluxio.user.network.native.rpc.enabled", "true")
                c = self._chans[key] = Channel(address, user, force_grpc=force,
                                               auth=client_auth_from_conf(self.conf, user), zero_copy=zc,
                                               native=nat)
            return c

    def drop(self, address: str, user: str | None = None) -> None:
        with self._lock:
            c = self._chans.pop((address, user), None)
        if c is not None:
            c.close()

    def close(self) -> None:
        with self._lock:
            for c in self._chans.values():
                c.close()
            self._chans.clear()


def is_local_address(address: str) -> bool:
    with _LOCAL_LOCK:
        return address in _LOCAL


def local_servicer(address: str, service: str):
    with _LOCAL_LOCK:
        return _LOCAL.get(address, {}).get(service)


class _FailoverStub:
    def __init__(self, fch: "FailoverChannel", service: str):
        self._f = fch
        self._service = service

    def __getattr__(self, name):
        if name not in SERVICES[self._service]:
            raise AttributeError(name)
        f = self._f

        def call(request, timeout=None, metadata=None):
            deadline = time.time() + f.max_duration_s
            delay = 0.02
            while True:
                addr = f.current
                try:
                    return getattr(f.channel(addr).stub(self._service), name)(request, timeout=timeout)
                except (ex.UnavailableException, ex.UnimplementedException) as e:
                    if time.time() > deadline or len(f.addresses) == 0:
                        raise
                    LOG.debug("master %s unavailable for %s (%s); trying next", addr, name, e)
                    f.rotate(addr)
                    time.sleep(delay)
                    delay = min(delay * 2, 0.5)
        return call


class FailoverChannel:
    """A channel to whichever of several HA masters is primary.

    Reference: core/client/fs/.../PollingMasterInquireClient.java (probe each configured master
    address until one answers as primary) + AbstractClient.retryRPC (reconnect and retry on
    UNAVAILABLE).  Standby masters refuse every RPC with UNAVAILABLE (their RpcServer gate), so
    "answers" == "is primary"; calls rotate through the addresses with backoff until one does.
    """

    def __init__(self, addresses, user: str | None = None, pool: "ChannelPool | None" = None,
                 max_duration_s: float = 120.0):
        if isinstance(addresses, str):
            addresses = [a.strip() for a in addresses.split(",") if a.strip()]
        self.addresses = list(addresses)
        self.user = user
        self.pool = pool or ChannelPool()
        self.max_duration_s = max_duration_s
        self._i = 0
        self._lock = threading.Lock()

    @property
    def current(self) -> str:
        # lock-free read (one int + list index, GIL-atomic); rotate() mutates under the lock
        return self.addresses[self._i % len(self.addresses)]

    @property
    def address(self) -> str:
        return self.current

    @property
    def is_local(self) -> bool:
        return self.channel(self.current).is_local

    def rotate(self, failed: str) -> None:
        with self._lock:
            if self.addresses[self._i % len(self.addresses)] == failed:
                self._i += 1
                # refresh: a restarted in-process server re-registers under the same address
                self.pool.drop(failed, self.user)

    def channel(self, address: str) -> Channel:
        return self.pool.get(address, self.user)

    def stub(self, service: str) -> _FailoverStub:
        return _FailoverStub(self, service)

    def raw_stream(self, service: str, method: str):
        return self.channel(self.current).raw_stream(service, method)

    def close(self) -> None:
        pass


def master_channel(addresses, user: str | None = None, pool: "ChannelPool | None" = None,
                   max_duration_s: float = 120.0):
    """A plain Channel for one master address, a FailoverChannel for an HA address list."""
    addrs = [a.strip() for a in addresses.split(",")] if isinstance(addresses, str) else list(addresses)
    if len(addrs) == 1:
        return (pool or ChannelPool()).get(addrs[0], user) if pool else Channel(addrs[0], user)
    return FailoverChannel(addrs, user, pool, max_duration_s)
