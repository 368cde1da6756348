"""Channel authentication (SASL handshake) for the gRPC transport.

Parity: core/common/src/main/java/alluxio/security/authentication/ — AuthType (NOSASL | SIMPLE |
CUSTOM), plain/PlainSaslServer (``authzid \\0 authcid \\0 password`` payload), plain/
SimpleAuthenticationProvider (accept any user), plain/CustomAuthenticationProvider (user class from
``alluxio.security.authentication.custom.provider.class``), DefaultAuthenticationServer
(channel-id -> authenticated user registry, ``SaslAuthenticationService.authenticate`` bidi
handshake) and ChannelAuthenticator (client side: handshake once per channel, then every call
carries the ``channel-id`` header).  The server derives the RPC user from the channel registry,
not from anything the client claims per call.
"""
from __future__ import annotations

import importlib
import threading
import time

from ..utils.exceptions import UnauthenticatedException

SCHEMES = {"NOSASL": 0, "SIMPLE": 1, "CUSTOM": 2}


class AuthenticationProvider:
    def authenticate(self, user: str, password: str) -> None:  # pragma: no cover - interface
        raise NotImplementedError


class SimpleAuthenticationProvider(AuthenticationProvider):
    def authenticate(self, user: str, password: str) -> None:
        if not user:
            raise UnauthenticatedException("empty user name")


def load_custom_provider(spec: str) -> AuthenticationProvider:
    """``pkg.module:Class`` / ``pkg.module.Class`` / ``pkg.module:function(user, password)``."""
    if not spec:
        raise UnauthenticatedException("CUSTOM authentication needs "
                                       "alluxio.security.authentication.custom.provider.class")
    mod, _, attr = spec.partition(":") if ":" in spec else spec.rpartition(".")
    obj = getattr(importlib.import_module(mod), attr)
    if isinstance(obj, type):
        return obj()

    class _Fn(AuthenticationProvider):
        def authenticate(self, user, password):
            if obj(user, password) is False:
                raise UnauthenticatedException(f"user {user} rejected")
    return _Fn()


def plain_payload(user: str, password: str = "", impersonate: str = "") -> bytes:
    return f"{impersonate}\0{user}\0{password}".encode()


def parse_plain(payload: bytes) -> tuple[str, str, str]:
    parts = payload.decode(errors="replace").split("\0")
    if len(parts) != 3:
        raise UnauthenticatedException("malformed PLAIN payload")
    authz, user, password = parts
    return authz, user, password


class ServerAuthenticator:
    """Channel registry + SaslAuthenticationService servicer."""

    def __init__(self, auth_type: str, provider: AuthenticationProvider | None = None,
                 channel_ttl_s: float = 24 * 3600):
        self.auth_type = auth_type.upper()
        self.provider = provider or SimpleAuthenticationProvider()
        self.ttl = channel_ttl_s
        self._channels: dict[str, tuple[str, float]] = {}
        self._lock = threading.Lock()
        # fn(channel id, user | None): native front ends mirror the registry (data_server.cpp)
        self._listeners: list = []

    def add_listener(self, fn) -> None:
        with self._lock:
            self._listeners.append(fn)
            current = [(c, u) for c, (u, _t) in self._channels.items()]
        for c, u in current:
            fn(c, u)

    def remove_listener(self, fn) -> None:
        with self._lock:
            self._listeners = [f for f in self._listeners if f is not fn]

    def _notify(self, cid: str, user: str | None) -> None:
        for fn in list(self._listeners):
            try:
                fn(cid, user)
            except Exception:  # noqa: BLE001 - a stopped front end
                pass

    @classmethod
    def from_conf(cls, conf):
        t = conf.get("alluxio.security.authentication.type", "SIMPLE").upper()
        if t == "NOSASL":
            return None
        provider = None
        if t == "CUSTOM":
            provider = load_custom_provider(conf.get_raw("alluxio.security.authentication.custom.provider.class") or "")
        return cls(t, provider)

    def user_for(self, channel_id: str | None) -> str:
        if not channel_id:
            raise UnauthenticatedException("channel is not authenticated (no channel-id)")
        with self._lock:
            ent = self._channels.get(channel_id)
        if ent is None:
            raise UnauthenticatedException(f"channel {channel_id} is not authenticated")
        return ent[0]

    def unregister(self, channel_id: str) -> None:
        with self._lock:
            self._channels.pop(channel_id, None)
        self._notify(channel_id, None)

    def purge(self) -> int:
        cutoff = time.time() - self.ttl
        with self._lock:
            old = [c for c, (_, t) in self._channels.items() if t < cutoff]
            for c in old:
                del self._channels[c]
        for c in old:
            self._notify(c, None)
        return len(old)

    # SaslAuthenticationService.authenticate (bidi stream)
    def authenticate(self, request_iter, ctx):
        from ..proto import pb
        for msg in request_iter:
            scheme = pb.sasl.ChannelAuthenticationScheme.values_by_number[msg.authenticationScheme].name
            if scheme != self.auth_type:
                raise UnauthenticatedException(f"client uses {scheme} authentication, server expects "
                                               f"{self.auth_type}")
            authz, user, password = parse_plain(msg.message)
            self.provider.authenticate(user, password)
            # impersonation (authz != user) is not granted: the channel acts as the authenticated user
            effective = user
            cid = msg.channelRef or msg.clientId
            with self._lock:
                self._channels[cid] = (effective, time.time())
            self._notify(cid, effective)
            yield pb.sasl.SaslMessage(messageType=pb.sasl.SaslMessageType.values_by_name["SUCCESS"].number,
                                      clientId=msg.clientId, channelRef=msg.channelRef,
                                      authenticationScheme=msg.authenticationScheme)
            return


def client_auth_from_conf(conf, user: str | None):
    """(auth type, user, password) a client channel authenticates with; None for NOSASL."""
    from . import login_user
    if conf is None:
        return ("SIMPLE", user or login_user(), "")
    t = conf.get("alluxio.security.authentication.type", "SIMPLE").upper()
    if t == "NOSASL":
        return None
    return (t, user or login_user(conf), conf.get_raw("alluxio.security.login.password") or "")
