"""Messaging transport for the embedded journal: Raft RPCs tunnelled through one bidirectional
``MessagingService.connect`` stream per peer.

Parity: core/transport/src/main/proto/grpc/messaging_transport.proto and
core/common/src/main/java/alluxio/grpc/GrpcMessagingConnection.java / GrpcMessagingClient.java /
GrpcMessagingServer.java -- the reference runs its consensus library's messages over a long-lived
bidi stream: every request carries a ``MessagingRequestHeader.requestId``, the reply echoes it in a
``MessagingResponseHeader`` (``isThrowable`` marks a failure whose text is the payload), and
replies may be matched out of order.  Here the payload is one method byte + the serialized Raft
request (RequestVote / AppendEntries / TimeoutNow).  A broken stream fails every pending call and
the next call reconnects.
"""
from __future__ import annotations

import itertools
import queue
import threading

from ..proto import pb
from ..utils.exceptions import UnavailableException

SVC_MESSAGING = "alluxio.grpc.messaging.MessagingService"
METHODS = {"RequestVote": 1, "AppendEntries": 2, "TimeoutNow": 3}
_REQ = {1: pb.raft.RequestVotePRequest, 2: pb.raft.AppendEntriesPRequest, 3: pb.raft.TimeoutNowPRequest}
_RESP = {1: pb.raft.RequestVotePResponse, 2: pb.raft.AppendEntriesPResponse, 3: pb.raft.TimeoutNowPResponse}
_CLOSE = object()


class MessagingServiceHandler:
    """Server half: answers tunnelled Raft RPCs with the node's RaftServiceHandler."""

    def __init__(self, raft_handler):
        self.h = raft_handler

    def connect(self, request_iter, ctx):
        for m in request_iter:
            rid = m.requestHeader.requestId
            try:
                code = m.message[0]
                req = _REQ[code].FromString(m.message[1:])
                name = next(k for k, v in METHODS.items() if v == code)
                resp = getattr(self.h, name)(req, ctx)
                yield pb.messaging.TransportMessage(
                    responseHeader=pb.messaging.MessagingResponseHeader(requestId=rid, isThrowable=False),
                    message=resp.SerializeToString())
            except Exception as e:  # noqa: BLE001 - reported to the caller, the stream stays up
                yield pb.messaging.TransportMessage(
                    responseHeader=pb.messaging.MessagingResponseHeader(requestId=rid, isThrowable=True),
                    message=f"{type(e).__name__}: {e}".encode())


class MessagingConnection:
    """Client half: one open stream to a peer, calls multiplexed by request id."""

    def __init__(self, channel):
        self._q: queue.Queue = queue.Queue()
        self._pending: dict[int, list] = {}
        self._lock = threading.Lock()
        self._ids = itertools.count(1)
        self.closed = False
        self._stream = channel.raw_stream(SVC_MESSAGING, "connect")(self._requests())
        self._reader = threading.Thread(target=self._read, name="raft-messaging", daemon=True)
        self._reader.start()

    def _requests(self):
        while True:
            m = self._q.get()
            if m is _CLOSE:
                return
            yield m

    def _read(self) -> None:
        err = "messaging stream closed"
        try:
            for m in self._stream:
                with self._lock:
                    slot = self._pending.pop(m.responseHeader.requestId, None)
                if slot is not None:
                    slot[1] = m
                    slot[0].set()
        except Exception as e:  # noqa: BLE001
            err = f"messaging stream failed: {e}"
        self._fail(err)

    def _fail(self, why: str) -> None:
        with self._lock:
            self.closed = True
            pending, self._pending = self._pending, {}
        for slot in pending.values():
            slot[1] = UnavailableException(why)
            slot[0].set()

    def call(self, method: str, req, timeout: float):
        if self.closed:
            raise UnavailableException("messaging stream closed")
        code = METHODS[method]
        rid = next(self._ids)
        slot = [threading.Event(), None]
        with self._lock:
            self._pending[rid] = slot
        self._q.put(pb.messaging.TransportMessage(
            requestHeader=pb.messaging.MessagingRequestHeader(requestId=rid),
            message=bytes([code]) + req.SerializeToString()))
        if not slot[0].wait(timeout):
            with self._lock:
                self._pending.pop(rid, None)
            raise UnavailableException(f"{method} timed out after {timeout:.1f}s")
        r = slot[1]
        if isinstance(r, Exception):
            raise r
        if r.responseHeader.isThrowable:
            raise UnavailableException(r.message.decode(errors="replace"))
        return _RESP[code].FromString(r.message)

    def close(self) -> None:
        self._q.put(_CLOSE)
        try:
            self._stream.cancel()
        except Exception:  # noqa: BLE001
            pass
        self._fail("messaging connection closed")
