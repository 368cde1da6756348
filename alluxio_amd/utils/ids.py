"""Identifier schemes.

Block ids follow the reference's 64-bit layout exactly (core/common/src/main/java/alluxio/master/
block/BlockId.java:15-60): a 40-bit *container id* in the high bits and a 24-bit *sequence number*
in the low bits.  A file's id is its container id with the maximum sequence number, so every
block id maps back to the owning file id without a lookup.  Keeping this identical keeps journals
and wire messages interchangeable with reference clients.
"""
from __future__ import annotations

import itertools
import os
import random
import threading
import uuid

CONTAINER_ID_BITS = 40
SEQUENCE_NUMBER_BITS = 64 - CONTAINER_ID_BITS
CONTAINER_ID_MASK = (1 << CONTAINER_ID_BITS) - 1
SEQUENCE_NUMBER_MASK = (1 << SEQUENCE_NUMBER_BITS) - 1
MAX_SEQUENCE_NUMBER = SEQUENCE_NUMBER_MASK

_INT64_SIGN = 1 << 63


def _to_signed64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v & _INT64_SIGN else v


def create_block_id(container_id: int, sequence_number: int) -> int:
    return _to_signed64(((container_id & CONTAINER_ID_MASK) << SEQUENCE_NUMBER_BITS)
                        | (sequence_number & SEQUENCE_NUMBER_MASK))


def get_container_id(block_id: int) -> int:
    return (block_id >> SEQUENCE_NUMBER_BITS) & CONTAINER_ID_MASK


def get_sequence_number(block_id: int) -> int:
    return block_id & SEQUENCE_NUMBER_MASK


def get_file_id(block_id: int) -> int:
    return create_block_id(get_container_id(block_id), MAX_SEQUENCE_NUMBER)


def create_file_id(container_id: int) -> int:
    return create_block_id(container_id, MAX_SEQUENCE_NUMBER)


class IdGenerator:
    """Thread-safe monotonically increasing id source (reference ``IdUtils`` counters)."""

    def __init__(self, start: int = 0):
        self._it = itertools.count(start)
        self._lock = threading.Lock()

    def next(self) -> int:
        with self._lock:
            return next(self._it)


_session_gen = IdGenerator(1)
_rng = random.Random(os.getpid() ^ int.from_bytes(os.urandom(4), "little"))

INVALID_WORKER_ID = -1
INVALID_SESSION_ID = -1
INVALID_BLOCK_ID = -1

# Reserved session ids used by internal worker tasks (reference Sessions.java constants).
MIGRATE_DATA_SESSION_ID = -3
ASYNC_CACHE_UFS_SESSION_ID = -4
ASYNC_CACHE_REMOTE_SESSION_ID = -5
CACHE_UFS_SESSION_ID = -6
MASTER_COMMAND_SESSION_ID = -7
ACCESS_BLOCK_SESSION_ID = -8


def create_session_id() -> int:
    """Positive random session id (reference ``IdUtils.createSessionId``)."""
    return _rng.randrange(1, 1 << 62)


def get_random_non_negative_long() -> int:
    return _rng.randrange(0, 1 << 63)


def create_rpc_id() -> str:
    return uuid.uuid4().hex


def create_mount_id() -> int:
    return get_random_non_negative_long()
