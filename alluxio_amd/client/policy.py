"""Block location policies (where to write a block / which worker reads a UFS block).

Parity: core/client/fs/src/main/java/alluxio/client/block/policy/*.java — LocalFirstPolicy
(default write & UFS-read policy), LocalFirstAvoidEvictionPolicy, MostAvailableFirstPolicy,
RoundRobinPolicy, SpecificHostPolicy, DeterministicHashPolicy (consistent hashing of block ids
over workers; on a GPU node this maps a block to a fixed GPU rank).
"""
from __future__ import annotations

import hashlib
import itertools
import random
import threading


class BlockLocationPolicy:
    def get_worker(self, workers, block_id: int, block_size: int, context=None):  # pragma: no cover
        raise NotImplementedError


def _free(w) -> int:
    return w.capacityBytes - w.usedBytes


class LocalFirstPolicy(BlockLocationPolicy):
    def get_worker(self, workers, block_id, block_size, context=None):
        local = [w for w in workers if context is not None and context.is_local(w.address)]
        inproc = []
        if context is not None:
            inproc = [w for w in local if context.in_process_worker(w.address) is not None]
            if inproc:
                local = inproc
        # deterministic among several local workers (one per GPU): a file's blocks stay together
        local = sorted(local, key=lambda w: (w.address.host, w.address.rpcPort))
        cands = [w for w in local if _free(w) >= block_size] or local
        if cands:
            if not inproc and len(cands) > 1:
                # no worker in this process (e.g. picking replicas of a block whose primary is
                # ours): spread blocks over the node's GPU workers so every xGMI link carries load
                return cands[(block_id * 0x9E3779B97F4A7C15 >> 17) % len(cands)]
            return cands[0]
        fit = [w for w in workers if _free(w) >= block_size]
        return random.choice(fit or workers) if workers else None


class LocalFirstAvoidEvictionPolicy(LocalFirstPolicy):
    def __init__(self, reserved: int = 0):
        self.reserved = reserved

    def get_worker(self, workers, block_id, block_size, context=None):
        fit = [w for w in workers if _free(w) - self.reserved >= block_size]
        return super().get_worker(fit or workers, block_id, block_size, context)


class MostAvailableFirstPolicy(BlockLocationPolicy):
    def get_worker(self, workers, block_id, block_size, context=None):
        return max(workers, key=_free) if workers else None


class RoundRobinPolicy(BlockLocationPolicy):
    def __init__(self):
        self._it = itertools.count()
        self._lock = threading.Lock()

    def get_worker(self, workers, block_id, block_size, context=None):
        if not workers:
            return None
        ws = sorted(workers, key=lambda w: (w.address.host, w.address.rpcPort))
        with self._lock:
            start = next(self._it)
        for k in range(len(ws)):
            w = ws[(start + k) % len(ws)]
            if _free(w) >= block_size:
                return w
        return None


class SpecificHostPolicy(BlockLocationPolicy):
    def __init__(self, host: str, port: int | None = None):
        self.host = host
        self.port = port

    def get_worker(self, workers, block_id, block_size, context=None):
        for w in workers:
            if w.address.host == self.host and (self.port is None or w.address.rpcPort == self.port):
                return w
        return None


class DeterministicHashPolicy(BlockLocationPolicy):
    """Consistent-hash a block id onto the worker ring; ``shards`` > 1 spreads hot blocks."""

    def __init__(self, shards: int = 1, seed: int = 0):
        self.shards = max(1, shards)
        self.seed = seed

    def get_worker(self, workers, block_id, block_size, context=None):
        if not workers:
            return None
        ws = sorted(workers, key=lambda w: (w.address.host, w.address.rpcPort))
        ranked = sorted(ws, key=lambda w: hashlib.md5(
            f"{block_id}:{w.address.host}:{w.address.rpcPort}".encode()).hexdigest())
        pick = ranked[: self.shards]
        return random.Random(self.seed ^ block_id).choice(pick)


_BY_NAME = {
    "LocalFirstPolicy": LocalFirstPolicy,
    "LocalFirstAvoidEvictionPolicy": LocalFirstAvoidEvictionPolicy,
    "MostAvailableFirstPolicy": MostAvailableFirstPolicy,
    "RoundRobinPolicy": RoundRobinPolicy,
    "SpecificHostPolicy": SpecificHostPolicy,
    "DeterministicHashPolicy": DeterministicHashPolicy,
}


def create_policy(class_name: str, conf=None) -> BlockLocationPolicy:
    short = class_name.rsplit(".", 1)[-1]
    cls = _BY_NAME.get(short)
    if cls is None:
        raise ValueError(f"unknown block location policy {class_name}")
    if cls is DeterministicHashPolicy and conf is not None:
        return cls(conf.get_int("alluxio.user.ufs.block.read.location.policy.deterministic.hash.shards", 1))
    if cls is LocalFirstAvoidEvictionPolicy and conf is not None:
        return cls(conf.get_bytes("alluxio.user.block.avoid.eviction.policy.reserved.size.bytes"))
    if cls is SpecificHostPolicy:
        return cls(conf.get("alluxio.worker.hostname", "127.0.0.1") if conf else "127.0.0.1")
    return cls()
