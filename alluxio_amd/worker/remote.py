"""Worker-to-worker block transfer.

Parity: core/server/worker/src/main/java/alluxio/worker/block/RemoteBlockReader.java (pull a
block from another worker's ReadBlock stream) used by AsyncCacheRequestManager.java:213-240.
On a multi-GPU node the same transfer goes over RCCL/xGMI instead (alluxio_amd/parallel/
transfer.py); ``peer_transfer`` is the control-plane entry for that path.
"""
from __future__ import annotations

import logging

from ..proto import pb
from ..utils import ids

LOG = logging.getLogger(__name__)


def remote_block_fetcher(worker, host: str, port: int, length: int | None = None):
    def fetch(block_id: int) -> None:
        from ..rpc import Channel
        ch = Channel(f"{host}:{port}")
        session = ids.ASYNC_CACHE_REMOTE_SESSION_ID
        reqs = iter([pb.block.ReadRequest(block_id=block_id, offset=0, length=length or -1, chunk_size=1 << 20)])
        stream = ch.raw_stream("alluxio.grpc.block.BlockWorker", "ReadBlock")(reqs)
        worker.create_block(session, block_id, 0, "", length or (1 << 20))
        pos = 0
        try:
            for resp in stream:
                worker.write_bytes(session, block_id, pos, resp.chunk.data)
                pos += len(resp.chunk.data)
            worker.commit_block(session, block_id)
        except Exception:
            worker.abort_block(session, block_id)
            raise
    return fetch


def peer_transfer(worker, req) -> tuple[bool, str]:
    """``PeerTransfer``: pull ``req.block_id`` from ``req.src_address`` (any same-node worker) or
    from transfer-group rank ``req.src_rank``."""
    if req.src_address:
        from ..parallel.peer import is_same_node, pull_block
        try:
            host = req.src_address.rsplit(":", 1)[0]
            pull_block(worker, req.block_id, req.src_address, req.length, same_node=is_same_node(worker, host))
            return True, ""
        except Exception as e:  # noqa: BLE001
            LOG.exception("peer transfer of block %d from %s failed", req.block_id, req.src_address)
            return False, str(e)
    plane = getattr(worker, "transfer_plane", None)
    if plane is None:
        return False, "no RCCL transfer plane on this worker"
    try:
        plane.serve(req)
        return True, ""
    except Exception as e:  # noqa: BLE001
        LOG.exception("peer transfer failed")
        return False, str(e)
