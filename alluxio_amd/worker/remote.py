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


def _block_length(worker, block_id: int) -> int:
    """Block length from the master's block info (BlockMasterClientService.GetBlockInfo)."""
    ch = worker.master_channel
    if ch is None:
        raise ValueError(f"length of block {block_id} unknown and no master channel")
    bi = ch.stub("alluxio.grpc.block.BlockMasterClientService").GetBlockInfo(
        pb.block.GetBlockInfoPRequest(blockId=block_id)).blockInfo
    return int(bi.length)


def remote_block_fetcher(worker, host: str, port: int, length: int | None = None, chunk_size: int = 1 << 20):
    """Block source that streams ``block_id`` out of worker ``host:port``'s ``ReadBlock`` service
    into this worker (RemoteBlockReader.java + GrpcDataReader.java:123-160): the request stream
    stays open and every received chunk is acknowledged with ``offset_received``, so the source's
    flow-control window (``alluxio.worker.network.reader.buffer.size.bytes``, 4 MB) paces it;
    the channel comes from the worker's peer pool; the block length comes from the master."""
    def fetch(block_id: int) -> None:
        import queue
        n = length if length and length > 0 else _block_length(worker, block_id)
        ch = worker.peer_channel(f"{host}:{port}")
        acks: "queue.Queue" = queue.Queue()

        def requests():
            yield pb.block.ReadRequest(block_id=block_id, offset=0, length=n, chunk_size=chunk_size)
            while True:
                off = acks.get()
                if off is None:
                    return
                yield pb.block.ReadRequest(offset_received=off)

        session = ids.ASYNC_CACHE_REMOTE_SESSION_ID
        stream = ch.raw_stream("alluxio.grpc.block.BlockWorker", "ReadBlock")(requests())
        worker.create_block(session, block_id, 0, "", max(n, 1))
        pos = 0
        try:
            for resp in stream:
                data = resp.chunk.data
                worker.write_bytes(session, block_id, pos, data)
                pos += len(data)
                acks.put(pos)
                if pos >= n:
                    break
            if pos != n:
                raise IOError(f"block {block_id} from {host}:{port}: got {pos} of {n} bytes")
            worker.commit_block(session, block_id)
        except Exception:
            worker.abort_block(session, block_id)
            raise
        finally:
            acks.put(None)
            cancel = getattr(stream, "cancel", None)
            if cancel is not None and pos < n:
                cancel()
    return fetch


def peer_transfer(worker, req) -> tuple[bool, str]:
    """``PeerTransfer``: pull ``req.block_id`` from ``req.src_address`` (any same-node worker) or
    from transfer-group rank ``req.src_rank``."""
    if req.src_address:
        import time

        from ..parallel.peer import _add_time, is_same_node, pull_block
        t0 = time.perf_counter()
        try:
            host = req.src_address.rsplit(":", 1)[0]
            pull_block(worker, req.block_id, req.src_address, req.length, same_node=is_same_node(worker, host),
                       handle=req.handle if req.HasField("handle") else None)
            return True, ""
        except Exception as e:  # noqa: BLE001
            LOG.exception("peer transfer of block %d from %s failed", req.block_id, req.src_address)
            return False, str(e)
        finally:
            # the replica's handler, entry to exit (the writer's PeerTransfer round trip minus this
            # is the RPC's own cost)
            _add_time("handler", time.perf_counter() - t0)
    plane = getattr(worker, "transfer_plane", None)
    if plane is None:
        return False, "no RCCL transfer plane on this worker"
    try:
        plane.serve(req)
        return True, ""
    except Exception as e:  # noqa: BLE001
        LOG.exception("peer transfer failed")
        return False, str(e)
