"""Wire schema registry.

``from alluxio_amd.proto import pb`` then ``pb.block.ReadRequest``, ``pb.file.FileInfo``,
``pb.journal.JournalEntry`` ...; ``services()`` lists every gRPC method with its full path
(``/alluxio.grpc.block.BlockWorker/ReadBlock``) and streaming shape.
"""
from __future__ import annotations

import types

from .defs import block, common, file, journal, meta, metric, raft, table
from .dsl import Schema

_ALIASES = {
    "alluxio.grpc": "grpc",
    "alluxio.grpc.fscommon": "fscommon",
    "alluxio.proto.shared": "shared",
    "alluxio.proto.status": "status",
    "alluxio.proto.dataserver": "dataserver",
    "alluxio.grpc.version": "version",
    "alluxio.grpc.sasl": "sasl",
    "alluxio.grpc.block": "block",
    "alluxio.grpc.file": "file",
    "alluxio.proto.journal": "journal",
    "alluxio.proto.meta": "metastore",
    "alluxio.grpc.metric": "metric",
    "alluxio.grpc.meta": "meta",
    "alluxio.grpc.job": "job",
    "alluxio.grpc.journal": "journal_master",
    "alluxio.grpc.table": "table",
    "alluxio.grpc.messaging": "messaging",
    "alluxio.proto.client": "client_cache",
    "alluxio.grpc.raft": "raft",
}

SCHEMA = Schema()
for _mod in (common, block, file, journal, metric, meta, table, raft):
    SCHEMA.add(_mod.SCHEMA)
SCHEMA.build()


def _namespace() -> types.SimpleNamespace:
    ns = types.SimpleNamespace()
    for pkg, alias in _ALIASES.items():
        setattr(ns, alias, types.SimpleNamespace())
    for full, kind in SCHEMA.symbols.items():
        pkg = SCHEMA.owner[full]
        alias = _ALIASES[pkg]
        short = full[len(pkg) + 1:]
        sub = getattr(ns, alias)
        if kind == "msg":
            setattr(sub, short, SCHEMA.classes[full])
        else:
            setattr(sub, short, SCHEMA.pool.FindEnumTypeByName(full))
    return ns


pb = _namespace()


def enum_value(enum_desc, name: str) -> int:
    return enum_desc.values_by_name[name].number


def enum_name(enum_desc, number: int) -> str:
    return enum_desc.values_by_number[number].name


class MethodSpec:
    __slots__ = ("service", "name", "path", "request", "response", "client_streaming",
                 "server_streaming")

    def __init__(self, service, name, request, response, cs, ss):
        self.service = service
        self.name = name
        self.path = f"/{service}/{name}"
        self.request = request
        self.response = response
        self.client_streaming = cs
        self.server_streaming = ss


def services() -> dict[str, dict[str, MethodSpec]]:
    out: dict[str, dict[str, MethodSpec]] = {}
    for full_svc, methods in SCHEMA.services.items():
        sd = SCHEMA.pool.FindServiceByName(full_svc)
        d = out.setdefault(full_svc, {})
        for m in sd.methods:
            d[m.name] = MethodSpec(full_svc, m.name,
                                   SCHEMA.classes[m.input_type.full_name],
                                   SCHEMA.classes[m.output_type.full_name],
                                   m.client_streaming, m.server_streaming)
    return out


SERVICES = services()
