"""Compact schema language -> protobuf descriptors -> message classes (no ``protoc`` needed).

The reference's wire contract is a set of proto2 files (core/transport/src/main/proto/**).  This
image has neither ``protoc`` nor ``grpc_tools``, so the schema is written in a terse line format
and turned into ``FileDescriptorProto``s at import time; the resulting message classes are the
regular upb/python protobuf classes and serialise byte-identically to what protoc would generate
for the same field numbers, types and labels.

Line format (``#`` starts a comment, indented lines continue the previous declaration)::

    package alluxio.grpc.block
    enum RequestType ALLUXIO_BLOCK=0 UFS_FILE=1 UFS_FALLBACK_BLOCK=2
    msg ReadRequest block_id=1:i64 offset=2:i64 chunk_size=5:i64
        open_ufs_block_options=6:alluxio.proto.dataserver.OpenUfsBlockOptions
    msg WriteRequest command=1:WriteRequestCommand|value chunk=2:Chunk|value   # oneof "value"
    msg Metric tags=6:{str,str} metricType=5:MetricType!                        # map, required
    msg FileInfo blockIds=13:i64* ttlAction=22:TtlAction@DELETE                  # repeated, default
    rpc BlockWorker ReadBlock *ReadRequest *ReadResponse                         # * = stream
"""
from __future__ import annotations

import re

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto

SCALARS = {
    "i32": F.TYPE_INT32, "i64": F.TYPE_INT64, "u32": F.TYPE_UINT32, "u64": F.TYPE_UINT64,
    "si32": F.TYPE_SINT32, "si64": F.TYPE_SINT64, "bool": F.TYPE_BOOL, "str": F.TYPE_STRING,
    "bytes": F.TYPE_BYTES, "f64": F.TYPE_DOUBLE, "f32": F.TYPE_FLOAT,
    "fx32": F.TYPE_FIXED32, "fx64": F.TYPE_FIXED64, "sfx32": F.TYPE_SFIXED32, "sfx64": F.TYPE_SFIXED64,
}

_FIELD = re.compile(
    r"^(?P<name>\w+)=(?P<num>\d+):(?P<type>\{[\w.]+,[\w.]+\}|[\w.]+)"
    r"(?P<mods>[*!]?)(?:\|(?P<oneof>\w+))?(?:@(?P<default>[\w.\-]+))?$")


class Schema:
    """Collects packages, resolves type names, registers descriptors in a private pool."""

    def __init__(self):
        self.packages: dict[str, list[tuple]] = {}
        self.symbols: dict[str, str] = {}   # full name -> "msg" | "enum"
        self.owner: dict[str, str] = {}     # full name -> package
        self.services: dict[str, list[tuple]] = {}
        self.pool = descriptor_pool.DescriptorPool()
        self.classes: dict[str, type] = {}

    # --- parsing ----------------------------------------------------------------------------
    def add(self, text: str) -> None:
        decls: list[str] = []
        for raw in text.splitlines():
            line = raw.split("#", 1)[0].rstrip()
            if not line.strip():
                continue
            if raw[:1].isspace() and decls:
                decls[-1] += " " + line.strip()
            else:
                decls.append(line.strip())
        pkg = None
        for d in decls:
            toks = d.split()
            kind = toks[0]
            if kind == "package":
                pkg = toks[1]
                self.packages.setdefault(pkg, [])
                continue
            if pkg is None:
                raise ValueError("schema declaration before 'package'")
            if kind in ("msg", "enum"):
                full = f"{pkg}.{toks[1]}"
                if full in self.symbols:
                    raise ValueError(f"duplicate schema symbol {full}")
                self.symbols[full] = kind
                self.owner[full] = pkg
                self.packages[pkg].append((kind, toks[1], toks[2:]))
            elif kind == "rpc":
                self.services.setdefault(f"{pkg}.{toks[1]}", []).append(tuple(toks[2:5]))
                self.packages[pkg].append(("rpc", toks[1], toks[2:5]))
            else:
                raise ValueError(f"unknown schema declaration {kind!r}")

    def _resolve(self, pkg: str, name: str) -> str:
        if name in self.symbols:
            return name
        full = f"{pkg}.{name}"
        if full in self.symbols:
            return full
        # walk up the package chain: alluxio.grpc.block -> alluxio.grpc
        parts = pkg.split(".")
        while parts:
            cand = ".".join(parts + [name])
            if cand in self.symbols:
                return cand
            parts.pop()
        raise KeyError(f"unresolved schema type {name!r} in package {pkg}")

    # --- building ---------------------------------------------------------------------------
    @staticmethod
    def _file_name(pkg: str) -> str:
        return pkg.replace(".", "/") + ".amdproto"

    def build(self) -> None:
        files: dict[str, descriptor_pb2.FileDescriptorProto] = {}
        deps: dict[str, set[str]] = {}
        for pkg, decls in self.packages.items():
            fdp = descriptor_pb2.FileDescriptorProto(
                name=self._file_name(pkg), package=pkg, syntax="proto2")
            dset: set[str] = set()
            services: dict[str, descriptor_pb2.ServiceDescriptorProto] = {}
            for kind, name, body in decls:
                if kind == "enum":
                    e = fdp.enum_type.add(name=name)
                    for tok in body:
                        k, v = tok.split("=")
                        e.value.add(name=k, number=int(v))
                elif kind == "msg":
                    self._build_message(pkg, fdp.message_type.add(name=name), body, dset)
                else:
                    svc = services.get(name)
                    if svc is None:
                        svc = services[name] = fdp.service.add(name=name)
                    meth, req, resp = body
                    cs, ss = req.startswith("*"), resp.startswith("*")
                    rq, rs = self._resolve(pkg, req.lstrip("*")), self._resolve(pkg, resp.lstrip("*"))
                    for t in (rq, rs):
                        if self.owner[t] != pkg:
                            dset.add(self.owner[t])
                    svc.method.add(name=meth, input_type="." + rq, output_type="." + rs,
                                   client_streaming=cs, server_streaming=ss)
            deps[pkg] = dset
            files[pkg] = fdp
        for pkg, dset in deps.items():
            for d in sorted(dset):
                files[pkg].dependency.append(self._file_name(d))
        done: set[str] = set()

        def add(pkg: str, stack=()):
            if pkg in done:
                return
            if pkg in stack:
                raise ValueError(f"schema package cycle: {' -> '.join(stack + (pkg,))}")
            for d in sorted(deps[pkg]):
                add(d, stack + (pkg,))
            self.pool.Add(files[pkg])
            done.add(pkg)
        for pkg in files:
            add(pkg)
        for full, kind in self.symbols.items():
            if kind == "msg":
                desc = self.pool.FindMessageTypeByName(full)
                self.classes[full] = message_factory.GetMessageClass(desc)

    def _build_message(self, pkg, mdp, body, dset) -> None:
        oneofs: dict[str, int] = {}
        for tok in body:
            m = _FIELD.match(tok)
            if not m:
                raise ValueError(f"bad field spec {tok!r} in {pkg}.{mdp.name}")
            name, num, typ = m.group("name"), int(m.group("num")), m.group("type")
            mods, oneof, default = m.group("mods"), m.group("oneof"), m.group("default")
            fd = mdp.field.add(name=name, number=num, json_name=name)
            if typ.startswith("{"):
                ktype, vtype = typ[1:-1].split(",")
                entry = mdp.nested_type.add(name=_map_entry_name(name))
                entry.options.map_entry = True
                self._set_type(pkg, entry.field.add(name="key", number=1, json_name="key",
                                                    label=F.LABEL_OPTIONAL), ktype, dset)
                self._set_type(pkg, entry.field.add(name="value", number=2, json_name="value",
                                                    label=F.LABEL_OPTIONAL), vtype, dset)
                fd.label = F.LABEL_REPEATED
                fd.type = F.TYPE_MESSAGE
                fd.type_name = f".{pkg}.{mdp.name}.{entry.name}"
                continue
            fd.label = {"*": F.LABEL_REPEATED, "!": F.LABEL_REQUIRED}.get(mods, F.LABEL_OPTIONAL)
            self._set_type(pkg, fd, typ, dset)
            if default is not None:
                fd.default_value = default
            if oneof:
                if oneof not in oneofs:
                    oneofs[oneof] = len(mdp.oneof_decl)
                    mdp.oneof_decl.add(name=oneof)
                fd.oneof_index = oneofs[oneof]

    def _set_type(self, pkg, fd, typ, dset) -> None:
        if typ in SCALARS:
            fd.type = SCALARS[typ]
            return
        full = self._resolve(pkg, typ)
        fd.type = F.TYPE_MESSAGE if self.symbols[full] == "msg" else F.TYPE_ENUM
        fd.type_name = "." + full
        if self.owner[full] != pkg:
            dset.add(self.owner[full])


def _map_entry_name(field: str) -> str:
    # protoc: CamelCase the field name (underscores removed, next letter upper) + "Entry"
    parts = field.split("_")
    camel = "".join(p[:1].upper() + p[1:] for p in parts if p)
    return camel + "Entry"
