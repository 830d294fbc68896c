"""Mesos v1 protobuf messages, built at import time from ``mesos_v1.proto``.

There is no ``protoc`` in this image, so this module carries a small ``.proto`` (proto2 subset)
parser that emits a real ``FileDescriptorProto`` and registers it in a private descriptor pool.
The resulting classes are ordinary upb-backed protobuf messages: binary serialization is
byte-compatible with the Mesos bindings the reference uses (``org.apache.mesos.Protos``), and
``google.protobuf.json_format`` gives the Mesos v1 HTTP JSON mapping for free.

Usage::

    from dcos_commons_amd.mesos import protos as P
    t = P.TaskInfo(name="hello-0-server")
    t.task_id.value = "..."
    P.TASK_RUNNING, P.Value.SCALAR, P.Offer.Operation.LAUNCH_GROUP
"""
from __future__ import annotations

import os
import re
from typing import Dict, List, Optional, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory, text_format
from google.protobuf import json_format
from google.protobuf.internal import enum_type_wrapper

_PROTO_FILE = os.path.join(os.path.dirname(__file__), "mesos_v1.proto")

_SCALAR_TYPES = {
    "double": descriptor_pb2.FieldDescriptorProto.TYPE_DOUBLE,
    "float": descriptor_pb2.FieldDescriptorProto.TYPE_FLOAT,
    "int64": descriptor_pb2.FieldDescriptorProto.TYPE_INT64,
    "uint64": descriptor_pb2.FieldDescriptorProto.TYPE_UINT64,
    "int32": descriptor_pb2.FieldDescriptorProto.TYPE_INT32,
    "uint32": descriptor_pb2.FieldDescriptorProto.TYPE_UINT32,
    "bool": descriptor_pb2.FieldDescriptorProto.TYPE_BOOL,
    "string": descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
    "bytes": descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
    "sint32": descriptor_pb2.FieldDescriptorProto.TYPE_SINT32,
    "sint64": descriptor_pb2.FieldDescriptorProto.TYPE_SINT64,
}
_LABELS = {
    "optional": descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL,
    "required": descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL,  # see .proto header
    "repeated": descriptor_pb2.FieldDescriptorProto.LABEL_REPEATED,
}
_TOKEN_RE = re.compile(r'"(?:[^"\\]|\\.)*"|[A-Za-z_][A-Za-z0-9_.]*|-?\d+(?:\.\d+)?|[{}=;\[\],]')


class ProtoParseError(ValueError):
    pass


class _Parser:
    def __init__(self, text: str):
        text = re.sub(r"//[^\n]*", "", text)
        self.toks: List[str] = _TOKEN_RE.findall(text)
        self.i = 0
        self.package = ""
        # fully qualified name (without leading dot) -> "message" | "enum"
        self.kinds: Dict[str, str] = {}
        # (field proto, scope list, raw type name) for later resolution
        self.pending: List[Tuple[descriptor_pb2.FieldDescriptorProto, List[str], str]] = []

    def peek(self) -> Optional[str]:
        return self.toks[self.i] if self.i < len(self.toks) else None

    def take(self, expect: Optional[str] = None) -> str:
        tok = self.peek()
        if tok is None:
            raise ProtoParseError("unexpected end of proto text")
        if expect is not None and tok != expect:
            raise ProtoParseError(f"expected {expect!r}, got {tok!r} at token {self.i}")
        self.i += 1
        return tok

    def parse(self) -> descriptor_pb2.FileDescriptorProto:
        fdp = descriptor_pb2.FileDescriptorProto(name="dcos_commons_amd/mesos_v1.proto", syntax="proto2")
        while self.peek() is not None:
            tok = self.take()
            if tok == "syntax":
                self.take("=")
                self.take()
                self.take(";")
            elif tok == "package":
                self.package = self.take()
                fdp.package = self.package
                self.take(";")
            elif tok == "message":
                self._message(fdp.message_type.add(), [])
            elif tok == "enum":
                self._enum(fdp.enum_type.add(), [])
            else:
                raise ProtoParseError(f"unexpected top-level token {tok!r}")
        self._resolve()
        return fdp

    def _fq(self, scope: List[str], name: str) -> str:
        parts = ([self.package] if self.package else []) + scope + [name]
        return ".".join(parts)

    def _message(self, msg: descriptor_pb2.DescriptorProto, scope: List[str]) -> None:
        msg.name = self.take()
        self.kinds[self._fq(scope, msg.name)] = "message"
        inner = scope + [msg.name]
        self.take("{")
        while self.peek() != "}":
            tok = self.take()
            if tok == "message":
                self._message(msg.nested_type.add(), inner)
            elif tok == "enum":
                self._enum(msg.enum_type.add(), inner)
            elif tok in _LABELS:
                self._field(msg.field.add(), inner, tok)
            else:
                raise ProtoParseError(f"unexpected token {tok!r} in message {msg.name}")
        self.take("}")

    def _enum(self, enum: descriptor_pb2.EnumDescriptorProto, scope: List[str]) -> None:
        enum.name = self.take()
        self.kinds[self._fq(scope, enum.name)] = "enum"
        self.take("{")
        while self.peek() != "}":
            name = self.take()
            self.take("=")
            num = int(self.take())
            self.take(";")
            enum.value.add(name=name, number=num)
        self.take("}")

    def _field(self, fld: descriptor_pb2.FieldDescriptorProto, scope: List[str], label: str) -> None:
        fld.label = _LABELS[label]
        type_name = self.take()
        fld.name = self.take()
        self.take("=")
        fld.number = int(self.take())
        if self.peek() == "[":
            self.take("[")
            while True:
                opt = self.take()
                self.take("=")
                val = self.take()
                if opt == "default":
                    fld.default_value = val[1:-1] if val.startswith('"') else val
                if self.peek() == ",":
                    self.take(",")
                    continue
                break
            self.take("]")
        self.take(";")
        fld.json_name = _camel(fld.name)
        if type_name in _SCALAR_TYPES:
            fld.type = _SCALAR_TYPES[type_name]
        else:
            self.pending.append((fld, scope, type_name))

    def _resolve(self) -> None:
        for fld, scope, raw in self.pending:
            found = None
            for depth in range(len(scope), -1, -1):
                cand = self._fq(scope[:depth], raw)
                if cand in self.kinds:
                    found = cand
                    break
            if found is None:
                raise ProtoParseError(f"unresolved type {raw!r} for field {fld.name} in {'.'.join(scope)}")
            fld.type_name = "." + found
            if self.kinds[found] == "message":
                fld.type = descriptor_pb2.FieldDescriptorProto.TYPE_MESSAGE
            else:
                fld.type = descriptor_pb2.FieldDescriptorProto.TYPE_ENUM


def _camel(name: str) -> str:
    parts = name.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


def _build():
    with open(_PROTO_FILE, "r", encoding="utf-8") as f:
        parser = _Parser(f.read())
    fdp = parser.parse()
    pool = descriptor_pool.DescriptorPool()
    file_desc = pool.Add(fdp)
    if file_desc is None:  # older API returns None; look it up
        file_desc = pool.FindFileByName(fdp.name)
    return pool, file_desc


POOL, FILE_DESCRIPTOR = _build()
_exports = {}
for _name, _mdesc in FILE_DESCRIPTOR.message_types_by_name.items():
    _exports[_name] = message_factory.GetMessageClass(_mdesc)
for _name, _edesc in FILE_DESCRIPTOR.enum_types_by_name.items():
    _exports[_name] = enum_type_wrapper.EnumTypeWrapper(_edesc)
    for _v in _edesc.values:
        _exports[_v.name] = _v.number
globals().update(_exports)

# Explicit names for linters / readers.
FrameworkID = _exports["FrameworkID"]
OfferID = _exports["OfferID"]
AgentID = _exports["AgentID"]
TaskID = _exports["TaskID"]
ExecutorID = _exports["ExecutorID"]
FrameworkInfo = _exports["FrameworkInfo"]
MasterInfo = _exports["MasterInfo"]
Value = _exports["Value"]
Attribute = _exports["Attribute"]
Resource = _exports["Resource"]
Offer = _exports["Offer"]
TaskInfo = _exports["TaskInfo"]
TaskGroupInfo = _exports["TaskGroupInfo"]
TaskStatus = _exports["TaskStatus"]
ExecutorInfo = _exports["ExecutorInfo"]
CommandInfo = _exports["CommandInfo"]
Environment = _exports["Environment"]
Labels = _exports["Labels"]
Label = _exports["Label"]
ContainerInfo = _exports["ContainerInfo"]
Volume = _exports["Volume"]
NetworkInfo = _exports["NetworkInfo"]
HealthCheck = _exports["HealthCheck"]
CheckInfo = _exports["CheckInfo"]
CheckStatusInfo = _exports["CheckStatusInfo"]
KillPolicy = _exports["KillPolicy"]
DiscoveryInfo = _exports["DiscoveryInfo"]
Port = _exports["Port"]
Ports = _exports["Ports"]
DomainInfo = _exports["DomainInfo"]
Secret = _exports["Secret"]
Image = _exports["Image"]
LinuxInfo = _exports["LinuxInfo"]
RLimitInfo = _exports["RLimitInfo"]
SeccompInfo = _exports["SeccompInfo"]
Filters = _exports["Filters"]
Credential = _exports["Credential"]
DurationInfo = _exports["DurationInfo"]
ContainerStatus = _exports["ContainerStatus"]
Event = _exports["Event"]
Call = _exports["Call"]
TaskState = _exports["TaskState"]


def task_state_name(state: int) -> str:
    return TaskState.Name(state)


def to_json(msg) -> dict:
    """Mesos v1 JSON mapping (field names as declared, enums as names)."""
    return json_format.MessageToDict(msg, preserving_proto_field_name=True)


def from_json(cls, data):
    return json_format.ParseDict(data, cls(), ignore_unknown_fields=True)


def to_text(msg) -> str:
    return text_format.MessageToString(msg, as_one_line=True)


_V0_NAMES = {"agentId": "slaveId", "agentInfo": "slaveInfo"}


def _rename_v0(node):
    if isinstance(node, dict):
        return {_V0_NAMES.get(k, k): _rename_v0(v) for k, v in node.items()}
    if isinstance(node, list):
        return [_rename_v0(v) for v in node]
    return node


def to_v0_json(msg) -> dict:
    """JSON as the reference's HTTP API renders Mesos protos (Jackson protobuf module over the v0
    ``org.apache.mesos.Protos``): camelCase field names and the v0 ``slave*`` names, e.g.
    ``{"taskId": {...}, "slaveId": {...}}`` (helloworld/tests/test_sanity.py:231)."""
    return _rename_v0(json_format.MessageToDict(msg))

