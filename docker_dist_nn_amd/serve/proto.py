"""The reference's wire schema, built at runtime (no protoc / grpc_tools in this image).

Equivalent to /root/reference/src/proto/dist_nn.proto:1-15:

    package grpc_dist_nn;
    message Row    { repeated double values = 1; }
    message Matrix { repeated Row rows = 1; }
    service LayerService { rpc Process (Matrix) returns (Matrix); }

The hot path never builds these message objects -- :mod:`.codec` maps wire bytes to/from
numpy in C++ -- but standard message classes are provided for interoperability tests and for
callers that want protobuf objects.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "grpc_dist_nn"
SERVICE = f"{PACKAGE}.LayerService"
METHOD = f"/{SERVICE}/Process"

_pool = descriptor_pool.DescriptorPool()


def _build():
    f = descriptor_pb2.FileDescriptorProto(name="dist_nn.proto", package=PACKAGE,
                                           syntax="proto3")
    F = descriptor_pb2.FieldDescriptorProto
    row = f.message_type.add(name="Row")
    row.field.add(name="values", number=1, type=F.TYPE_DOUBLE, label=F.LABEL_REPEATED)
    mat = f.message_type.add(name="Matrix")
    mat.field.add(name="rows", number=1, type=F.TYPE_MESSAGE, label=F.LABEL_REPEATED,
                  type_name=f".{PACKAGE}.Row")
    svc = f.service.add(name="LayerService")
    svc.method.add(name="Process", input_type=f".{PACKAGE}.Matrix",
                   output_type=f".{PACKAGE}.Matrix")
    _pool.Add(f)
    get = getattr(message_factory, "GetMessageClass", None)
    if get is None:  # older protobuf
        fac = message_factory.MessageFactory(_pool)
        get = lambda d: fac.GetPrototype(d)  # noqa: E731
    return (get(_pool.FindMessageTypeByName(f"{PACKAGE}.Row")),
            get(_pool.FindMessageTypeByName(f"{PACKAGE}.Matrix")))


Row, Matrix = _build()
