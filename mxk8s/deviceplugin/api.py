"""Kubelet Device Plugin API v1beta1, built at run time (no protoc).

The schema reproduces ``k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto``
(package ``v1beta1``): the same service/method names and field numbers, so the
wire bytes are what the kubelet sends and expects.  The descriptors are
assembled with ``descriptor_pb2`` into a private pool and the message classes
are generated from it; gRPC handlers/stubs are wired with explicit
(de)serializers.  ``tests/test_deviceplugin.py::test_golden_wire_bytes`` pins the
golden wire bytes.

This replaces the Go device plugin inside the reference's GPU Operator
(/root/reference/README.md:264-272).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool
from google.protobuf import message_factory

API_VERSION = "v1beta1"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
KUBELET_SOCKET_NAME = "kubelet.sock"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"

_F = descriptor_pb2.FieldDescriptorProto
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
_STR, _BOOL, _I32, _I64, _MSG = _F.TYPE_STRING, _F.TYPE_BOOL, _F.TYPE_INT32, _F.TYPE_INT64, _F.TYPE_MESSAGE

# (message name, [(field name, number, label, type, type_name | None, json_name | None)])
_MESSAGES = [
    ("DevicePluginOptions", [("pre_start_required", 1, _OPT, _BOOL, None),
                             ("get_preferred_allocation_available", 2, _OPT, _BOOL, None)]),
    ("RegisterRequest", [("version", 1, _OPT, _STR, None), ("endpoint", 2, _OPT, _STR, None),
                         ("resource_name", 3, _OPT, _STR, None),
                         ("options", 4, _OPT, _MSG, ".v1beta1.DevicePluginOptions")]),
    ("Empty", []),
    ("ListAndWatchResponse", [("devices", 1, _REP, _MSG, ".v1beta1.Device")]),
    ("TopologyInfo", [("nodes", 1, _REP, _MSG, ".v1beta1.NUMANode")]),
    ("NUMANode", [("ID", 1, _OPT, _I64, None)]),
    ("Device", [("ID", 1, _OPT, _STR, None), ("health", 2, _OPT, _STR, None),
                ("topology", 3, _OPT, _MSG, ".v1beta1.TopologyInfo")]),
    ("PreStartContainerRequest", [("devices_ids", 1, _REP, _STR, None)]),
    ("PreStartContainerResponse", []),
    ("PreferredAllocationRequest", [("container_requests", 1, _REP, _MSG,
                                     ".v1beta1.ContainerPreferredAllocationRequest")]),
    ("ContainerPreferredAllocationRequest", [("available_deviceIDs", 1, _REP, _STR, None),
                                             ("must_include_deviceIDs", 2, _REP, _STR, None),
                                             ("allocation_size", 3, _OPT, _I32, None)]),
    ("PreferredAllocationResponse", [("container_responses", 1, _REP, _MSG,
                                      ".v1beta1.ContainerPreferredAllocationResponse")]),
    ("ContainerPreferredAllocationResponse", [("deviceIDs", 1, _REP, _STR, None)]),
    ("AllocateRequest", [("container_requests", 1, _REP, _MSG, ".v1beta1.ContainerAllocateRequest")]),
    ("ContainerAllocateRequest", [("devices_ids", 1, _REP, _STR, None)]),
    ("CDIDevice", [("name", 1, _OPT, _STR, None)]),
    ("AllocateResponse", [("container_responses", 1, _REP, _MSG, ".v1beta1.ContainerAllocateResponse")]),
    ("ContainerAllocateResponse", [
        ("envs", 1, _REP, _MSG, ".v1beta1.ContainerAllocateResponse.EnvsEntry"),
        ("mounts", 2, _REP, _MSG, ".v1beta1.Mount"),
        ("devices", 3, _REP, _MSG, ".v1beta1.DeviceSpec"),
        ("annotations", 4, _REP, _MSG, ".v1beta1.ContainerAllocateResponse.AnnotationsEntry"),
        ("cdi_devices", 5, _REP, _MSG, ".v1beta1.CDIDevice")]),
    ("Mount", [("container_path", 1, _OPT, _STR, None), ("host_path", 2, _OPT, _STR, None),
               ("read_only", 3, _OPT, _BOOL, None)]),
    ("DeviceSpec", [("container_path", 1, _OPT, _STR, None), ("host_path", 2, _OPT, _STR, None),
                    ("permissions", 3, _OPT, _STR, None)]),
]

# map<string,string> fields are nested *Entry messages with map_entry=true
_MAP_ENTRIES = {"ContainerAllocateResponse": ["EnvsEntry", "AnnotationsEntry"]}

# service -> [(method, input, output, server_streaming)]
SERVICES = {
    "Registration": [("Register", "RegisterRequest", "Empty", False)],
    "DevicePlugin": [
        ("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
        ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
        ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse", False),
        ("Allocate", "AllocateRequest", "AllocateResponse", False),
        ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False),
    ],
}


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "mxk8s/deviceplugin/v1beta1/api.proto"
    fd.package = API_VERSION
    fd.syntax = "proto3"
    fd.options.go_package = "v1beta1"
    for name, fields in _MESSAGES:
        m = fd.message_type.add()
        m.name = name
        for fname, num, label, ftype, tname in fields:
            f = m.field.add()
            f.name, f.number, f.label, f.type = fname, num, label, ftype
            if tname:
                f.type_name = tname
        for entry in _MAP_ENTRIES.get(name, []):
            e = m.nested_type.add()
            e.name = entry
            e.options.map_entry = True
            for fname, num in (("key", 1), ("value", 2)):
                f = e.field.add()
                f.name, f.number, f.label, f.type = fname, num, _OPT, _STR
    for sname, methods in SERVICES.items():
        s = fd.service.add()
        s.name = sname
        for mname, inp, out, stream in methods:
            md = s.method.add()
            md.name = mname
            md.input_type = f".{API_VERSION}.{inp}"
            md.output_type = f".{API_VERSION}.{out}"
            md.server_streaming = stream
    return fd


FILE_DESCRIPTOR = _build_file()
_pool = descriptor_pool.DescriptorPool()
_file = _pool.Add(FILE_DESCRIPTOR)


def _cls(name: str):
    return message_factory.GetMessageClass(_pool.FindMessageTypeByName(f"{API_VERSION}.{name}"))


DevicePluginOptions = _cls("DevicePluginOptions")
RegisterRequest = _cls("RegisterRequest")
Empty = _cls("Empty")
ListAndWatchResponse = _cls("ListAndWatchResponse")
TopologyInfo = _cls("TopologyInfo")
NUMANode = _cls("NUMANode")
Device = _cls("Device")
PreStartContainerRequest = _cls("PreStartContainerRequest")
PreStartContainerResponse = _cls("PreStartContainerResponse")
PreferredAllocationRequest = _cls("PreferredAllocationRequest")
ContainerPreferredAllocationRequest = _cls("ContainerPreferredAllocationRequest")
PreferredAllocationResponse = _cls("PreferredAllocationResponse")
ContainerPreferredAllocationResponse = _cls("ContainerPreferredAllocationResponse")
AllocateRequest = _cls("AllocateRequest")
ContainerAllocateRequest = _cls("ContainerAllocateRequest")
CDIDevice = _cls("CDIDevice")
AllocateResponse = _cls("AllocateResponse")
ContainerAllocateResponse = _cls("ContainerAllocateResponse")
Mount = _cls("Mount")
DeviceSpec = _cls("DeviceSpec")

_BY_NAME = {n: _cls(n) for n, _ in _MESSAGES}


def method_path(service: str, method: str) -> str:
    return f"/{API_VERSION}.{service}/{method}"


def generic_handler(service: str, impl) -> "grpc.GenericRpcHandler":  # noqa: F821
    """gRPC handler for ``service`` dispatching to ``impl.<Method>(request, context)``."""
    import grpc
    handlers = {}
    for mname, inp, out, stream in SERVICES[service]:
        fn = getattr(impl, mname)
        req_cls, resp_cls = _BY_NAME[inp], _BY_NAME[out]
        factory = grpc.unary_stream_rpc_method_handler if stream else grpc.unary_unary_rpc_method_handler
        handlers[mname] = factory(fn, request_deserializer=req_cls.FromString,
                                  response_serializer=resp_cls.SerializeToString)
    return grpc.method_handlers_generic_handler(f"{API_VERSION}.{service}", handlers)


class Stub:
    """Client stub for ``service`` over ``channel`` (used by the plugin to call
    Registration, and by the fake kubelet / doctor to call the plugin)."""

    def __init__(self, channel, service: str):
        for mname, inp, out, stream in SERVICES[service]:
            req_cls, resp_cls = _BY_NAME[inp], _BY_NAME[out]
            mk = channel.unary_stream if stream else channel.unary_unary
            setattr(self, mname, mk(method_path(service, mname),
                                    request_serializer=req_cls.SerializeToString,
                                    response_deserializer=resp_cls.FromString))
