"""Kubelet PodResources API v1 (``List`` only), built at run time (no protoc).

Reproduces ``k8s.io/kubelet/pkg/apis/podresources/v1/api.proto`` field
numbers so the exporter can attribute each GPU to the pod/container it was
allocated to (dcgm-exporter does the same for ``nvidia.com/gpu`` [ext]).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto
OPT, REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
STR, I64, MSG = _F.TYPE_STRING, _F.TYPE_INT64, _F.TYPE_MESSAGE

_MESSAGES = [
    ("ListPodResourcesRequest", []),
    ("ListPodResourcesResponse", [("pod_resources", 1, REP, MSG, ".v1.PodResources")]),
    ("PodResources", [("name", 1, OPT, STR, None), ("namespace", 2, OPT, STR, None),
                      ("containers", 3, REP, MSG, ".v1.ContainerResources")]),
    ("ContainerResources", [("name", 1, OPT, STR, None),
                            ("devices", 2, REP, MSG, ".v1.ContainerDevices"),
                            ("cpu_ids", 3, REP, I64, None)]),
    ("ContainerDevices", [("resource_name", 1, OPT, STR, None),
                          ("device_ids", 2, REP, STR, None),
                          ("topology", 3, OPT, MSG, ".v1.TopologyInfo")]),
    ("TopologyInfo", [("nodes", 1, REP, MSG, ".v1.NUMANode")]),
    ("NUMANode", [("ID", 1, OPT, I64, None)]),
]


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="mxk8s/podresources/v1/api.proto", package="v1",
                                            syntax="proto3")
    for name, fields in _MESSAGES:
        m = fd.message_type.add(name=name)
        for fname, num, label, ftype, tname in fields:
            f = m.field.add(name=fname, number=num, label=label, type=ftype)
            if tname:
                f.type_name = tname
    s = fd.service.add(name="PodResourcesLister")
    s.method.add(name="List", input_type=".v1.ListPodResourcesRequest",
                 output_type=".v1.ListPodResourcesResponse")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return {n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"v1.{n}"))
            for n, _ in _MESSAGES}


_C = _build()
ListPodResourcesRequest = _C["ListPodResourcesRequest"]
ListPodResourcesResponse = _C["ListPodResourcesResponse"]
LIST_METHOD = "/v1.PodResourcesLister/List"


def physical_id(device_id: str) -> str:
    """Device-plugin ID -> physical GPU index: time-sliced replicas are
    advertised as ``<i>::<r>`` (mxk8s.deviceplugin.plugin.DeviceState)."""
    return device_id.partition("::")[0]


def gpu_owners(socket_path: str, resource: str = "amd.com/gpu", timeout: float = 2.0) -> dict:
    """physical GPU index -> [(namespace, pod, container), ...] from the kubelet
    socket.  Counts both ``resource`` and its time-sliced ``<resource>.shared``
    rename, maps ``<i>::<r>`` replica IDs to GPU ``i`` and keeps every owner
    of a shared GPU (in first-seen order, no duplicates)."""
    import grpc
    names = {resource, resource + ".shared"}
    out: dict = {}
    with grpc.insecure_channel("unix:" + socket_path) as ch:
        call = ch.unary_unary(LIST_METHOD, request_serializer=ListPodResourcesRequest.SerializeToString,
                              response_deserializer=ListPodResourcesResponse.FromString)
        resp = call(ListPodResourcesRequest(), timeout=timeout)
    for pr in resp.pod_resources:
        for c in pr.containers:
            for d in c.devices:
                if d.resource_name not in names:
                    continue
                for i in d.device_ids:
                    owner = (pr.namespace, pr.name, c.name)
                    lst = out.setdefault(physical_id(i), [])
                    if owner not in lst:
                        lst.append(owner)
    return out


def serve_fake(socket_path: str, response):
    """Test helper: a fake kubelet PodResources server returning ``response``."""
    import concurrent.futures

    import grpc
    handler = grpc.method_handlers_generic_handler("v1.PodResourcesLister", {
        "List": grpc.unary_unary_rpc_method_handler(
            lambda req, ctx: response, request_deserializer=ListPodResourcesRequest.FromString,
            response_serializer=ListPodResourcesResponse.SerializeToString)})
    srv = grpc.server(concurrent.futures.ThreadPoolExecutor(max_workers=2))
    srv.add_generic_rpc_handlers((handler,))
    srv.add_insecure_port("unix:" + socket_path)
    srv.start()
    return srv
