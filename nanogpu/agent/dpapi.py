"""Kubelet device-plugin API (k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1) without protoc.

The message descriptors are assembled at import time with descriptor_pb2 (field names,
numbers and types as in upstream `api.proto` [ext]), and the two services are served /
called through grpc generic handlers, so the agent needs only the grpcio and protobuf
runtimes that ship in the image. Wire format is what kubelet speaks:

  service Registration  { Register(RegisterRequest) returns (Empty) }
  service DevicePlugin  { GetDevicePluginOptions(Empty) returns (DevicePluginOptions);
                          ListAndWatch(Empty) returns (stream ListAndWatchResponse);
                          GetPreferredAllocation(PreferredAllocationRequest) returns (PreferredAllocationResponse);
                          Allocate(AllocateRequest) returns (AllocateResponse);
                          PreStartContainer(PreStartContainerRequest) returns (PreStartContainerResponse) }
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

VERSION = "v1beta1"
PACKAGE = "v1beta1"
KUBELET_SOCKET = "/var/lib/kubelet/device-plugins/kubelet.sock"
PLUGIN_DIR = "/var/lib/kubelet/device-plugins"
HEALTHY, UNHEALTHY = "Healthy", "Unhealthy"

_F = descriptor_pb2.FieldDescriptorProto
_T = {"string": _F.TYPE_STRING, "bool": _F.TYPE_BOOL, "int64": _F.TYPE_INT64, "int32": _F.TYPE_INT32}

# name -> [(field, number, type or .Message, repeated)]
_MESSAGES: dict[str, list[tuple[str, int, str, bool]]] = {
    "DevicePluginOptions": [("pre_start_required", 1, "bool", False),
                            ("get_preferred_allocation_available", 2, "bool", False)],
    "RegisterRequest": [("version", 1, "string", False), ("endpoint", 2, "string", False),
                        ("resource_name", 3, "string", False), ("options", 4, ".DevicePluginOptions", False)],
    "Empty": [],
    "ListAndWatchResponse": [("devices", 1, ".Device", True)],
    "TopologyInfo": [("nodes", 1, ".NUMANode", True)],
    "NUMANode": [("ID", 1, "int64", False)],
    "Device": [("ID", 1, "string", False), ("health", 2, "string", False),
               ("topology", 3, ".TopologyInfo", False)],
    "PreStartContainerRequest": [("devices_ids", 1, "string", True)],
    "PreStartContainerResponse": [],
    "PreferredAllocationRequest": [("container_requests", 1, ".ContainerPreferredAllocationRequest", True)],
    "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, "string", True),
                                            ("must_include_deviceIDs", 2, "string", True),
                                            ("allocation_size", 3, "int32", False)],
    "PreferredAllocationResponse": [("container_responses", 1, ".ContainerPreferredAllocationResponse", True)],
    "ContainerPreferredAllocationResponse": [("deviceIDs", 1, "string", True)],
    "AllocateRequest": [("container_requests", 1, ".ContainerAllocateRequest", True)],
    "ContainerAllocateRequest": [("devices_ids", 1, "string", True)],
    "AllocateResponse": [("container_responses", 1, ".ContainerAllocateResponse", True)],
    "ContainerAllocateResponse": [("envs", 1, "map", False), ("mounts", 2, ".Mount", True),
                                  ("devices", 3, ".DeviceSpec", True), ("annotations", 4, "map", False),
                                  ("cdi_devices", 5, ".CDIDevice", True)],
    "Mount": [("container_path", 1, "string", False), ("host_path", 2, "string", False),
              ("read_only", 3, "bool", False)],
    "DeviceSpec": [("container_path", 1, "string", False), ("host_path", 2, "string", False),
                   ("permissions", 3, "string", False)],
    "CDIDevice": [("name", 1, "string", False)],
}

_SERVICES = {
    "Registration": [("Register", "RegisterRequest", "Empty", False)],
    "DevicePlugin": [("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
                     ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
                     ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse", False),
                     ("Allocate", "AllocateRequest", "AllocateResponse", False),
                     ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False)],
}


def _map_entry(msg: descriptor_pb2.DescriptorProto, field: str, package: str = PACKAGE) -> str:
    entry = msg.nested_type.add()
    entry.name = "".join(p.capitalize() for p in field.split("_")) + "Entry"
    entry.options.map_entry = True
    for i, k in enumerate(("key", "value"), 1):
        f = entry.field.add()
        f.name, f.number, f.type, f.label = k, i, _F.TYPE_STRING, _F.LABEL_OPTIONAL
    return f".{package}.{msg.name}.{entry.name}"


def _build(package: str = PACKAGE, file_name: str = "nanogpu/deviceplugin_v1beta1.proto",
           messages: dict | None = None, services: dict | None = None):
    """Message classes of one proto package, assembled from the field tables above."""
    messages = _MESSAGES if messages is None else messages
    services = _SERVICES if services is None else services
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = file_name
    fd.package = package
    fd.syntax = "proto3"
    for name, fields in messages.items():
        m = fd.message_type.add()
        m.name = name
        for fname, num, ftype, rep in fields:
            f = m.field.add()
            f.name, f.number = fname, num
            if ftype == "map":
                f.type, f.label = _F.TYPE_MESSAGE, _F.LABEL_REPEATED
                f.type_name = _map_entry(m, fname, package)
            elif ftype.startswith("."):
                f.type = _F.TYPE_MESSAGE
                f.type_name = f".{package}{ftype}"
                f.label = _F.LABEL_REPEATED if rep else _F.LABEL_OPTIONAL
            else:
                f.type = _T[ftype]
                f.label = _F.LABEL_REPEATED if rep else _F.LABEL_OPTIONAL
    for sname, methods in services.items():
        s = fd.service.add()
        s.name = sname
        for mname, req, resp, stream in methods:
            md = s.method.add()
            md.name, md.input_type, md.output_type = mname, f".{package}.{req}", f".{package}.{resp}"
            md.server_streaming = stream
    pool = descriptor_pool.DescriptorPool()
    fdesc = pool.Add(fd)
    fdesc = pool.FindFileByName(fd.name)
    return {name: message_factory.GetMessageClass(fdesc.message_types_by_name[name]) for name in messages}


M = _build()
globals().update(M)  # DevicePluginOptions, RegisterRequest, Empty, Device, AllocateRequest, ...


def method_path(service: str, method: str) -> str:
    return f"/{PACKAGE}.{service}/{method}"


def generic_handler(service: str, impl, package: str = PACKAGE, services: dict | None = None,
                    messages: dict | None = None) -> "object":
    """grpc generic handler for `service` dispatching to `impl.<Method>(request, context)`."""
    import grpc

    services = _SERVICES if services is None else services
    messages = M if messages is None else messages
    handlers = {}
    for mname, req, resp, stream in services[service]:
        fn = getattr(impl, mname)
        de, se = messages[req].FromString, messages[resp].SerializeToString
        if stream:
            handlers[mname] = grpc.unary_stream_rpc_method_handler(fn, request_deserializer=de, response_serializer=se)
        else:
            handlers[mname] = grpc.unary_unary_rpc_method_handler(fn, request_deserializer=de, response_serializer=se)
    return grpc.method_handlers_generic_handler(f"{package}.{service}", handlers)


class Stub:
    """Client for either service over a grpc channel (tests' fake kubelet uses it too)."""

    def __init__(self, channel, service: str, package: str = PACKAGE, services: dict | None = None,
                 messages: dict | None = None):
        services = _SERVICES if services is None else services
        messages = M if messages is None else messages
        for mname, req, resp, stream in services[service]:
            path = f"/{package}.{service}/{mname}"
            ser, de = messages[req].SerializeToString, messages[resp].FromString
            if stream:
                call = channel.unary_stream(path, request_serializer=ser, response_deserializer=de)
            else:
                call = channel.unary_unary(path, request_serializer=ser, response_deserializer=de)
            setattr(self, mname, call)
