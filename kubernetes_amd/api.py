"""The subset of pkg/api types the Filter/Score pass reads.

Mirrors (field names in Go / here):
  api.Pod{ObjectMeta{Name,Namespace,Labels}, Spec{Containers,Volumes,
          NodeSelector,Host}, Status{Host}}          pkg/api/types.go (PodSpec ~:700, PodStatus)
  api.Container{Ports[].HostPort, Resources.Limits}  pkg/api/types.go:492-495
  api.Volume{GCEPersistentDisk{PDName}}              pkg/api/types.go:351-365
  api.Node{ObjectMeta{Name,Labels}, Spec.Capacity}   pkg/api/types.go (NodeSpec)
  api.Service{ObjectMeta{Name,Namespace}, Spec.Selector}
Resource quantities are kubernetes_amd.resource.Quantity (or strings / ints
parsed with ParseQuantity). Everything else in pkg/api is out of scope.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

from .resource import Quantity, parse_quantity

NamespaceDefault = "default"


def _q(v) -> Quantity:
    if isinstance(v, Quantity):
        return v
    if isinstance(v, int):
        return Quantity.from_int(v)
    return parse_quantity(str(v))


class ResourceList(dict):
    """map[ResourceName]Quantity with Cpu()/Memory() (resource_helpers.go:29-42)."""

    def __init__(self, *a, **kw):
        super().__init__()
        for k, v in dict(*a, **kw).items():
            self[k] = _q(v)

    def cpu(self) -> Quantity:
        q = self.get("cpu")
        return q if q is not None else Quantity.zero()

    def memory(self) -> Quantity:
        q = self.get("memory")
        return q if q is not None else Quantity.zero()


@dataclass
class ObjectMeta:
    name: str = ""
    namespace: str = ""
    labels: Optional[Dict[str, str]] = None
    creation_timestamp: float = 0.0  # seconds; the kubelet's admission order (kubelet.go:1692-1694)


@dataclass
class ContainerPort:
    container_port: int = 0
    host_port: int = 0
    protocol: str = "TCP"
    host_ip: str = ""


@dataclass
class ResourceRequirements:
    limits: ResourceList = field(default_factory=ResourceList)


@dataclass
class Container:
    name: str = ""
    ports: List[ContainerPort] = field(default_factory=list)
    resources: ResourceRequirements = field(default_factory=ResourceRequirements)


@dataclass
class GCEPersistentDiskVolumeSource:
    pd_name: str = ""
    read_only: bool = False


@dataclass
class Volume:
    name: str = ""
    gce_persistent_disk: Optional[GCEPersistentDiskVolumeSource] = None


@dataclass
class PodSpec:
    containers: List[Container] = field(default_factory=list)
    volumes: List[Volume] = field(default_factory=list)
    node_selector: Optional[Dict[str, str]] = None
    host: str = ""


@dataclass
class PodStatus:
    host: str = ""


@dataclass
class Pod:
    metadata: ObjectMeta = field(default_factory=ObjectMeta)
    spec: PodSpec = field(default_factory=PodSpec)
    status: PodStatus = field(default_factory=PodStatus)

    @property
    def name(self):
        return self.metadata.name

    @property
    def namespace(self):
        return self.metadata.namespace

    @property
    def labels(self):
        return self.metadata.labels

    def key(self) -> str:
        """cache.MetaNamespaceKeyFunc: namespace/name."""
        return f"{self.metadata.namespace}/{self.metadata.name}"


@dataclass
class NodeSpec:
    capacity: ResourceList = field(default_factory=ResourceList)


@dataclass
class Node:
    metadata: ObjectMeta = field(default_factory=ObjectMeta)
    spec: NodeSpec = field(default_factory=NodeSpec)

    @property
    def name(self):
        return self.metadata.name

    @property
    def labels(self):
        return self.metadata.labels


@dataclass
class ServiceSpec:
    selector: Optional[Dict[str, str]] = None


@dataclass
class Service:
    metadata: ObjectMeta = field(default_factory=ObjectMeta)
    spec: ServiceSpec = field(default_factory=ServiceSpec)

    @property
    def name(self):
        return self.metadata.name

    @property
    def namespace(self):
        return self.metadata.namespace


# ---- constructors used by tests and the workload generator -----------------

def make_node(name: str, milli_cpu: int = 0, memory: int = 0, labels: Optional[Dict[str, str]] = None) -> Node:
    """makeMinion (priorities_test.go:28-38): NewMilliQuantity cpu + NewQuantity memory."""
    return Node(
        metadata=ObjectMeta(name=name, labels=labels),
        spec=NodeSpec(capacity=ResourceList(cpu=Quantity.from_milli(milli_cpu), memory=Quantity.from_int(memory))),
    )


def resource_container(milli_cpu: Optional[int] = None, memory: Optional[int] = None, host_ports=()) -> Container:
    lim = ResourceList()
    if milli_cpu is not None:
        lim["cpu"] = Quantity.from_milli(milli_cpu)
    if memory is not None:
        lim["memory"] = Quantity.from_int(memory)
    return Container(ports=[ContainerPort(host_port=p) for p in host_ports], resources=ResourceRequirements(lim))
