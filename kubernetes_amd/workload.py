"""Synthetic scheduler_perf-style workloads (the reference ships none).

Seeded with splitmix64 (workload seed 42; tie-break stream seed 1234, one Int63
draw per successful schedule). Shapes follow SURVEY.md 8(d):
  nodes   `node-%06d`; cpu in {4000,8000,16000,32000} milli; memory in
          {8,16,32,64} Gi; labels zone=z{0..7}, region=r{zone//4},
          rack=z{zone}-r{0..3} (+ `dense_labels` extra keys k{j}=v{0..7})
  pods    cpu 100..1000 m step 100; memory {128,...,2048} Mi; 10% one hostPort
          from a pool of 16; 5% one GCE PD from a pool of 2000; 20% a nodeSelector
          zone=z{0..7}; label app=a{0..n_apps-1}; namespace `default`
  services one per app label, selector app=a{i}, namespace `default`
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

from . import factory
from .api import (Container, ContainerPort, GCEPersistentDiskVolumeSource, Node, NodeSpec, ObjectMeta, Pod,
                  PodSpec, ResourceList, ResourceRequirements, Service, ServiceSpec, Volume)
from .resource import Quantity

WORKLOAD_SEED = 42
TIEBREAK_SEED = 1234
GI = 1 << 30
MI = 1 << 20


class _SM:
    MASK = (1 << 64) - 1

    def __init__(self, seed):
        self.s = seed & self.MASK

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & self.MASK
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & self.MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & self.MASK
        return z ^ (z >> 31)

    def below(self, n):
        return self.next() % n


@dataclass
class Workload:
    name: str
    nodes: List[Node]
    pods: List[Pod]
    services: List[Service]
    config: factory.SchedulerConfig
    existing: List[Pod]


def make_nodes(n: int, rng: _SM, dense_labels: int = 0) -> List[Node]:
    cpus = (4000, 8000, 16000, 32000)
    mems = (8 * GI, 16 * GI, 32 * GI, 64 * GI)
    out = []
    for i in range(n):
        zone = rng.below(8)
        labels = {"zone": f"z{zone}", "region": f"r{zone // 4}", "rack": f"z{zone}-r{rng.below(4)}"}
        for j in range(dense_labels):
            labels[f"k{j}"] = f"v{rng.below(8)}"
        out.append(Node(
            metadata=ObjectMeta(name=f"node-{i:06d}", labels=labels),
            spec=NodeSpec(capacity=ResourceList(cpu=Quantity.from_milli(cpus[rng.below(4)]),
                                                memory=Quantity.from_int(mems[rng.below(4)]))),
        ))
    return out


def make_pods(n: int, rng: _SM, n_apps: int = 100, port_frac=0.10, pd_frac=0.05, sel_frac=0.20,
              dense_sel: int = 0, prefix: str = "pod") -> List[Pod]:
    mems = (128, 256, 512, 1024, 2048)
    out = []
    for i in range(n):
        cpu = 100 * (1 + rng.below(10))
        mem = mems[rng.below(5)] * MI
        ports = []
        if rng.below(1000) < int(port_frac * 1000):
            ports = [ContainerPort(container_port=80, host_port=8000 + rng.below(16))]
        vols = []
        if rng.below(1000) < int(pd_frac * 1000):
            vols = [Volume(name="data", gce_persistent_disk=GCEPersistentDiskVolumeSource(pd_name=f"pd-{rng.below(2000)}"))]
        sel = None
        if rng.below(1000) < int(sel_frac * 1000):
            sel = {"zone": f"z{rng.below(8)}"}
            if dense_sel:
                sel[f"k{rng.below(dense_sel)}"] = f"v{rng.below(8)}"
        app = rng.below(n_apps)
        out.append(Pod(
            metadata=ObjectMeta(name=f"{prefix}-{i:07d}", namespace="default", labels={"app": f"a{app}"}),
            spec=PodSpec(
                containers=[Container(name="c", ports=ports, resources=ResourceRequirements(
                    ResourceList(cpu=Quantity.from_milli(cpu), memory=Quantity.from_int(mem))))],
                volumes=vols,
                node_selector=sel,
            ),
        ))
    return out


def make_services(n_apps: int = 100) -> List[Service]:
    return [Service(metadata=ObjectMeta(name=f"svc-a{i}", namespace="default"),
                    spec=ServiceSpec(selector={"app": f"a{i}"})) for i in range(n_apps)]


def config1() -> factory.SchedulerConfig:
    """SchedulingBasic analogue: PodFitsResources + LeastRequestedPriority (BASELINE config 1)."""
    return factory.create_from_keys(["PodFitsResources"], ["LeastRequestedPriority"])


def config_default() -> factory.SchedulerConfig:
    return factory.create_from_provider(factory.DefaultProvider)


def config4() -> factory.SchedulerConfig:
    """Policy: defaults + ServiceAffinity{region}; ServiceAntiAffinity{zone} + LR + spreading."""
    policy = {
        "predicates": [{"name": n} for n in
                       ("PodFitsPorts", "PodFitsResources", "NoDiskConflict", "MatchNodeSelector", "HostName")]
        + [{"name": "RegionAffinity", "argument": {"serviceAffinity": {"labels": ["region"]}}}],
        "priorities": [{"name": "LeastRequestedPriority", "weight": 1},
                       {"name": "ServiceSpreadingPriority", "weight": 1},
                       {"name": "ZoneSpread", "weight": 1, "argument": {"serviceAntiAffinity": {"label": "zone"}}}],
    }
    return factory.create_from_config(policy)


def build(name: str, n_nodes: Optional[int] = None, n_pods: Optional[int] = None, seed: int = WORKLOAD_SEED) -> Workload:
    """BASELINE.json configs: 'config1'..'config5' (sizes overridable)."""
    rng = _SM(seed)
    if name == "config1":
        nn, npods, cfg, dense = 500, 1000, config1(), 0
    elif name == "config2":
        nn, npods, cfg, dense = 5000, 10000, config_default(), 0
    elif name == "config3":
        nn, npods, cfg, dense = 15000, 50000, config_default(), 0
    elif name == "config4":
        nn, npods, cfg, dense = 5000, 10000, config4(), 0
    elif name == "config5":
        nn, npods, cfg, dense = 100000, 100000, config_default(), 32
    else:
        raise ValueError(name)
    nn = nn if n_nodes is None else n_nodes
    npods = npods if n_pods is None else n_pods
    nodes = make_nodes(nn, rng, dense_labels=dense)
    pods = make_pods(npods, rng, dense_sel=dense)
    if name == "config1":  # resources only: no ports / PDs / selectors matter, keep them off
        pods = [Pod(metadata=p.metadata, spec=PodSpec(containers=[Container(name="c", resources=p.spec.containers[0].resources)]))
                for p in pods]
    cfg.max_conflict_keys = 4096
    return Workload(name, nodes, pods, make_services(), cfg, [])


def extension_data(n_nodes: int, n_pods: int, seed: int = 11, taints: bool = True, gpus: bool = True,
                   w_taint: int = 1, w_bal: int = 1):
    """Seeded taints / tolerations / extended resources for a workload of n_nodes x
    n_pods (the extensions beyond this reference vintage, kubernetes_amd/extensions.py;
    parity unpinned): per node 0-3 taints from a pool of six (NoSchedule, NoExecute,
    PreferNoSchedule), 0/0/4/8 GPUs and 0-2 FPGAs; per pod 0-2 tolerations (10%),
    0-2 GPUs and an FPGA for one pod in ten.
    -> (ExtConfig, node_taints, node_scalar, pod_tolerations, pod_scalar)."""
    from .extensions import NO_EXECUTE, NO_SCHEDULE, PREFER_NO_SCHEDULE, ExtConfig, Taint, Toleration

    rng = _SM(seed)
    gpu, fpga = "nvidia.com/gpu", "example.com/fpga"
    cfg = ExtConfig(taints=taints, scalar_resources=(gpu, fpga) if gpus else (), w_taint_toleration=w_taint,
                    w_balanced=w_bal)
    pool = [Taint("dedicated", "db", NO_SCHEDULE), Taint("dedicated", "ml", NO_SCHEDULE),
            Taint("maint", "", NO_EXECUTE), Taint("spot", "true", PREFER_NO_SCHEDULE),
            Taint("slow-disk", "", PREFER_NO_SCHEDULE), Taint("zone-drain", "z1", PREFER_NO_SCHEDULE)]
    node_taints = []
    for _ in range(n_nodes):
        k = rng.below(4)
        node_taints.append(sorted({pool[rng.below(len(pool))] for _ in range(k)}, key=pool.index))
    node_scalar = {gpu: [[0, 0, 4, 8][rng.below(4)] for _ in range(n_nodes)],
                   fpga: [rng.below(3) for _ in range(n_nodes)]}
    tol_pool = [Toleration("dedicated", "Equal", "db", NO_SCHEDULE), Toleration("dedicated", "Exists"),
                Toleration("maint", "Exists", "", NO_EXECUTE), Toleration("spot", "Equal", "true"),
                Toleration("", "Exists"), Toleration("slow-disk", "Exists", "", PREFER_NO_SCHEDULE),
                Toleration("zone-drain", "Equal", "z2")]
    tols, scal = [], []
    for _ in range(n_pods):
        k = rng.below(3) if rng.below(10) else 0
        tols.append([tol_pool[rng.below(len(tol_pool) - 1) if rng.below(20) else len(tol_pool) - 2]
                     for _ in range(k)])
        scal.append({gpu: [0, 0, 0, 1, 2][rng.below(5)], fpga: 1 if rng.below(10) == 0 else 0})
    return cfg, node_taints, node_scalar if gpus else None, tols, scal
