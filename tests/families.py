"""Input families the BASELINE configs never produce, for parity tests on every engine.

Each builder returns a workload.Workload (nodes, pending pods, services, config,
existing pods with their Status.Host) that the reference's semantics define
completely; tests run it through ref_model, the C restatement and the HIP
library and compare every decision.

  multi_service   pods matching 2-3 overlapping services, one of them with an empty
                  selector (matches every pod of its namespace: SelectorFromSet(nil/{})
                  is Everything, pkg/labels/labels.go:60-61, cache/listers.go:109-129);
                  a commit of a pod in service A moves service B's maxCount
  namespaces      two namespaces with identical labels and services: counts and peers
                  stay per namespace (spreading.go:61-70, predicates.go:284-290)
  negative        negative weights on every priority kind (Policy weights are not
                  validated, plugins.go:159,169): the batch takes the exact path
  big_weights     weights just under the window path's int32 score bound
  huge_weights    Go int weights around 2^40 and 2^62 (combined scores wrap like
                  Go's int64, generic_scheduler.go:145-159): the exact kernels
                  with int64 scores
  many_anti       six ServiceAntiAffinity priorities (two per label: the reference
                  registers any number, plugins.go:145-183): the exact kernels
  existing_hosts  pre-existing pods with Status.Host == "" and on hosts outside the
                  node list (MapPodsToMachines keys on Status.Host, predicates.go:354-375)
  invalid_selectors  ServiceAffinity over two predicates with invalid nodeSelector
                  values and invalid node label values (SelectorFromSet's trap)
  past_caps       a Policy past round 3's caps: six ServiceAffinity labels in ten
                  predicates (label groups) and twenty ServiceAntiAffinity priorities
                  (the reference registers any number of each, plugins.go:81-117,
                  145-183): the exact kernels
"""
from __future__ import annotations

from kubernetes_amd import factory, workload
from kubernetes_amd.api import ObjectMeta, PodStatus, Quantity, Service, ServiceSpec

FAMILIES = ("multi_service", "namespaces", "negative", "big_weights", "huge_weights", "many_anti", "existing_hosts",
            "invalid_selectors", "past_caps")

# the window path keeps 10 * sum|w| + |w_equal| below 2^30 (KSG_SCORE_BOUND, ksg_internal.h)
BIG_W = (1 << 30) // 10 // 4 - 1


def _policy(preds, prios, tag):
    pol = {"predicates": [p if isinstance(p, dict) else {"name": p} for p in preds],
           "priorities": [dict(p, name=f"{tag}-{p['name']}") if "argument" in p else p for p in prios]}
    return factory.create_from_config(pol)


_DEFAULT_PREDS = ("PodFitsPorts", "PodFitsResources", "NoDiskConflict", "MatchNodeSelector", "HostName")


def _tighten(nodes, rng):
    for n in nodes:
        n.spec.capacity["cpu"] = Quantity.from_milli(1500 + 500 * rng.below(4))


def build(family: str, nn: int, npods: int, seed: int = 7) -> workload.Workload:
    rng = workload._SM(seed * 7919 + len(family))
    nodes = workload.make_nodes(nn, rng)
    existing = []
    if family == "multi_service":
        pods = workload.make_pods(npods + npods // 4, rng, n_apps=6)
        for i, p in enumerate(pods):
            p.metadata.labels["tier"] = f"t{i % 3}"
        services = workload.make_services(6)
        services.insert(2, Service(metadata=ObjectMeta(name="svc-tier0", namespace="default"),
                                   spec=ServiceSpec(selector={"tier": "t0"})))
        services.insert(4, Service(metadata=ObjectMeta(name="svc-all", namespace="default"),
                                   spec=ServiceSpec(selector={})))
        services.append(Service(metadata=ObjectMeta(name="svc-a1-t1", namespace="default"),
                                spec=ServiceSpec(selector={"app": "a1", "tier": "t1"})))
        existing, pods = pods[:npods // 4], pods[npods // 4:]
        names = [n.metadata.name for n in nodes]
        for i, p in enumerate(existing):
            p.status = PodStatus(host=names[(i * 13) % len(names)])
        cfg = _policy(_DEFAULT_PREDS + ({"name": "RegionAff", "argument": {"serviceAffinity": {"labels": ["region"]}}},),
                      [{"name": "LeastRequestedPriority", "weight": 1}, {"name": "ServiceSpreadingPriority", "weight": 2},
                       {"name": "ZoneSpread", "weight": 1, "argument": {"serviceAntiAffinity": {"label": "zone"}}}],
                      "ms")
    elif family == "namespaces":
        pods = workload.make_pods(npods, rng, n_apps=5)
        for i, p in enumerate(pods):
            p.metadata.namespace = "default" if i % 2 else "other"
        services = workload.make_services(5)
        for s in workload.make_services(5):
            s.metadata.namespace = "other"
            services.append(s)
        cfg = _policy(_DEFAULT_PREDS + ({"name": "RegionAff", "argument": {"serviceAffinity": {"labels": ["region"]}}},),
                      [{"name": "LeastRequestedPriority", "weight": 1}, {"name": "ServiceSpreadingPriority", "weight": 1}],
                      "ns")
    elif family == "negative":
        pods = workload.make_pods(npods, rng, n_apps=8)
        services = workload.make_services(8)
        _tighten(nodes, rng)
        cfg = _policy(_DEFAULT_PREDS,
                      [{"name": "LeastRequestedPriority", "weight": 1}, {"name": "ServiceSpreadingPriority", "weight": 1},
                       {"name": "EqualPriority", "weight": 1},
                       {"name": "NegZone", "weight": -2, "argument": {"serviceAntiAffinity": {"label": "zone"}}},
                       {"name": "NegRack", "weight": -3,
                        "argument": {"labelPreference": {"label": "rack", "presence": True}}}],
                      "neg")
        # builtin names keep their registered weight (plugins.go:173-176): negate them
        # through a custom provider-free config instead
        cfg.priorities = [factory.PriorityDesc(p.kind, -abs(p.weight) if p.kind in (
            "LeastRequestedPriority", "ServiceSpreadingPriority", "EqualPriority") else p.weight, p.label, p.presence)
            for p in cfg.priorities]
    elif family == "big_weights":
        pods = workload.make_pods(npods, rng, n_apps=8)
        services = workload.make_services(8)
        cfg = _policy(_DEFAULT_PREDS,
                      [{"name": "LeastRequestedPriority", "weight": 1}, {"name": "ServiceSpreadingPriority", "weight": 1},
                       {"name": "BigRack", "weight": BIG_W,
                        "argument": {"labelPreference": {"label": "rack", "presence": True}}}],
                      "big")
        cfg.priorities = [factory.PriorityDesc(p.kind, BIG_W if p.kind in (
            "LeastRequestedPriority", "ServiceSpreadingPriority") else p.weight, p.label, p.presence)
            for p in cfg.priorities]
    elif family == "huge_weights":
        pods = workload.make_pods(npods, rng, n_apps=8)
        services = workload.make_services(8)
        _tighten(nodes, rng)
        cfg = _policy(_DEFAULT_PREDS,
                      [{"name": "LeastRequestedPriority", "weight": 1}, {"name": "ServiceSpreadingPriority", "weight": 1},
                       {"name": "HugeRack", "weight": (1 << 62) + 12345,  # 10 * w wraps past 2^63
                        "argument": {"labelPreference": {"label": "rack", "presence": True}}},
                       {"name": "HugeZone", "weight": -(3 << 40),
                        "argument": {"serviceAntiAffinity": {"label": "zone"}}}],
                      "huge")
        cfg.priorities = [factory.PriorityDesc(p.kind, (3 << 40) + 7 if p.kind == "LeastRequestedPriority" else
                                               (5 << 39) if p.kind == "ServiceSpreadingPriority" else p.weight,
                                               p.label, p.presence)
                          for p in cfg.priorities]
    elif family == "many_anti":
        pods = workload.make_pods(npods, rng, n_apps=6)
        services = workload.make_services(6)
        anti = [{"name": f"Anti{i}-{lab}", "weight": w, "argument": {"serviceAntiAffinity": {"label": lab}}}
                for i, (lab, w) in enumerate((("zone", 1), ("rack", 2), ("region", 1), ("zone", 3), ("rack", 1),
                                              ("region", 2)))]
        cfg = _policy(_DEFAULT_PREDS, [{"name": "LeastRequestedPriority", "weight": 1},
                                       {"name": "ServiceSpreadingPriority", "weight": 1}] + anti, "ma")
    elif family == "four_anti":
        # four ServiceAntiAffinity priorities over 50 label domains (8 + 2 + 32 + 8): within
        # the grid drop-in server's 64, with priorities past its register-held two
        pods = workload.make_pods(npods, rng, n_apps=6)
        services = workload.make_services(6)
        anti = [{"name": f"Anti{i}-{lab}", "weight": w, "argument": {"serviceAntiAffinity": {"label": lab}}}
                for i, (lab, w) in enumerate((("zone", 1), ("region", 2), ("rack", 1), ("zone", 3)))]
        cfg = _policy(_DEFAULT_PREDS, [{"name": "LeastRequestedPriority", "weight": 1},
                                       {"name": "ServiceSpreadingPriority", "weight": 1}] + anti, "fa")
    elif family == "existing_hosts":
        pods = workload.make_pods(npods + npods // 3, rng, n_apps=4)
        services = workload.make_services(4)
        existing, pods = pods[:npods // 3], pods[npods // 3:]
        names = [n.metadata.name for n in nodes]
        for i, p in enumerate(existing):
            host = "" if i % 4 == 0 else ("gone-node-%d" % (i % 3) if i % 4 == 1 else names[(i * 7) % len(names)])
            p.status = PodStatus(host=host)
        cfg = _policy(_DEFAULT_PREDS, [{"name": "LeastRequestedPriority", "weight": 1},
                                       {"name": "ServiceSpreadingPriority", "weight": 1}], "ex")
    elif family == "invalid_selectors":
        pods = workload.make_pods(npods, rng, n_apps=6, sel_frac=0.0)
        services = workload.make_services(6)
        for i, n in enumerate(nodes):
            if i % 9 == 0:
                n.metadata.labels["region"] = "bad value!"
            if i % 13 == 0:
                n.metadata.labels["rack"] = "-bad-"
        for i, p in enumerate(pods):
            k = rng.below(8)
            if k == 0:
                p.spec.node_selector = {"region": "bad value!"}
            elif k == 1:
                p.spec.node_selector = {"rack": "-bad-", "zone": f"z{rng.below(8)}"}
            elif k == 2:
                p.spec.node_selector = {"region": f"r{rng.below(2)}"}
        cfg = _policy(_DEFAULT_PREDS + ({"name": "RegionAff", "argument": {"serviceAffinity": {"labels": ["region"]}}},
                                        {"name": "RackZoneAff",
                                         "argument": {"serviceAffinity": {"labels": ["rack", "zone"]}}}),
                      [{"name": "LeastRequestedPriority", "weight": 1}, {"name": "ServiceSpreadingPriority", "weight": 1}],
                      "inv")
    elif family == "past_caps":
        # labels derived from the zone (region, pool, tier pin it together), two
        # single-valued ones and one on half the nodes (a peer node without the label
        # constrains nothing for it, predicates.go:293-300)
        for i, n in enumerate(nodes):
            z = int(n.metadata.labels["zone"][1:])
            n.metadata.labels.update({"pool": f"p{z % 2}", "tier": f"t{(z // 2) % 2}", "hw": "h0", "os": "linux"})
            if i % 2:
                n.metadata.labels["fabric"] = "f0"
        pods = workload.make_pods(npods, rng, n_apps=6)
        for i, p in enumerate(pods):
            if i % 11 == 0:
                p.spec.node_selector = dict(p.spec.node_selector or {}, pool=f"p{i % 2}")
        services = workload.make_services(6)
        groups = (["region"], ["pool"], ["tier"], ["hw"], ["os"], ["fabric"], ["region", "pool"], ["tier", "hw"],
                  ["os", "fabric"], ["region", "tier", "fabric"])
        aff = tuple({"name": f"Aff{g}", "argument": {"serviceAffinity": {"labels": labels}}}
                    for g, labels in enumerate(groups))
        anti = [{"name": f"Anti{i}", "weight": 1 + i % 3,
                 "argument": {"serviceAntiAffinity": {"label": ("zone", "rack", "region", "pool")[i % 4]}}}
                for i in range(20)]
        cfg = _policy(_DEFAULT_PREDS + aff, [{"name": "LeastRequestedPriority", "weight": 1},
                                             {"name": "ServiceSpreadingPriority", "weight": 1}] + anti, "pc")
    else:
        raise ValueError(family)
    cfg.max_conflict_keys = 4096
    return workload.Workload(family, nodes, pods, services, cfg, existing)


class FamilyCase:
    """A family workload through the product ingest (the shape of tests.helpers.Case)."""

    def __init__(self, family: str, nn: int, npods: int, seed: int = 7):
        from kubernetes_amd import ingest

        self.w = build(family, nn, npods, seed)
        self.it = ingest.Interner()
        for k in self.w.config.label_keys():
            self.it.key_id(k)
        self.view = ingest.ClusterView(self.w.nodes, self.w.services, self.it)
        self.aff = self.w.config.affinity_labels()
        self.existing = ingest.ingest_pods(self.view, self.w.existing, uids=list(range(1, len(self.w.existing) + 1)),
                                           aff_labels=self.aff)
        self.batch = ingest.ingest_pods(self.view, self.w.pods,
                                        uids=list(range(10 ** 6, 10 ** 6 + len(self.w.pods))), aff_labels=self.aff)
        self.cfg = self.w.config.compile(self.it.key_id)

    def load(self, engine):
        """set_cluster + the existing pods on their Status.Host (lister order)."""
        engine.set_cluster(self.view.arrays)
        for i, p in enumerate(self.w.existing):
            engine.add_pod(self.view.host_id(p.status.host), self.existing, i)
        return engine
