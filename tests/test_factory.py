"""Registry / provider / Policy compilation (plugin/pkg/scheduler/factory, algorithmprovider),
checked against the reference's factory tests and its traps; evaluated through the C oracle."""
import pytest

from kubernetes_amd import abi, factory
from kubernetes_amd.api import Node, ObjectMeta, Pod, make_node
from oracle.pyoracle import OracleScheduler
from tests.golden_util import run_engine


def test_algorithm_name_validation():
    """TestAlgorithmNameValidation (factory/plugins_test.go:21-42)."""
    for n in ("1SomeAlgo1rithm", "someAlgor-ithm1"):
        factory._validate_name(n)
    for n in ("-SomeAlgorithm", "SomeAlgorithm-", "Some,Alg:orithm"):
        with pytest.raises(factory.ConfigError):
            factory._validate_name(n)


def test_default_provider():
    """TestDefaultConfigExists / TestAlgorithmProviders (algorithmprovider/plugins_test.go:31-62)."""
    preds, prios = factory.get_algorithm_provider(factory.DefaultProvider)
    assert sorted(preds) == ["HostName", "MatchNodeSelector", "NoDiskConflict", "PodFitsPorts", "PodFitsResources"]
    assert sorted(prios) == ["EqualPriority", "LeastRequestedPriority", "ServiceSpreadingPriority"]
    assert all(factory.is_fit_predicate_registered(p) for p in preds)
    assert all(factory.is_priority_function_registered(p) for p in prios)
    cfg = factory.create_from_provider().compile(lambda k: 0)
    assert cfg.w_least_requested == 1 and cfg.w_service_spreading == 1 and cfg.w_equal == 0
    assert cfg.n_priority_configs == 3


def test_create_from_config_policy():
    """TestCreateFromConfig (factory/factory_test.go:53-93) with the built-in names."""
    cfg = factory.create_from_config("""{
        "kind": "Policy", "apiVersion": "v1",
        "predicates": [
            {"name": "TestZoneAffinity", "argument": {"serviceAffinity": {"labels": ["zone"]}}},
            {"name": "TestRequireZone", "argument": {"labelsPresence": {"labels": ["zone"], "presence": true}}},
            {"name": "PodFitsResources"}, {"name": "PodFitsPorts"}],
        "priorities": [
            {"name": "RackSpread", "weight": 3, "argument": {"serviceAntiAffinity": {"label": "rack"}}},
            {"name": "LeastRequestedPriority", "weight": 2},
            {"name": "ServiceSpreadingPriority", "weight": 1}]}""")
    keys = {"zone": 0, "rack": 1}
    c = cfg.compile(keys.__getitem__)
    assert c.predicates == (abi.PRED_SERVICEAFFINITY | abi.PRED_LABELSPRESENCE | abi.PRED_PODFITSRESOURCES
                            | abi.PRED_PODFITSPORTS)
    assert c.n_aff_labels == 1 and c.aff_key[0] == 0
    assert c.n_presence == 1 and c.presence_flag[0] == 1 and c.presence_keys[0][0] == 0
    assert c.n_anti == 1 and c.anti_key[0] == 1 and c.w_anti[0] == 3
    # trap (plugins.go:173-176): a registered name without argument keeps its registered weight
    assert c.w_least_requested == 1


def test_empty_policy_is_equal_priority():
    """TestCreateFromEmptyConfig (factory_test.go:95-115): no predicates, no priorities ->
    prioritizeNodes falls back to EqualPriority (generic_scheduler.go:139-141): every node scores 1."""
    cfg = factory.create_from_config("{}")
    nodes = [make_node(f"n{i}", 1000, 1000) for i in range(5)]
    rc, got = run_engine(OracleScheduler, cfg, nodes, [], [], Pod())
    assert rc == abi.KSG_OK and all(v == (0, 1) for v in got.values())


def test_all_zero_weights_is_fit_error():
    """prioritizeNodes skips weight-0 configs; all zero -> empty list -> FitError (a11 trap)."""
    cfg = factory.create_from_keys(["PodFitsResources"], ["EqualPriority"])
    c = cfg.compile(lambda k: 0)
    assert c.n_priority_configs == 1 and c.w_equal == 0
    from kubernetes_amd import ingest

    it = ingest.Interner()
    view = ingest.ClusterView([make_node("a", 1000, 1000)], [], it)
    o = OracleScheduler(c)
    o.set_cluster(view.arrays)
    rc, m, k, _ = o.begin(ingest.ingest_pods(view, [Pod()]), 0)
    assert rc == abi.KSG_NOFIT


def test_invalid_names_and_arguments():
    with pytest.raises(factory.ConfigError):
        factory.create_from_keys(["NoSuchPredicate"], [])
    with pytest.raises(factory.ConfigError):
        factory.create_from_keys([], ["NoSuchPriority"])
    with pytest.raises(factory.ConfigError):
        factory.create_from_config({"predicates": [{"name": "Unregistered"}]})
    with pytest.raises(factory.ConfigError):  # exactly one argument kind (plugins.go:86-88)
        factory.create_from_config({"predicates": [{"name": "Both", "argument": {
            "serviceAffinity": {"labels": ["a"]}, "labelsPresence": {"labels": ["b"]}}}]})
    with pytest.raises(factory.ConfigError):
        factory.create_from_config({"priorities": [{"name": "Unregistered", "weight": 1}]})


def test_fail_code_names():
    cfg = factory.create_from_provider()
    names = cfg.fail_code_names()
    assert names[abi.FAIL_PODFITSRESOURCES] == "PodFitsResources"
    assert names[abi.FAIL_HOSTNAME] == "HostName"


def test_weighted_sum_through_oracle():
    """combined[host] += score * weight over configs (generic_scheduler.go:146-158)."""
    cfg = factory.create_from_config({"priorities": [
        {"name": "PrefZone2", "weight": 4, "argument": {"labelPreference": {"label": "zone", "presence": True}}},
        {"name": "LeastRequestedPriority", "weight": 1}]})
    nodes = [make_node("a", 1000, 1000, labels={"zone": "z"}), make_node("b", 1000, 1000)]
    rc, got = run_engine(OracleScheduler, cfg, nodes, [], [], Pod())
    assert rc == abi.KSG_OK
    assert got["a"][1] == 4 * 10 + 10 and got["b"][1] == 10


@pytest.mark.parametrize("seed", range(6))
def test_pod_services_index_matches_scan(seed):
    """ClusterView.pod_services (indexed by each selector's first requirement) equals
    the plain GetPodServices scan: same namespace, selector matches the pod's labels,
    service-list order; empty and invalid selectors (SelectorFromSet's trap) match all."""
    import random

    from kubernetes_amd.api import Service, ServiceSpec
    from kubernetes_amd.ingest import ClusterView, Interner
    from kubernetes_amd.labels import selector_from_set

    rng = random.Random(seed)
    keys, vals = ["app", "tier", "zone", "bad key!"], ["a", "b", "c", "-bad-"]
    svcs = []
    for i in range(60):
        sel = {rng.choice(keys): rng.choice(vals) for _ in range(rng.randrange(0, 3))}
        svcs.append(Service(metadata=ObjectMeta(name=f"s{i}", namespace=rng.choice(["", "default", "x"])),
                            spec=ServiceSpec(selector=sel if sel or rng.random() < 0.5 else None)))
    view = ClusterView([make_node("n0", 1000, 1 << 30)], svcs, Interner())
    for j in range(300):
        labels = {k: rng.choice(vals) for k in rng.sample(keys, rng.randrange(0, 4))}
        pod = Pod(metadata=ObjectMeta(name=f"p{j}", namespace=rng.choice(["", "default", "x"]),
                                      labels=labels if labels or rng.random() < 0.5 else None))
        want = [i for i, s in enumerate(svcs) if s.metadata.namespace == pod.metadata.namespace
                and selector_from_set(s.spec.selector).matches(pod.metadata.labels)]
        assert view.pod_services(pod) == want


def test_weights_are_go_ints_and_wrap():
    """Policy weights are Go ints (plugin/pkg/scheduler/api/types.go:46: int64): compile()
    keeps any weight in int64 (the library runs weights past the window path's int32
    score bound on the exact kernels with int64 scores), refuses one outside it, and
    two builtin configs of one kind add up mod 2^64 like Go's combinedScores."""
    for w in (1 << 63, -(1 << 63) - 1):
        cfg = factory.create_from_config({"priorities": [
            {"name": f"HugePref{abs(w)}", "weight": w, "argument": {"labelPreference": {"label": "rack"}}}]})
        with pytest.raises(factory.ConfigError, match="outside Go's int"):
            cfg.compile(lambda k: 0)
    for w in ((1 << 63) - 1, -(1 << 63), 1 << 40, (1 << 31) - 1):
        ok = factory.create_from_config({"priorities": [
            {"name": f"Pref{w}", "weight": w, "argument": {"labelPreference": {"label": "rack"}}}]})
        assert ok.compile(lambda k: 0).w_pref[0] == w
    two = factory.SchedulerConfig({}, [factory.PriorityDesc("LeastRequestedPriority", (1 << 62) + 5),
                                       factory.PriorityDesc("LeastRequestedPriority", 3 << 61)])
    assert two.compile(lambda k: 0).w_least_requested == ((1 << 62) + 5 + (3 << 61)) - (1 << 64)


def test_policy_lists_past_the_window_caps_compile():
    """Six ServiceAntiAffinity priorities and twenty LabelPreference ones: the
    reference registers any number (plugins.go:81-183); the library takes them on
    the exact kernels (the window path keeps four anti-affinity terms in registers)."""
    prios = [{"name": f"Anti{i}", "weight": 1 + i, "argument": {"serviceAntiAffinity": {"label": "zone"}}}
             for i in range(6)]
    prios += [{"name": f"Pref{i}", "weight": 1, "argument": {"labelPreference": {"label": "rack"}}}
              for i in range(20)]
    cfg = factory.create_from_config({"priorities": prios}).compile(lambda k: 0)
    assert cfg.n_anti == 6 and cfg.n_label_pref == 20
    assert [cfg.w_anti[a] for a in range(6)] == [1, 2, 3, 4, 5, 6]
