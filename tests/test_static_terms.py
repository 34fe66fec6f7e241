"""Static node terms past ksg_config's fixed slots (factory.SchedulerConfig.split_static /
static_terms, folded in by ksg_set_static_terms): the host evaluation against the
object-level restatement (oracle/ref_model: CheckNodeLabelPresence,
predicates.go:194-229; CalculateNodeLabelPriority, priorities.go:98-134; Go-int sums,
generic_scheduler.go:145-159)."""
import numpy as np

from kubernetes_amd import abi, factory
from kubernetes_amd.ingest import ClusterView, Interner
from oracle import ref_model as R
from tests.test_oracle_crosscheck import _policy_many_labels, _workload


def test_split_keeps_slots_and_extras():
    cfg = _policy_many_labels()
    p_slot, p_extra, l_slot, l_extra = cfg.split_static()
    assert len(p_slot) == abi.MAX_PRESENCE and len(l_slot) == abi.MAX_LABEL_PREF
    assert any(len(d.labels) > abi.MAX_PRESENCE_KEYS for d in p_extra)
    assert len(p_slot) + len(p_extra) == abi.MAX_PRESENCE + 4
    assert len(l_slot) + len(l_extra) == abi.MAX_LABEL_PREF + 4
    c = cfg.compile(Interner().key_id)  # no ConfigError past the slots
    assert c.n_presence == abi.MAX_PRESENCE and c.n_label_pref == abi.MAX_LABEL_PREF
    assert c.n_priority_configs == abi.MAX_LABEL_PREF + 5


def test_static_terms_match_ref_model():
    w = _workload("policy_many_labels", 97, 4)
    cfg = w.config
    view = ClusterView(w.nodes, [], Interner())
    fit, score, weighted = cfg.static_terms(view.nodes)
    _, p_extra, _, l_extra = cfg.split_static()
    info = R.NodeInfo(view.nodes)
    preds = [R.new_node_label_predicate(info, d.labels, d.presence) for d in p_extra]
    for i, n in enumerate(view.nodes):
        want = all(p(None, [], n.metadata.name) for p in preds)
        assert bool((int(fit[i >> 6]) >> (i & 63)) & 1) == want, n.metadata.name
    want_s = np.zeros(len(view.nodes), np.int64)
    for p in l_extra:
        for i, (host, s) in enumerate(R.new_node_label_priority(p.label, p.presence)(None, None, view.nodes)):
            assert host == view.nodes[i].metadata.name
            want_s[i] = factory._go_int(int(want_s[i]) + s * p.weight)
    assert np.array_equal(score, want_s) and weighted
    assert 0 < int(sum(bin(int(x)).count("1") for x in fit)) < len(view.nodes)  # some nodes fail, some pass


def test_go_int_wrap_of_extra_weights():
    big = (1 << 62) + 3
    cfg = factory.create_from_config({
        "predicates": [{"name": "PodFitsResources"}],
        "priorities": [{"name": f"P{j}", "weight": big, "argument": {"labelPreference": {"label": "zone",
                                                                                            "presence": True}}}
                       for j in range(abi.MAX_LABEL_PREF + 2)]})
    w = _workload("policy_many_labels", 5, 1)
    _, _, l_slot, l_extra = cfg.split_static()
    assert len(l_extra) == 2
    fit, score, weighted = cfg.static_terms(w.nodes)
    assert fit is None and weighted
    assert int(score[0]) == factory._go_int(2 * 10 * big)
