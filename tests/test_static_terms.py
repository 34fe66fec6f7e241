"""Static node terms past ksg_config's fixed slots (factory.SchedulerConfig.split_static /
static_passes, evaluated on the device by ksg_add_static_config): the slot passes,
evaluated here the way ksg_static_kernel does (every key of a presence slot, the
passes ANDed / their scores Go-int summed), against the object-level restatement
(oracle/ref_model: CheckNodeLabelPresence, predicates.go:194-229;
CalculateNodeLabelPriority, priorities.go:98-134; Go-int sums,
generic_scheduler.go:145-159). The device evaluation itself is checked on the GPU
(tests/test_gpu_scheduler_api.py, policy_many_labels)."""
import numpy as np

from kubernetes_amd import abi, factory
from kubernetes_amd.ingest import ClusterView, Interner
from oracle import ref_model as R
from tests.test_oracle_crosscheck import N_PREF, N_U, _policy_many_labels, _workload


def test_split_keeps_slots_and_extras():
    cfg = _policy_many_labels()
    p_slot, p_extra, l_slot, l_extra = cfg.split_static()
    assert len(p_slot) == abi.MAX_PRESENCE and len(l_slot) == abi.MAX_LABEL_PREF
    assert any(len(d.labels) > abi.MAX_PRESENCE_KEYS for d in p_extra)
    assert len(p_slot) + len(p_extra) == N_U + 3
    assert len(l_slot) + len(l_extra) == N_PREF
    c = cfg.compile(Interner().key_id)  # no ConfigError past the slots
    assert c.n_presence == abi.MAX_PRESENCE and c.n_label_pref == abi.MAX_LABEL_PREF
    assert c.n_priority_configs == N_PREF + 1
    assert len(cfg.static_passes(Interner().key_id)) == 2  # (LabelPreference: 36 past the slots)


def _eval_passes(cfg, nodes):
    """ksg_static_kernel over the slot passes (test-side restatement of the kernel)."""
    it = Interner()
    passes = cfg.static_passes(it.key_id)
    n = len(nodes)
    fit = np.ones(n, bool)
    score = np.zeros(n, np.int64)
    has_fit = any(c.n_presence for c in passes)
    has_score = any(c.n_label_pref for c in passes)
    weighted = any(int(c.w_pref[q]) != 0 for c in passes for q in range(c.n_label_pref))
    for i, node in enumerate(nodes):
        labels = set((node.metadata.labels or {}).keys())
        ids = {it.key_id(l) for l in labels}
        for c in passes:
            for q in range(c.n_presence):
                for k in range(c.presence_n_keys[q]):
                    if (int(c.presence_keys[q][k]) in ids) != bool(c.presence_flag[q]):
                        fit[i] = False
            for q in range(c.n_label_pref):
                ok = (int(c.pref_key[q]) in ids) == bool(c.pref_presence[q])
                score[i] = factory._go_int(int(score[i]) + int(c.w_pref[q]) * (10 if ok else 0))
    words = np.zeros((n + 63) // 64, np.uint64)
    for i in np.nonzero(fit)[0]:
        words[i >> 6] |= np.uint64(1) << np.uint64(i & 63)
    return (words if has_fit else None), (score if has_score else None), weighted


def test_static_passes_match_ref_model():
    w = _workload("policy_many_labels", 97, 4)
    cfg = w.config
    view = ClusterView(w.nodes, [], Interner())
    fit, score, weighted = _eval_passes(cfg, view.nodes)
    assert len(cfg.static_passes(Interner().key_id)) >= 1
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
    fit, score, weighted = _eval_passes(cfg, w.nodes)
    assert fit is None and weighted
    assert int(score[0]) == factory._go_int(2 * 10 * big)
