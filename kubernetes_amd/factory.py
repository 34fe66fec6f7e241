"""Predicate / priority registry, algorithm providers and Policy compilation.

Mirrors plugin/pkg/scheduler/factory/plugins.go:31-248,
plugin/pkg/scheduler/algorithmprovider/defaults/defaults.go:26-72 and
plugin/pkg/scheduler/api/types.go:23-103. Instead of a map of Go closures the
registry holds *descriptions* of the built-in and policy-configured
predicates/priorities; `SchedulerConfig.compile()` turns a selection of them
into the `ksg_config` the HIP kernels are specialised with.

Reference traps kept:
  * RegisterCustomPriorityFunction for an already-registered name with no
    argument reuses the registered factory, so the Policy weight is IGNORED
    (plugins.go:173-176): {"name":"LeastRequestedPriority","weight":5} still
    has weight 1.
  * Priority configs are instantiated in sorted name order (plugins.go:235-248);
    weight-0 configs are skipped by prioritizeNodes; all-zero => empty list.
"""
from __future__ import annotations

import json
import re
import threading
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional

from . import abi

DefaultProvider = "DefaultProvider"

_I64_MIN, _I64_MAX = -(1 << 63), (1 << 63) - 1


def _go_int(x: int) -> int:
    """x wrapped to Go's int (int64, two's complement)."""
    return ((int(x) + (1 << 63)) % (1 << 64)) - (1 << 63)
_VALID_NAME = re.compile(r"[a-zA-Z0-9]([-a-zA-Z0-9]*[a-zA-Z0-9])")


class ConfigError(ValueError):
    pass


@dataclass(frozen=True)
class PredicateDesc:
    kind: str  # PodFitsPorts | PodFitsResources | NoDiskConflict | MatchNodeSelector | HostName
    #          | ServiceAffinity | LabelsPresence
    labels: tuple = ()
    presence: bool = False


@dataclass(frozen=True)
class PriorityDesc:
    kind: str  # LeastRequestedPriority | ServiceSpreadingPriority | EqualPriority
    #          | ServiceAntiAffinity | LabelPreference
    weight: int = 1
    label: str = ""
    presence: bool = False


_BUILTIN_PRED_BITS = {
    "PodFitsPorts": abi.PRED_PODFITSPORTS,
    "PodFitsResources": abi.PRED_PODFITSRESOURCES,
    "NoDiskConflict": abi.PRED_NODISKCONFLICT,
    "MatchNodeSelector": abi.PRED_MATCHNODESELECTOR,
    "HostName": abi.PRED_HOSTNAME,
    "ServiceAffinity": abi.PRED_SERVICEAFFINITY,
    "LabelsPresence": abi.PRED_LABELSPRESENCE,
}

_lock = threading.Lock()
_fit_predicates: Dict[str, PredicateDesc] = {}
_priorities: Dict[str, PriorityDesc] = {}
_providers: Dict[str, tuple] = {}


def _validate_name(name: str):
    if not _VALID_NAME.fullmatch(name):
        raise ConfigError(f"algorithm name {name} does not match the name validation regexp")


def register_fit_predicate(name: str, desc: PredicateDesc) -> str:
    """RegisterFitPredicate / RegisterFitPredicateFactory (plugins.go:63-77)."""
    with _lock:
        _validate_name(name)
        _fit_predicates[name] = desc
    return name


def register_priority_function(name: str, desc: PriorityDesc) -> str:
    """RegisterPriorityFunction / RegisterPriorityConfigFactory (plugins.go:127-141)."""
    with _lock:
        _validate_name(name)
        _priorities[name] = desc
    return name


def register_algorithm_provider(name: str, predicate_keys: Iterable[str], priority_keys: Iterable[str]) -> str:
    with _lock:
        _validate_name(name)
        _providers[name] = (frozenset(predicate_keys), frozenset(priority_keys))
    return name


def get_algorithm_provider(name: str):
    with _lock:
        if name not in _providers:
            raise ConfigError(f"plugin {name!r} has not been registered")
        return _providers[name]


def is_fit_predicate_registered(name: str) -> bool:
    with _lock:
        return name in _fit_predicates


def is_priority_function_registered(name: str) -> bool:
    with _lock:
        return name in _priorities


def register_custom_fit_predicate(policy: dict) -> str:
    """RegisterCustomFitPredicate (plugins.go:81-117)."""
    name = policy["name"]
    arg = policy.get("argument")
    desc = None
    if arg is not None:
        sa, lp = arg.get("serviceAffinity"), arg.get("labelsPresence")
        if (sa is not None) + (lp is not None) != 1:
            raise ConfigError("Exactly 1 predicate argument is required")
        if sa is not None:
            desc = PredicateDesc("ServiceAffinity", labels=tuple(sa.get("labels") or ()))
        else:
            desc = PredicateDesc("LabelsPresence", labels=tuple(lp.get("labels") or ()),
                                 presence=bool(lp.get("presence", False)))
    else:
        with _lock:
            desc = _fit_predicates.get(name)
    if desc is None:
        raise ConfigError(f"Invalid configuration: Predicate type not found for {name}")
    return register_fit_predicate(name, desc)


def register_custom_priority_function(policy: dict) -> str:
    """RegisterCustomPriorityFunction (plugins.go:145-183)."""
    name = policy["name"]
    weight = int(policy.get("weight", 0))
    arg = policy.get("argument")
    if arg is not None:
        saa, lpf = arg.get("serviceAntiAffinity"), arg.get("labelPreference")
        if (saa is not None) + (lpf is not None) != 1:
            raise ConfigError("Exactly 1 priority argument is required")
        if saa is not None:
            desc = PriorityDesc("ServiceAntiAffinity", weight=weight, label=saa.get("label", ""))
        else:
            desc = PriorityDesc("LabelPreference", weight=weight, label=lpf.get("label", ""),
                                presence=bool(lpf.get("presence", False)))
        return register_priority_function(name, desc)
    with _lock:
        if name in _priorities:
            return name  # reused as registered: the policy's weight is ignored
    raise ConfigError(f"Invalid configuration: Priority type not found for {name}")


# ---- DefaultProvider (algorithmprovider/defaults/defaults.go:26-72) --------
def _register_defaults():
    preds = [
        register_fit_predicate("PodFitsPorts", PredicateDesc("PodFitsPorts")),
        register_fit_predicate("PodFitsResources", PredicateDesc("PodFitsResources")),
        register_fit_predicate("NoDiskConflict", PredicateDesc("NoDiskConflict")),
        register_fit_predicate("MatchNodeSelector", PredicateDesc("MatchNodeSelector")),
        register_fit_predicate("HostName", PredicateDesc("HostName")),
    ]
    prios = [
        register_priority_function("LeastRequestedPriority", PriorityDesc("LeastRequestedPriority", 1)),
        register_priority_function("ServiceSpreadingPriority", PriorityDesc("ServiceSpreadingPriority", 1)),
        register_priority_function("EqualPriority", PriorityDesc("EqualPriority", 0)),
    ]
    register_algorithm_provider(DefaultProvider, preds, prios)


_register_defaults()


# ---- compiled configuration -------------------------------------------------
@dataclass
class SchedulerConfig:
    """The selected predicates and priorities (what NewGenericScheduler receives)."""

    predicates: Dict[str, PredicateDesc]
    priorities: List[PriorityDesc]  # in sorted name order, weight-0 entries included
    priority_names: List[str] = field(default_factory=list)
    max_conflict_keys: int = 4096
    max_domains: int = 4096

    def label_keys(self) -> List[str]:
        """Every label key the configuration refers to (interned at context creation)."""
        ks = []
        for d in self.predicates.values():
            ks.extend(d.labels)
        for p in self.priorities:
            if p.label:
                ks.append(p.label)
        return ks

    def affinity_labels(self) -> List[str]:
        """Union of ServiceAffinity labels over every ServiceAffinity predicate (equivalent
        to their conjunction: one peer, pod-given labels never overridden)."""
        out = []
        for name in sorted(self.predicates):
            d = self.predicates[name]
            if d.kind == "ServiceAffinity":
                for l in d.labels:
                    if l not in out:
                        out.append(l)
        return out

    def fail_code_names(self) -> Dict[int, str]:
        """KSG_FAIL_* -> a predicate name for FailedPredicateMap (one failing name per
        node, as findNodesThatFit records; the reference's pick is Go-map order)."""
        by_kind: Dict[str, str] = {}
        for name in sorted(self.predicates):
            by_kind.setdefault(self.predicates[name].kind, name)
        codes = {
            abi.FAIL_HOSTNAME: "HostName",
            abi.FAIL_LABELSPRESENCE: "LabelsPresence",
            abi.FAIL_MATCHNODESELECTOR: "MatchNodeSelector",
            abi.FAIL_NODISKCONFLICT: "NoDiskConflict",
            abi.FAIL_PODFITSPORTS: "PodFitsPorts",
            abi.FAIL_PODFITSRESOURCES: "PodFitsResources",
            abi.FAIL_SERVICEAFFINITY: "ServiceAffinity",
        }
        return {c: by_kind.get(kind, kind) for c, kind in codes.items()}

    def split_static(self):
        """The static node terms that fit ksg_config's slots and the ones past them:
        (slotted LabelsPresence, extra LabelsPresence, slotted LabelPreference, extra
        LabelPreference). Extras are evaluated on the device per node in slot passes
        (static_passes, ksg_add_static_config): the reference registers any number
        of them (plugins.go:81-117, 145-183)."""
        p_slot, p_extra = [], []
        for name in sorted(self.predicates):
            d = self.predicates[name]
            if d.kind == "LabelsPresence":
                fits = len(p_slot) < abi.MAX_PRESENCE and len(d.labels) <= abi.MAX_PRESENCE_KEYS
                (p_slot if fits else p_extra).append(d)
        l_slot, l_extra = [], []
        for p in self.priorities:
            if p.kind == "LabelPreference":
                (l_slot if len(l_slot) < abi.MAX_LABEL_PREF else l_extra).append(p)
        return p_slot, p_extra, l_slot, l_extra

    def static_passes(self, key_id) -> List[abi.KsgConfig]:
        """The extra static terms as slot passes for ksg_add_static_config, evaluated
        on the device per node: a LabelsPresence predicate passes a node iff every
        label's presence matches (CheckNodeLabelPresence, predicates.go:194-229; a
        predicate with more keys than a slot holds is split over slots, their AND is
        the same); a LabelPreference priority scores 10 where the label's presence
        matches, else 0 (CalculateNodeLabelPriority, priorities.go:98-134), times its
        weight, summed as Go ints (generic_scheduler.go:145-159). key_id interns a
        label key (the ids of the cluster's label pairs)."""
        _, p_extra, _, l_extra = self.split_static()
        pres = []  # (keys, presence) per slot
        for d in p_extra:
            keys = list(d.labels)
            for at in range(0, max(len(keys), 1), abi.MAX_PRESENCE_KEYS):
                pres.append((keys[at:at + abi.MAX_PRESENCE_KEYS], bool(d.presence)))
        out = []
        n_pass = max((len(pres) + abi.MAX_PRESENCE - 1) // abi.MAX_PRESENCE,
                     (len(l_extra) + abi.MAX_LABEL_PREF - 1) // abi.MAX_LABEL_PREF)
        for k in range(n_pass):
            c = abi.KsgConfig()
            ps = pres[k * abi.MAX_PRESENCE:(k + 1) * abi.MAX_PRESENCE]
            c.n_presence = len(ps)
            for q, (keys, presence) in enumerate(ps):
                c.presence_n_keys[q] = len(keys)
                for i, l in enumerate(keys):
                    c.presence_keys[q][i] = key_id(l)
                c.presence_flag[q] = 1 if presence else 0
            ls = l_extra[k * abi.MAX_LABEL_PREF:(k + 1) * abi.MAX_LABEL_PREF]
            c.n_label_pref = len(ls)
            for q, p in enumerate(ls):
                c.pref_key[q] = key_id(p.label)
                c.pref_presence[q] = 1 if p.presence else 0
                c.w_pref[q] = _go_int(int(p.weight))
            out.append(c)
        return out

    def compile(self, key_id) -> abi.KsgConfig:
        """-> ksg_config. key_id(label_key) interns a label key to its id. Static
        terms past the config's slots are left to static_passes / ksg_add_static_config."""
        cfg = abi.KsgConfig()
        bits = 0
        for name in sorted(self.predicates):
            bits |= _BUILTIN_PRED_BITS[self.predicates[name].kind]
        cfg.predicates = bits
        presence, _, prefs, _ = self.split_static()
        cfg.n_presence = len(presence)
        for q, d in enumerate(presence):
            cfg.presence_n_keys[q] = len(d.labels)
            for i, l in enumerate(d.labels):
                cfg.presence_keys[q][i] = key_id(l)
            cfg.presence_flag[q] = 1 if d.presence else 0
        aff = self.affinity_labels()
        if len(aff) > abi.MAX_AFF:
            raise ConfigError("too many ServiceAffinity labels")
        cfg.n_aff_labels = len(aff)
        for j, l in enumerate(aff):
            cfg.aff_key[j] = key_id(l)
        # one label group per ServiceAffinity predicate: SelectorFromSet's trap
        # empties one predicate's selector only (predicates.go:311-315)
        groups = []
        for name in sorted(self.predicates):
            d = self.predicates[name]
            if d.kind == "ServiceAffinity" and d.labels:
                m = 0
                for l in d.labels:
                    m |= 1 << aff.index(l)
                if m not in groups:
                    groups.append(m)
        if len(groups) > abi.MAX_AFF_GROUPS:
            raise ConfigError("too many ServiceAffinity predicates")
        cfg.n_aff_groups = len(groups)
        for g, m in enumerate(groups):
            cfg.aff_group_mask[g] = m
        cfg.n_priority_configs = len(self.priorities)
        n_anti = n_pref = 0
        for p in self.priorities:
            # Policy weights are Go ints (plugin/pkg/scheduler/api/types.go:46: int64),
            # and combined scores wrap like them (generic_scheduler.go:145-159): two
            # configs of one kind add up to their summed weight, mod 2^64
            if not (_I64_MIN <= int(p.weight) <= _I64_MAX):
                raise ConfigError(f"priority weight {p.weight} of {p.kind} is outside Go's int")
        for p in self.priorities:
            if p.kind == "LeastRequestedPriority":
                cfg.w_least_requested = _go_int(cfg.w_least_requested + p.weight)
            elif p.kind == "ServiceSpreadingPriority":
                cfg.w_service_spreading = _go_int(cfg.w_service_spreading + p.weight)
            elif p.kind == "EqualPriority":
                cfg.w_equal = _go_int(cfg.w_equal + p.weight)
            elif p.kind == "ServiceAntiAffinity":
                if n_anti == abi.MAX_ANTI:
                    raise ConfigError("too many ServiceAntiAffinity priorities")
                cfg.anti_key[n_anti] = key_id(p.label)
                cfg.w_anti[n_anti] = p.weight
                n_anti += 1
            elif p.kind == "LabelPreference":
                if n_pref == len(prefs):
                    continue  # (past the slots: a static term, static_terms)
                cfg.pref_key[n_pref] = key_id(p.label)
                cfg.pref_presence[n_pref] = 1 if p.presence else 0
                cfg.w_pref[n_pref] = p.weight
                n_pref += 1
        cfg.n_anti = n_anti
        cfg.n_label_pref = n_pref
        cfg.max_conflict_keys = self.max_conflict_keys
        cfg.max_domains = self.max_domains
        return cfg


def create_from_keys(predicate_keys: Iterable[str], priority_keys: Iterable[str], **kw) -> SchedulerConfig:
    """ConfigFactory.CreateFromKeys (factory.go:107-124, plugins.go:220-248)."""
    with _lock:
        preds = {}
        for name in sorted(set(predicate_keys)):
            if name not in _fit_predicates:
                raise ConfigError(f"Invalid predicate name {name!r} specified - no corresponding function found")
            preds[name] = _fit_predicates[name]
        prios, names = [], []
        for name in sorted(set(priority_keys)):
            if name not in _priorities:
                raise ConfigError(f"Invalid priority name {name} specified - no corresponding function found")
            prios.append(_priorities[name])
            names.append(name)
    return SchedulerConfig(preds, prios, names, **kw)


def create_from_provider(provider: str = DefaultProvider, **kw) -> SchedulerConfig:
    preds, prios = get_algorithm_provider(provider)
    return create_from_keys(preds, prios, **kw)


def create_from_config(policy, **kw) -> SchedulerConfig:
    """ConfigFactory.CreateFromConfig (factory.go:88-104); policy is a dict or JSON text."""
    if isinstance(policy, (str, bytes)):
        policy = json.loads(policy)
    pk = [register_custom_fit_predicate(p) for p in policy.get("predicates") or []]
    rk = [register_custom_priority_function(p) for p in policy.get("priorities") or []]
    return create_from_keys(pk, rk, **kw)
