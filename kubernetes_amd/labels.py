"""Label sets and the selector semantics the Filter/Score pass depends on.

  labels.Set.Has/Get/AsSelector            pkg/labels/labels.go:38-62
  SelectorFromSet (validation trap)        pkg/labels/selector.go:654-668
  NewRequirement / Requirement.Matches     pkg/labels/selector.go:91-165
  LabelSelector.Matches / Everything       pkg/labels/selector.go:195-202
  IsQualifiedName / IsValidLabelValue      pkg/util/validation.go:24-44

Trap reproduced: SelectorFromSet returns an EMPTY selector (matches everything)
if any key or value of the set fails validation. A nil or empty set also
matches everything. Host-side only: the kernels receive the interned
(key,value) pair ids of a valid selector, or an empty list.
"""
from __future__ import annotations

import re
from typing import Dict, List, Optional, Tuple

_QNAME_CHAR = "[A-Za-z0-9]"
_QNAME_EXT = "[-A-Za-z0-9_.]"
_QNAME_TOKEN = "(" + _QNAME_CHAR + _QNAME_EXT + "*)?" + _QNAME_CHAR
_LABEL_VALUE_RE = re.compile("(" + _QNAME_TOKEN + ")?")
_QUALIFIED_NAME_RE = re.compile("(" + _QNAME_TOKEN + "/)?" + _QNAME_TOKEN)
LABEL_VALUE_MAX_LENGTH = 63
QUALIFIED_NAME_MAX_LENGTH = 253


def is_qualified_name(v: str) -> bool:
    return len(v) <= QUALIFIED_NAME_MAX_LENGTH and _QUALIFIED_NAME_RE.fullmatch(v) is not None


def is_valid_label_value(v: str) -> bool:
    return len(v) <= LABEL_VALUE_MAX_LENGTH and _LABEL_VALUE_RE.fullmatch(v) is not None


class Selector:
    """A conjunction of key==value requirements (the only kind SelectorFromSet builds)."""

    __slots__ = ("requirements",)

    def __init__(self, requirements: Optional[List[Tuple[str, str]]] = None):
        self.requirements = sorted(requirements or [])

    def empty(self) -> bool:
        return not self.requirements

    def matches(self, labels: Optional[Dict[str, str]]) -> bool:
        labels = labels or {}
        for k, v in self.requirements:
            if k not in labels or labels[k] != v:
                return False
        return True

    def __repr__(self):
        return "Selector(" + ",".join(f"{k}={v}" for k, v in self.requirements) + ")"


def everything() -> Selector:
    return Selector([])


def selector_from_set(ls: Optional[Dict[str, str]]) -> Selector:
    """SelectorFromSet: invalid key/value anywhere -> empty selector (matches all)."""
    if ls is None:
        return Selector([])
    reqs = []
    for k, v in ls.items():
        if not is_qualified_name(k) or not is_valid_label_value(v):
            return Selector([])
        reqs.append((k, v))
    return Selector(reqs)


def set_has(ls: Optional[Dict[str, str]], key: str) -> bool:
    return bool(ls) and key in ls


def set_get(ls: Optional[Dict[str, str]], key: str) -> str:
    return (ls or {}).get(key, "")
