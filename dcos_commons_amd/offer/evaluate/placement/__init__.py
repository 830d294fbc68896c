"""Placement rules and the Marathon constraint language.

Reference: sdk/.../offer/evaluate/placement/*.java (38 files, 3.3K LoC). Every rule implements
``filter(offer, pod_instance, tasks) -> EvaluationOutcome`` and serializes with the Jackson
``@type`` discriminator (PlacementRule.java:24) so persisted ServiceSpecs keep their rules.

MI355X note: agents advertise ``gpu_vendor``/``gpu_model``/``gpu_arch``/``xgmi_hive`` attributes (see
``dcos_commons_amd.ops.gpu``: KFD topology / amd-smi discovery), so ``[["xgmi_hive","GROUP_BY","2"]]`` or
``[["hostname","MAX_PER","1"]]`` give topology-aware 1:1 GPU pinning with no special rule.
"""
from __future__ import annotations

import enum
import json
import logging
import re
from typing import Any, Dict, Iterable, List, Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.evaluate.outcome import EvaluationOutcome
from dcos_commons_amd.offer.taskdata.labels import (
    TaskException,
    TaskLabelReader,
    attribute_join,
    attribute_split,
    attribute_to_string,
    attribute_to_value,
    attribute_value_to_string,
)

LOGGER = logging.getLogger(__name__)


class PlacementField(enum.Enum):
    HOSTNAME = "HOSTNAME"
    ZONE = "ZONE"
    REGION = "REGION"
    ATTRIBUTE = "ATTRIBUTE"


_RULE_TYPES: Dict[str, type] = {}
_MATCHER_TYPES: Dict[str, type] = {}


def _rule(cls):
    _RULE_TYPES[cls.__name__] = cls
    return cls


def _matcher(cls):
    _MATCHER_TYPES[cls.__name__] = cls
    return cls


def _are_equivalent(task: P.TaskInfo, pod_instance) -> bool:
    try:
        r = TaskLabelReader(task)
        return r.get_index() == pod_instance.index and r.get_type() == pod_instance.pod.type
    except (TaskException, ValueError):
        return False


# ---------------------------------------------------------------------------------------
# string matchers


class StringMatcher:
    def matches(self, value: str) -> bool:
        raise NotImplementedError

    def to_dict(self) -> dict:
        raise NotImplementedError

    def __eq__(self, other):
        return type(self) is type(other) and self.to_dict() == other.to_dict()

    def __hash__(self):
        return hash(json.dumps(self.to_dict(), sort_keys=True))


def _fmt_number(s: str) -> str:
    """Java DecimalFormat("0.###") for numeric strings; others unchanged."""
    try:
        f = float(s)
    except (TypeError, ValueError):
        return s
    if f != f or f in (float("inf"), float("-inf")):
        return s
    out = ("%.3f" % f).rstrip("0").rstrip(".")
    return "0" if out in ("-0", "") else out


@_matcher
class ExactMatcher(StringMatcher):
    def __init__(self, string: str):
        self.string = _fmt_number(string)

    @staticmethod
    def create(s: str) -> "ExactMatcher":
        return ExactMatcher(s)

    @staticmethod
    def create_attribute(name: str, value: str) -> "ExactMatcher":
        return ExactMatcher(attribute_join(name, value))

    def matches(self, value: str) -> bool:
        return self.string == _fmt_number(value)

    def to_dict(self):
        return {"@type": "ExactMatcher", "string": self.string}

    def __repr__(self):
        return f"ExactMatcher{{str='{self.string}'}}"


@_matcher
class RegexMatcher(StringMatcher):
    def __init__(self, pattern: str):
        self.pattern = pattern
        self._re = re.compile(pattern)

    @staticmethod
    def create(p: str) -> "RegexMatcher":
        return RegexMatcher(p)

    @staticmethod
    def create_attribute(name: str, value: str) -> "RegexMatcher":
        return RegexMatcher(attribute_join(name, value))

    def matches(self, value: str) -> bool:
        return self._re.fullmatch(value) is not None

    def to_dict(self):
        return {"@type": "RegexMatcher", "pattern": self.pattern}

    def __repr__(self):
        return f"RegexMatcher{{pattern='{self.pattern}'}}"


@_matcher
class AnyMatcher(StringMatcher):
    def matches(self, value: str) -> bool:
        return True

    @staticmethod
    def create() -> "AnyMatcher":
        return AnyMatcher()

    def to_dict(self):
        return {"@type": "AnyMatcher"}

    def __repr__(self):
        return "AnyMatcher{}"


def matcher_from_dict(d: Optional[dict]) -> Optional[StringMatcher]:
    if d is None:
        return None
    t = d.get("@type")
    if t == "ExactMatcher":
        m = ExactMatcher.__new__(ExactMatcher)
        m.string = d.get("string")
        return m
    if t == "RegexMatcher":
        return RegexMatcher(d.get("pattern"))
    if t == "AnyMatcher":
        return AnyMatcher()
    raise ValueError(f"Unknown matcher type {t}")


# ---------------------------------------------------------------------------------------
# base rule


class PlacementRule:
    def filter(self, offer: P.Offer, pod_instance, tasks) -> EvaluationOutcome:
        raise NotImplementedError

    def placement_fields(self) -> List[PlacementField]:
        return []

    def to_dict(self) -> dict:
        raise NotImplementedError

    def __eq__(self, other):
        return isinstance(other, PlacementRule) and self.to_dict() == other.to_dict()

    def __hash__(self):
        return hash(json.dumps(self.to_dict(), sort_keys=True))


def placement_rule_from_dict(d: Optional[dict]) -> Optional[PlacementRule]:
    if d is None:
        return None
    t = d.get("@type")
    cls = _RULE_TYPES.get(t)
    if cls is None:
        raise ValueError(f"Unknown placement rule type {t}")
    return cls.from_dict(d)


def _opt(v) -> str:
    """Java ``Optional.toString`` rendering, so rule descriptions read like the reference's."""
    return "Optional.empty" if v is None else f"Optional[{v}]"


def _m(d, key="task-filter"):
    return matcher_from_dict(d.get(key)) if d.get(key) is not None else None


@_rule
class PassthroughRule(PlacementRule):
    def filter(self, offer, pod_instance, tasks):
        return EvaluationOutcome.pass_(self, "Passthrough rule always passes.")

    def to_dict(self):
        return {"@type": "PassthroughRule"}

    @classmethod
    def from_dict(cls, d):
        return cls()

    def __repr__(self):
        return "PassthroughRule{}"


@_rule
class AndRule(PlacementRule):
    def __init__(self, rules: Iterable[PlacementRule]):
        self.rules = list(rules)

    def filter(self, offer, pod_instance, tasks):
        if not self.rules:
            return EvaluationOutcome.fail(self, "No rules to AND together is treated as 'always fail'")
        children = [r.filter(offer, pod_instance, tasks) for r in self.rules]
        passing = sum(1 for c in children if c.passing)
        fn = EvaluationOutcome.pass_ if passing == len(self.rules) else EvaluationOutcome.fail
        return fn(self, "%d of %d rules are passing:", passing, len(self.rules), children=children)

    def placement_fields(self):
        return [f for r in self.rules for f in r.placement_fields()]

    def to_dict(self):
        return {"@type": "AndRule", "rules": [r.to_dict() for r in self.rules]}

    @classmethod
    def from_dict(cls, d):
        return cls([placement_rule_from_dict(r) for r in d.get("rules") or ()])

    def __repr__(self):
        return f"AndRule{{rules={self.rules}}}"


@_rule
class OrRule(PlacementRule):
    def __init__(self, rules: Iterable[PlacementRule]):
        self.rules = list(rules)

    def filter(self, offer, pod_instance, tasks):
        if not self.rules:
            return EvaluationOutcome.fail(self, "No rules to OR together is treated as 'always fail'")
        children = [r.filter(offer, pod_instance, tasks) for r in self.rules]
        passing = sum(1 for c in children if c.passing)
        fn = EvaluationOutcome.pass_ if passing else EvaluationOutcome.fail
        return fn(self, "%d of %d rules are passing:", passing, len(self.rules), children=children)

    def placement_fields(self):
        return [f for r in self.rules for f in r.placement_fields()]

    def to_dict(self):
        return {"@type": "OrRule", "rules": [r.to_dict() for r in self.rules]}

    @classmethod
    def from_dict(cls, d):
        return cls([placement_rule_from_dict(r) for r in d.get("rules") or ()])

    def __repr__(self):
        return f"OrRule{{rules={self.rules}}}"


@_rule
class NotRule(PlacementRule):
    def __init__(self, rule: PlacementRule):
        self.rule = rule

    def filter(self, offer, pod_instance, tasks):
        child = self.rule.filter(offer, pod_instance, tasks)
        fn = EvaluationOutcome.fail if child.passing else EvaluationOutcome.pass_
        return fn(self, "Returning opposite of child rule", children=[child])

    def placement_fields(self):
        return self.rule.placement_fields()

    def to_dict(self):
        return {"@type": "NotRule", "rule": self.rule.to_dict()}

    @classmethod
    def from_dict(cls, d):
        return cls(placement_rule_from_dict(d["rule"]))

    def __repr__(self):
        return f"NotRule{{rule={self.rule}}}"


@_rule
class InvalidPlacementRule(PlacementRule):
    def __init__(self, constraints: str, exception: str):
        self.constraints = constraints
        self.exception = exception

    def filter(self, offer, pod_instance, tasks):
        return EvaluationOutcome.fail(
            self, "Invalid placement constraints for %s: %s", pod_instance.name, self.constraints)

    def to_dict(self):
        return {"@type": "InvalidPlacementRule", "constraints": self.constraints, "exception": self.exception}

    @classmethod
    def from_dict(cls, d):
        return cls(d.get("constraints") or d.get("constraints "), d.get("exception"))

    def __repr__(self):
        return f"InvalidPlacementRule{{constraints={self.constraints}, exception={self.exception}}}"


@_rule
class AgentRule(PlacementRule):
    def __init__(self, agent_id: str):
        self.agent_id = agent_id

    @staticmethod
    def require(*agent_ids) -> PlacementRule:
        ids = list(agent_ids[0]) if len(agent_ids) == 1 and not isinstance(agent_ids[0], str) else list(agent_ids)
        if len(ids) == 1 and len(agent_ids) == 1 and isinstance(agent_ids[0], str):
            return AgentRule(ids[0])
        return OrRule([AgentRule(a) for a in ids])

    @staticmethod
    def avoid(*agent_ids) -> PlacementRule:
        return NotRule(AgentRule.require(*agent_ids))

    def filter(self, offer, pod_instance, tasks):
        if offer.agent_id.value == self.agent_id:
            return EvaluationOutcome.pass_(self, "Offer matches required Agent ID '%s'", self.agent_id)
        return EvaluationOutcome.fail(self, "Offer lacks required Agent ID. Wanted: '%s' Got: '%s'",
                                      self.agent_id, offer.agent_id.value)

    def to_dict(self):
        return {"@type": "AgentRule", "agent-id": self.agent_id}

    @classmethod
    def from_dict(cls, d):
        return cls(d.get("agent-id"))

    def __repr__(self):
        return f"AgentRule{{agentId={self.agent_id}}}"


# -- string matcher rules ----------------------------------------------------------------


class _StringMatcherRule(PlacementRule):
    NAME = ""
    FIELD: Optional[PlacementField] = None

    def __init__(self, matcher: StringMatcher):
        self.matcher = matcher

    def keys(self, offer) -> List[str]:
        raise NotImplementedError

    def is_acceptable(self, offer) -> bool:
        return any(self.matcher.matches(k) for k in self.keys(offer))

    def placement_fields(self):
        return [self.FIELD]

    def to_dict(self):
        return {"@type": type(self).__name__, "matcher": self.matcher.to_dict()}

    @classmethod
    def from_dict(cls, d):
        return cls(matcher_from_dict(d["matcher"]))

    def __repr__(self):
        return f"{type(self).__name__}{{matcher={self.matcher}}}"


def _has_fault_domain(offer) -> bool:
    return offer.HasField("domain") and offer.domain.HasField("fault_domain")


@_rule
class HostnameRule(_StringMatcherRule):
    FIELD = PlacementField.HOSTNAME

    def keys(self, offer):
        return [offer.hostname]

    def filter(self, offer, pod_instance, tasks):
        if self.is_acceptable(offer):
            return EvaluationOutcome.pass_(self, "Offer hostname matches pattern: '%s'", self.matcher)
        return EvaluationOutcome.fail(self, "Offer hostname didn't match pattern: '%s'", self.matcher)


@_rule
class ZoneRule(_StringMatcherRule):
    FIELD = PlacementField.ZONE

    def keys(self, offer):
        return [offer.domain.fault_domain.zone.name] if _has_fault_domain(offer) else []

    def filter(self, offer, pod_instance, tasks):
        if not (_has_fault_domain(offer) and offer.domain.fault_domain.HasField("zone")):
            return EvaluationOutcome.fail(self, "Offer does not contain a zone.")
        if self.is_acceptable(offer):
            return EvaluationOutcome.pass_(self, "Offer zone matches pattern: '%s'", self.matcher)
        return EvaluationOutcome.fail(self, "Offer zone didn't match pattern: '%s'", self.matcher)


@_rule
class RegionRule(_StringMatcherRule):
    FIELD = PlacementField.REGION

    def keys(self, offer):
        return [offer.domain.fault_domain.region.name] if _has_fault_domain(offer) else []

    def filter(self, offer, pod_instance, tasks):
        if not _has_fault_domain(offer):
            return EvaluationOutcome.fail(self, "Offer does not contain a region.")
        if self.is_acceptable(offer):
            return EvaluationOutcome.pass_(self, "Offer region matches pattern: '%s'", self.matcher)
        return EvaluationOutcome.fail(self, "Offer region didn't match pattern: '%s'", self.matcher)


@_rule
class AttributeRule(_StringMatcherRule):
    FIELD = PlacementField.ATTRIBUTE

    def keys(self, offer):
        return [attribute_to_string(a) for a in offer.attributes]

    def filter(self, offer, pod_instance, tasks):
        if self.is_acceptable(offer):
            return EvaluationOutcome.pass_(self, "Match found for attribute pattern: '%s'", self.matcher)
        return EvaluationOutcome.fail(self, "None of %d attributes matched pattern: '%s'",
                                      len(offer.attributes), self.matcher)


class RuleFactory:
    """``require``/``avoid`` take one matcher, several, or one collection of them; several become
    an OrRule (negated for ``avoid``) (RuleFactory.java defaults, PlacementUtils.require)."""

    def __init__(self, cls):
        self.cls = cls

    @staticmethod
    def _matchers(matchers) -> List[StringMatcher]:
        if len(matchers) == 1 and not isinstance(matchers[0], StringMatcher):
            return list(matchers[0])
        return list(matchers)

    def require(self, *matchers) -> PlacementRule:
        ms = self._matchers(matchers)
        return self.cls(ms[0]) if len(ms) == 1 else OrRule([self.cls(m) for m in ms])

    def avoid(self, *matchers) -> PlacementRule:
        return NotRule(self.require(*matchers))


HostnameRuleFactory = RuleFactory(HostnameRule)
ZoneRuleFactory = RuleFactory(ZoneRule)
RegionRuleFactory = RuleFactory(RegionRule)
AttributeRuleFactory = RuleFactory(AttributeRule)


@_rule
class IsLocalRegionRule(PlacementRule):
    """Passes offers in the master's region (or with no region info)."""

    local_domain: Optional[P.DomainInfo] = None

    @classmethod
    def set_local_domain(cls, domain: Optional[P.DomainInfo]) -> None:
        cls.local_domain = domain

    def filter(self, offer, pod_instance, tasks):
        if not _has_fault_domain(offer):
            return EvaluationOutcome.pass_(self, "The Offer has no Region, so it is in the local region.")
        local = IsLocalRegionRule.local_domain
        if local is None or not local.HasField("fault_domain"):
            return EvaluationOutcome.pass_(
                self, "The Master has not reported a FaultDomain on registration, "
                      "so all offers are presumed to be in local region.")
        offer_region = offer.domain.fault_domain.region.name
        local_region = local.fault_domain.region.name
        if offer_region == local_region:
            return EvaluationOutcome.pass_(self, "The offer is in the local region: '%s'", local_region)
        return EvaluationOutcome.fail(self, "The offer is in region: '%s' NOT the local region: '%s'",
                                      offer_region, local_region)

    def placement_fields(self):
        return [PlacementField.REGION]

    def to_dict(self):
        return {"@type": "IsLocalRegionRule"}

    @classmethod
    def from_dict(cls, d):
        return cls()

    def __repr__(self):
        return "IsLocalRegionRule"


# -- MAX_PER -----------------------------------------------------------------------------


class _MaxPerRule(PlacementRule):
    FIELD: PlacementField = PlacementField.HOSTNAME

    def __init__(self, max: int, task_filter: Optional[StringMatcher] = None):
        if max is None or max < 1:
            raise ValueError("max must be >= 1")
        self.max = int(max)
        self.task_filter = task_filter or AnyMatcher()

    def task_keys(self, task) -> List[str]:
        raise NotImplementedError

    def offer_keys(self, offer) -> List[str]:
        raise NotImplementedError

    def is_acceptable(self, offer, pod_instance, tasks) -> bool:
        counts: Dict[str, int] = {}
        offer_keys = self.offer_keys(offer)
        for k in offer_keys:
            counts[k] = counts.get(k, 0) + 1
        okeys = set(offer_keys)
        for task in tasks:
            if not self.task_filter.matches(task.name) or _are_equivalent(task, pod_instance):
                continue
            for k in self.task_keys(task):
                if k in okeys:
                    counts[k] = counts.get(k, 0) + 1
        return all(v <= self.max for v in counts.values())

    def placement_fields(self):
        return [self.FIELD]

    def to_dict(self):
        return {"@type": type(self).__name__, "max": self.max, "task-filter": self.task_filter.to_dict()}

    @classmethod
    def from_dict(cls, d):
        return cls(d["max"], _m(d))

    def __repr__(self):
        return f"{type(self).__name__}{{max={self.max}, task-filter={self.task_filter}}}"


@_rule
class MaxPerHostnameRule(_MaxPerRule):
    FIELD = PlacementField.HOSTNAME

    def task_keys(self, task):
        try:
            return [TaskLabelReader(task).get_hostname()]
        except TaskException:
            return []

    def offer_keys(self, offer):
        return [offer.hostname]

    def filter(self, offer, pod_instance, tasks):
        if self.is_acceptable(offer, pod_instance, tasks):
            return EvaluationOutcome.pass_(self, "Fewer than %d tasks matching filter '%s' are present on this host",
                                           self.max, self.task_filter)
        return EvaluationOutcome.fail(self, "%d tasks matching filter '%s' are already present on this host",
                                      self.max, self.task_filter)


@_rule
class MaxPerZoneRule(_MaxPerRule):
    FIELD = PlacementField.ZONE

    def task_keys(self, task):
        z = TaskLabelReader(task).get_zone()
        return [z] if z is not None else []

    def offer_keys(self, offer):
        return [offer.domain.fault_domain.zone.name] if _has_fault_domain(offer) else []

    def filter(self, offer, pod_instance, tasks):
        if not (_has_fault_domain(offer) and offer.domain.fault_domain.HasField("zone")):
            return EvaluationOutcome.fail(self, "Offer does not contain a zone.")
        if self.is_acceptable(offer, pod_instance, tasks):
            return EvaluationOutcome.pass_(self, "Fewer than %d tasks matching filter '%s' are present in this zone",
                                           self.max, self.task_filter)
        return EvaluationOutcome.fail(self, "%d tasks matching filter '%s' are already present in this zone",
                                      self.max, self.task_filter)


@_rule
class MaxPerRegionRule(_MaxPerRule):
    FIELD = PlacementField.REGION

    def task_keys(self, task):
        r = TaskLabelReader(task).get_region()
        return [r] if r is not None else []

    def offer_keys(self, offer):
        return [offer.domain.fault_domain.region.name] if _has_fault_domain(offer) else []

    def filter(self, offer, pod_instance, tasks):
        if not _has_fault_domain(offer):
            return EvaluationOutcome.fail(self, "Offer does not contain a region.")
        if self.is_acceptable(offer, pod_instance, tasks):
            return EvaluationOutcome.pass_(self, "Fewer than %d tasks matching filter '%s' are present in this region",
                                           self.max, self.task_filter)
        return EvaluationOutcome.fail(self, "%d tasks matching filter '%s' are already present in this region",
                                      self.max, self.task_filter)


@_rule
class MaxPerAttributeRule(_MaxPerRule):
    FIELD = PlacementField.ATTRIBUTE

    def __init__(self, max: int, matcher: StringMatcher, task_filter: Optional[StringMatcher] = None):
        super().__init__(max, task_filter)
        self.matcher = matcher

    def task_keys(self, task):
        if not self.task_filter.matches(task.name):
            return []
        return [a for a in TaskLabelReader(task).get_offer_attribute_strings() if self.matcher.matches(a)]

    def offer_keys(self, offer):
        return [s for s in (attribute_to_string(a) for a in offer.attributes) if self.matcher.matches(s)]

    def filter(self, offer, pod_instance, tasks):
        if self.is_acceptable(offer, pod_instance, tasks):
            return EvaluationOutcome.pass_(
                self, "Fits within limit of %d tasks matching filter '%s' on this agent with attribute: %s",
                self.max, self.task_filter, self.matcher)
        return EvaluationOutcome.fail(
            self, "Reached greater than %d tasks matching filter '%s' on this agent with attribute: %s",
            self.max, self.task_filter, self.matcher)

    def to_dict(self):
        d = super().to_dict()
        d["matcher"] = self.matcher.to_dict()
        return d

    @classmethod
    def from_dict(cls, d):
        return cls(d["max"], matcher_from_dict(d["matcher"]), _m(d))

    def __repr__(self):
        return f"MaxPerAttributeRule{{max={self.max}, matcher={self.matcher}, task-filter={self.task_filter}}}"


# -- GROUP_BY (round robin) --------------------------------------------------------------


class _RoundRobinRule(PlacementRule):
    FIELD: PlacementField = PlacementField.HOSTNAME
    COUNT_KEY = "agent-count"

    def __init__(self, distinct_key_count: Optional[int] = None, task_filter: Optional[StringMatcher] = None):
        self.distinct_key_count = distinct_key_count
        self.task_filter = task_filter or AnyMatcher()

    def offer_key(self, offer) -> Optional[str]:
        raise NotImplementedError

    def task_key(self, task) -> Optional[str]:
        raise NotImplementedError

    def filter(self, offer, pod_instance, tasks):
        offer_key = self.offer_key(offer)
        if offer_key is None:
            return EvaluationOutcome.fail(self, "Offer lacks needed information for round robin placement")
        counts: Dict[str, int] = {}
        for task in tasks:
            if not self.task_filter.matches(task.name) or _are_equivalent(task, pod_instance):
                continue
            k = self.task_key(task)
            if k is None:
                continue
            counts[k] = counts.get(k, 0) + 1
        max_known = max(counts.values()) if counts else 0
        min_known = min(counts.values()) if counts else 0
        offer_count = counts.get(offer_key, 0)
        if min_known == max_known or offer_count <= min_known:
            if self.distinct_key_count is None:
                return EvaluationOutcome.pass_(
                    self, "Distinct key count is unspecified, and '%s' has %d instances while others have %d to %d",
                    offer_key, offer_count, min_known, max_known)
            if len(counts) >= self.distinct_key_count:
                return EvaluationOutcome.pass_(
                    self, "All distinct keys are found, and '%s' has %d instances while others have %d to %d",
                    offer_key, offer_count, min_known, max_known)
            if offer_count == 0:
                return EvaluationOutcome.pass_(self, "Other keys have zero usage, and so does key '%s'", offer_key)
            return EvaluationOutcome.fail(self, "Other keys have zero instances, but key '%s' has %d",
                                          offer_key, offer_count)
        return EvaluationOutcome.fail(self, "Key '%s' is already full, and others are known to not be full",
                                      offer_key)

    def placement_fields(self):
        return [self.FIELD]

    def to_dict(self):
        return {"@type": type(self).__name__, self.COUNT_KEY: self.distinct_key_count,
                "task-filter": self.task_filter.to_dict()}

    @classmethod
    def from_dict(cls, d):
        return cls(d.get(cls.COUNT_KEY), _m(d))

    def __repr__(self):
        return f"{type(self).__name__}{{{self.COUNT_KEY}={_opt(self.distinct_key_count)}, task-filter={self.task_filter}}}"


@_rule
class RoundRobinByHostnameRule(_RoundRobinRule):
    FIELD = PlacementField.HOSTNAME
    COUNT_KEY = "agent-count"

    def offer_key(self, offer):
        return offer.hostname

    def task_key(self, task):
        try:
            return TaskLabelReader(task).get_hostname()
        except TaskException:
            return None


@_rule
class RoundRobinByZoneRule(_RoundRobinRule):
    FIELD = PlacementField.ZONE
    COUNT_KEY = "zone-count"

    def offer_key(self, offer):
        if _has_fault_domain(offer) and offer.domain.fault_domain.HasField("zone"):
            return offer.domain.fault_domain.zone.name
        return None

    def task_key(self, task):
        return TaskLabelReader(task).get_zone()


@_rule
class RoundRobinByRegionRule(_RoundRobinRule):
    FIELD = PlacementField.REGION
    COUNT_KEY = "region-count"

    def offer_key(self, offer):
        if _has_fault_domain(offer):
            return offer.domain.fault_domain.region.name
        return None

    def task_key(self, task):
        return TaskLabelReader(task).get_region()


@_rule
class RoundRobinByAttributeRule(_RoundRobinRule):
    FIELD = PlacementField.ATTRIBUTE
    COUNT_KEY = "value-count"

    def __init__(self, attribute_name: str, distinct_key_count: Optional[int] = None,
                 task_filter: Optional[StringMatcher] = None):
        super().__init__(distinct_key_count, task_filter)
        self.attribute_name = attribute_name

    def offer_key(self, offer):
        for a in offer.attributes:
            if a.name.lower() == self.attribute_name.lower():
                return attribute_value_to_string(attribute_to_value(a))
        return None

    def task_key(self, task):
        for s in TaskLabelReader(task).get_offer_attribute_strings():
            name, value = attribute_split(s)
            if name.lower() == self.attribute_name.lower():
                return value
        return None

    def to_dict(self):
        d = super().to_dict()
        d["name"] = self.attribute_name
        return d

    @classmethod
    def from_dict(cls, d):
        return cls(d.get("name"), d.get(cls.COUNT_KEY), _m(d))

    def __repr__(self):
        return (f"RoundRobinByAttributeRule{{attribute={self.attribute_name}, "
                f"attribute-count={_opt(self.distinct_key_count)}, task-filter={self.task_filter}}}")


# -- task type affinity ------------------------------------------------------------------


@_rule
class TaskTypeRule(PlacementRule):
    AVOID = "AVOID"
    COLOCATE = "COLOCATE"

    def __init__(self, type_to_find: str, behavior: str):
        self.type_to_find = type_to_find
        self.behavior = behavior

    @staticmethod
    def avoid(t: str) -> "TaskTypeRule":
        return TaskTypeRule(t, TaskTypeRule.AVOID)

    @staticmethod
    def colocate_with(t: str) -> "TaskTypeRule":
        return TaskTypeRule(t, TaskTypeRule.COLOCATE)

    @staticmethod
    def _task_type(task) -> Optional[str]:
        try:
            return TaskLabelReader(task).get_type()
        except TaskException:
            return None

    def filter(self, offer, pod_instance, tasks):
        matching = [t for t in tasks if self._task_type(t) == self.type_to_find]
        if self.behavior == self.AVOID:
            if not matching:
                return EvaluationOutcome.pass_(self, "No tasks of avoided type '%s' are currently running.",
                                               self.type_to_find)
            for t in matching:
                if _are_equivalent(t, pod_instance):
                    continue
                if t.agent_id.value == offer.agent_id.value:
                    return EvaluationOutcome.fail(self, "Found a task matching avoided type '%s' on this agent.",
                                                  self.type_to_find)
            return EvaluationOutcome.pass_(self, "No tasks of avoided type '%s' found on this agent.",
                                           self.type_to_find)
        if not matching:
            return EvaluationOutcome.pass_(self, "No tasks of colocated type '%s' are currently running.",
                                           self.type_to_find)
        for t in matching:
            if _are_equivalent(t, pod_instance):
                continue
            if t.agent_id.value == offer.agent_id.value:
                return EvaluationOutcome.pass_(self, "Found a task matching colocated type '%s' on this agent.",
                                               self.type_to_find)
        return EvaluationOutcome.fail(self, "Didn't find a task matching colocated type '%s' on this agent.",
                                      self.type_to_find)

    def to_dict(self):
        return {"@type": "TaskTypeRule", "type": self.type_to_find,
                "converter": {"@type": "TaskTypeLabelConverter"}, "behavior": self.behavior}

    @classmethod
    def from_dict(cls, d):
        return cls(d["type"], d["behavior"])

    def __repr__(self):
        return f"TaskTypeRule{{type={self.type_to_find}, behavior={self.behavior}}}"


# ---------------------------------------------------------------------------------------
# helpers (PlacementUtils)

HOSTNAME_FIELD_LEGACY = "hostname"
HOSTNAME_FIELD = "@hostname"
REGION_FIELD = "@region"
ZONE_FIELD = "@zone"


def get_field(name: str) -> PlacementField:
    if name in (HOSTNAME_FIELD_LEGACY, HOSTNAME_FIELD):
        return PlacementField.HOSTNAME
    if name == REGION_FIELD:
        return PlacementField.REGION
    if name == ZONE_FIELD:
        return PlacementField.ZONE
    return PlacementField.ATTRIBUTE


def get_agent_placement_rule(avoid_agents: List[str], colocate_agents: List[str]) -> Optional[PlacementRule]:
    if avoid_agents:
        if colocate_agents:
            return AndRule([AgentRule.avoid(avoid_agents), AgentRule.require(colocate_agents)])
        return AgentRule.avoid(avoid_agents)
    if colocate_agents:
        return AgentRule.require(colocate_agents)
    return None


def placement_rule_references(field: PlacementField, pod_spec) -> bool:
    rule = pod_spec.placement_rule
    return rule is not None and field in rule.placement_fields()


def references_region(pod_spec) -> bool:
    return placement_rule_references(PlacementField.REGION, pod_spec)


def references_zone(pod_spec) -> bool:
    return placement_rule_references(PlacementField.ZONE, pod_spec)


def has_zone(offer) -> bool:
    return _has_fault_domain(offer) and offer.domain.fault_domain.HasField("zone")


# ---------------------------------------------------------------------------------------
# Marathon constraint parser (MarathonConstraintParser.java:36-503)


class ConstraintParseError(ValueError):
    pass


def escaped_split(s: str, split: str) -> List[str]:
    vals, buf, escaped = [], [], False
    for c in s:
        if escaped:
            if c == split:
                buf.append(c)
            else:
                buf.append("\\")
                buf.append(c)
            escaped = False
        elif c == "\\":
            escaped = True
        elif c == split:
            vals.append("".join(buf).strip())
            buf = []
        else:
            buf.append(c)
    if escaped:
        buf.append("\\")
    vals.append("".join(buf).strip())
    return vals


def split_constraints(constraints: str) -> List[List[str]]:
    try:
        parsed = json.loads(constraints)
        if isinstance(parsed, list) and all(isinstance(x, str) for x in parsed):
            return [parsed]
        if isinstance(parsed, list) and all(isinstance(x, list) and all(isinstance(y, str) for y in x)
                                            for x in parsed):
            return parsed
    except ValueError:
        pass
    return [escaped_split(row, ":") for row in escaped_split(constraints, ",")]


def _required(op: str, param: Optional[str]) -> str:
    if param is None:
        raise ConstraintParseError(f"Missing required parameter for operator '{op}'.")
    return param


def _int_param(op: str, param: Optional[str]) -> int:
    try:
        return int(_required(op, param))
    except ValueError:
        raise ConstraintParseError(f"Unable to parse max parameter as integer for '{op}' operation: {param}")


def _by_field(field_name: str, hostname, zone, region, attribute):
    f = get_field(field_name)
    return {PlacementField.HOSTNAME: hostname, PlacementField.ZONE: zone,
            PlacementField.REGION: region, PlacementField.ATTRIBUTE: attribute}[f]()


def _parse_row(task_filter: StringMatcher, row: List[str]) -> PlacementRule:
    if len(row) < 2 or len(row) > 3:
        raise ConstraintParseError(f"Invalid number of entries in rule. Expected 2 or 3, got {len(row)}: {row}")
    field_name, op = row[0], row[1]
    param = row[2] if len(row) >= 3 else None
    opu = op.upper()
    if opu in ("IS", "CLUSTER"):
        p = _required(op, param)
        return _by_field(field_name,
                         lambda: HostnameRuleFactory.require(ExactMatcher.create(p)),
                         lambda: ZoneRuleFactory.require(ExactMatcher.create(p)),
                         lambda: RegionRuleFactory.require(ExactMatcher.create(p)),
                         lambda: AttributeRuleFactory.require(ExactMatcher.create_attribute(field_name, p)))
    if opu == "UNIQUE":
        def attr():
            m = RegexMatcher.create_attribute(field_name, ".*")
            return AndRule([AttributeRuleFactory.require(m), MaxPerAttributeRule(1, m, task_filter)])
        return _by_field(field_name, lambda: MaxPerHostnameRule(1, task_filter),
                         lambda: MaxPerZoneRule(1, task_filter), lambda: MaxPerRegionRule(1, task_filter), attr)
    if opu == "GROUP_BY":
        num = None
        if param is not None:
            try:
                num = int(param)
            except ValueError:
                raise ConstraintParseError(
                    f"Unable to parse max parameter as integer for '{op}' operation: {param}")
        return _by_field(field_name, lambda: RoundRobinByHostnameRule(num, task_filter),
                         lambda: RoundRobinByZoneRule(num, task_filter),
                         lambda: RoundRobinByRegionRule(num, task_filter),
                         lambda: RoundRobinByAttributeRule(field_name, num, task_filter))
    if opu == "LIKE":
        p = _required(op, param)
        return _by_field(field_name,
                         lambda: HostnameRuleFactory.require(RegexMatcher.create(p)),
                         lambda: ZoneRuleFactory.require(RegexMatcher.create(p)),
                         lambda: RegionRuleFactory.require(RegexMatcher.create(p)),
                         lambda: AttributeRuleFactory.require(RegexMatcher.create_attribute(field_name, p)))
    if opu == "UNLIKE":
        p = _required(op, param)
        return _by_field(field_name,
                         lambda: HostnameRuleFactory.avoid(RegexMatcher.create(p)),
                         lambda: ZoneRuleFactory.avoid(RegexMatcher.create(p)),
                         lambda: RegionRuleFactory.avoid(RegexMatcher.create(p)),
                         lambda: AttributeRuleFactory.avoid(RegexMatcher.create_attribute(field_name, p)))
    if opu == "MAX_PER":
        mx = _int_param(op, param)

        def attr():
            m = RegexMatcher.create_attribute(field_name, ".*")
            return AndRule([AttributeRuleFactory.require(m), MaxPerAttributeRule(mx, m, task_filter)])
        return _by_field(field_name, lambda: MaxPerHostnameRule(mx, task_filter),
                         lambda: MaxPerZoneRule(mx, task_filter), lambda: MaxPerRegionRule(mx, task_filter), attr)
    raise ConstraintParseError(
        f"Unsupported operator: '{op}' in constraint: {row} "
        "(expected one of: UNIQUE, CLUSTER, GROUP_BY, LIKE, UNLIKE, or MAX_PER)")


def parse_marathon_constraints(pod_name: str, constraints: Optional[str]) -> PlacementRule:
    """``[["hostname","UNIQUE"]]`` (JSON), ``hostname:UNIQUE,...`` (colon/comma) -> rule."""
    if constraints is None or constraints == "" or constraints == "[]":
        return PassthroughRule()
    try:
        rows = split_constraints(constraints)
        task_filter = RegexMatcher.create(pod_name + "-.*")
        if len(rows) == 1:
            return _parse_row(task_filter, rows[0])
        return AndRule([_parse_row(task_filter, r) for r in rows])
    except (ConstraintParseError, re.error) as e:
        LOGGER.error("Failed to parse marathon constraints [%s] for %s", constraints, pod_name)
        return InvalidPlacementRule(constraints, str(e))
