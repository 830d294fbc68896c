"""Placement rule units beyond ``test_placement``: the MAX_PER counting core, the round-robin core,
task-type avoid/colocate against every pod instance, exact/regex matchers on every attribute
type, agent-rule helpers and region references through nested rules.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/offer/evaluate/placement/{MaxPerTest,
AbstractRoundRobinRuleTest,TaskTypeRuleTest,ExactMatcherTest,AttributeRuleTest,
PlacementUtilsTest}.java. The abstract-rule tests drive the shared base classes through small
subclasses whose keys are scripted, as the reference does.
"""
import json
import random
from types import SimpleNamespace

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.evaluate import placement as PL
from dcos_commons_amd.offer.taskdata.labels import TaskLabelWriter, attribute_to_string


def _pod(type_="test-pod-type", index=0):
    return SimpleNamespace(pod=SimpleNamespace(type=type_), index=index, name=f"{type_}-{index}")


def _offer(agent="test-agent"):
    o = P.Offer(hostname="test-hostname")
    o.id.value = "test-offer-id"
    o.framework_id.value = "test-framework-id"
    o.agent_id.value = agent
    return o


def _task(name="test-task-name", type_="different-type", index=100, agent="test-slave-id"):
    t = P.TaskInfo(name=name)
    t.task_id.value = name + "__uuid"
    t.agent_id.value = agent
    TaskLabelWriter(t).set_type(type_).set_index(index).apply()
    return t


# ---------------------------------------------------------------------------------------
# MaxPerRule core


class ScriptedMaxPer(PL._MaxPerRule):
    def __init__(self, max_, task_keys, offer_keys):
        super().__init__(max_, PL.AnyMatcher())
        self._task_keys, self._offer_keys = list(task_keys), list(offer_keys)

    def task_keys(self, task):
        return self._task_keys

    def offer_keys(self, offer):
        return self._offer_keys


def test_max_per_limit_zero_rejected():
    with pytest.raises(ValueError):
        PL.MaxPerHostnameRule(0)


@pytest.mark.parametrize("max_,task_keys,offer_keys,tasks,accepted", [
    (1, [], [], 0, True),                                        # nothing limits placement
    (1, [], [], 1, True),
    (1, ["key0"], [], 1, True),                                  # offer has no keys
    (1, ["key0"], ["key1"], 1, True),                            # different key
    (1, ["key0"], ["key0"], 1, False),                           # same key at the limit
    (1, ["key0", "key1"], ["key1"], 1, False),                   # one of several over the limit
    (2, ["key0", "key1", "key1"], ["key1"], 1, False),
    (1, ["key0", "key1"], ["key1", "key0"], 1, False),
    (2, ["key0", "key0", "key1", "key1"], ["key1", "key0"], 1, False),
    (1, ["key0", "key1"], ["key2", "key3"], 1, True),            # disjoint keys
])
def test_max_per_counting(max_, task_keys, offer_keys, tasks, accepted):
    rule = ScriptedMaxPer(max_, task_keys, offer_keys)
    assert rule.is_acceptable(_offer(), _pod(), [_task()] * tasks) is accepted


@pytest.mark.parametrize("max_,task_keys", [(1, ["key0"]), (2, ["key0", "key0"])])
def test_max_per_ignores_the_task_being_placed(max_, task_keys):
    pod = _pod()
    self_task = _task(type_=pod.pod.type, index=pod.index)
    assert ScriptedMaxPer(max_, task_keys, ["key0"]).is_acceptable(_offer(), pod, [self_task])


# ---------------------------------------------------------------------------------------
# Round-robin core


class ScriptedRoundRobin(PL._RoundRobinRule):
    def __init__(self, task_filter, count, offer_key, task_keys):
        super().__init__(count, task_filter)
        self._offer_key, self._task_keys = offer_key, task_keys
        self._i = 0

    def offer_key(self, offer):
        return self._offer_key

    def task_key(self, task):
        if self._task_keys is None:
            return None
        k = self._task_keys[self._i]
        self._i += 1
        return k


@pytest.mark.parametrize("task_filter,count,offer_key,task_keys,ntasks,passing", [
    (PL.AnyMatcher(), 1, None, None, 0, False),                          # offer lacks the key
    (PL.ExactMatcher.create("banana"), 1, "key0", None, 1, True),        # no task matches the filter
    (PL.AnyMatcher(), 1, "key0", None, 1, True),                         # tasks carry no key
    (PL.AnyMatcher(), 2, "key0", ["key0"], 1, False),                    # must spread to a 2nd key first
    (PL.AnyMatcher(), 2, "key1", ["key0"], 1, True),
    (PL.AnyMatcher(), 2, "key0", ["key0", "key1"], 2, True),             # second layer
    (PL.AnyMatcher(), 2, "key0", ["key0", "key1", "key0"], 3, False),    # key0 is full
])
def test_round_robin_core(task_filter, count, offer_key, task_keys, ntasks, passing):
    rule = ScriptedRoundRobin(task_filter, count, offer_key, task_keys)
    assert rule.filter(_offer(), _pod(), [_task()] * ntasks).is_passing() is passing


# ---------------------------------------------------------------------------------------
# TaskTypeRule


RNG = random.Random(7)


def _typed(type_, id_, agent):
    t = P.TaskInfo(name=id_.split("__")[0])
    t.task_id.value = id_
    t.agent_id.value = agent
    TaskLabelWriter(t).set_type(type_).set_index(RNG.randrange(1 << 30)).apply()
    return t


MATCH_1 = _typed("match", "matchtask-1__uuid", "agent1")
MATCH_3 = _typed("match", "matchtask-3__uuid", "agent3")
MISMATCH_1 = _typed("mismatch", "othertask-1__uuid", "agent1")
MISMATCH_2 = _typed("mismatch", "othertask-2__uuid", "agent2")
MISMATCH_3 = _typed("mismatch", "othertask-3__uuid", "agent3")
TASKS = [MISMATCH_1, MATCH_1, MISMATCH_2, MISMATCH_3, MATCH_3]
MISMATCHES = [MISMATCH_1, MISMATCH_2, MISMATCH_3]
OFFERS = [_offer("agent1"), _offer("agent2"), _offer("agent3")]
OTHER_POD = _pod("pod-type", 0)


def _pod_of(task):
    from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader

    r = TaskLabelReader(task)
    return _pod(r.get_type(), r.get_index())


def _results(rule, pod, tasks=TASKS):
    return [rule.filter(o, pod, tasks).is_passing() for o in OFFERS]


def test_task_type_label_is_read():
    assert PL.TaskTypeRule._task_type(_typed("hey", "hello-1234__uuid", "agent")) == "hey"
    assert PL.TaskTypeRule._task_type(P.TaskInfo(name="unlabelled")) is None


def test_colocate():
    assert _results(PL.TaskTypeRule.colocate_with("match"), OTHER_POD) == [True, False, True]


def test_avoid():
    assert _results(PL.TaskTypeRule.avoid("match"), OTHER_POD) == [False, True, False]


@pytest.mark.parametrize("task,colocate,avoid", [
    # the pod being placed ignores its own (stale) task
    (MATCH_1, [False, False, True], [True, True, False]),
    (MATCH_3, [True, False, False], [False, True, True]),
    (MISMATCH_1, [True, False, True], [False, True, False]),
    (MISMATCH_2, [True, False, True], [False, True, False]),
    (MISMATCH_3, [True, False, True], [False, True, False]),
])
def test_rules_with_the_pods_own_task_present(task, colocate, avoid):
    pod = _pod_of(task)
    assert _results(PL.TaskTypeRule.colocate_with("match"), pod) == colocate
    assert _results(PL.TaskTypeRule.avoid("match"), pod) == avoid


@pytest.mark.parametrize("rule", [PL.TaskTypeRule.colocate_with("match"), PL.TaskTypeRule.avoid("match")])
def test_no_task_of_the_type_running_passes_everywhere(rule):
    assert _results(rule, OTHER_POD, MISMATCHES) == [True, True, True]


@pytest.mark.parametrize("rule", [PL.TaskTypeRule.avoid("match"), PL.TaskTypeRule.colocate_with("match")])
def test_task_type_rule_round_trips(rule):
    assert PL.placement_rule_from_dict(json.loads(json.dumps(rule.to_dict()))) == rule


@pytest.mark.parametrize("doc", [
    {"@type": "TaskTypeRule", "type": "foo", "behavior": "AVOID"},
    {"@type": "TaskTypeRule", "type": "foo", "converter": {"@type": "TaskTypeLabelConverter"}, "behavior": "AVOID"},
])
def test_task_type_rule_documents(doc):
    rule = PL.placement_rule_from_dict(doc)
    assert rule == PL.TaskTypeRule.avoid("foo")


# ---------------------------------------------------------------------------------------
# ExactMatcher


@pytest.mark.parametrize("pattern,value,matches", [
    ("", "", True), ("", "foo", False), ("foo", "bar", False), ("foo", "foo", True), ("100", "100", True),
    ("100.0", "100", True), ("100", "100.0", True),
    ("100", "100.00001", True), ("100", "100.0001", True), ("100", "100.00011", True),  # 3-decimal comparison
    ("100", "100.01", False),
])
def test_exact_matcher(pattern, value, matches):
    assert PL.ExactMatcher.create(pattern).matches(value) is matches


# ---------------------------------------------------------------------------------------
# AttributeRule over every attribute type


def _attr(kind):
    if kind == "text":
        a = P.Attribute(name="footext", type=P.Value.TEXT)
        a.text.value = "bar"
    elif kind == "scalar":
        a = P.Attribute(name="fooscalar", type=P.Value.SCALAR)
        a.scalar.value = 123.456
    elif kind == "ranges":
        a = P.Attribute(name="fooranges", type=P.Value.RANGES)
        a.ranges.range.add(begin=234, end=345)
        a.ranges.range.add(begin=456, end=567)
    else:
        a = P.Attribute(name="fooset", type=P.Value.SET)
        a.set.item.extend(["bar", "baz"])
    return a


KINDS = ["text", "scalar", "ranges", "set"]
REGEX = {"text": "footext:...", "scalar": ".*:[0-9.]+", "ranges": ".*ranges:.+", "set": r".*:\{bar,baz\}"}


def _attr_offer(*kinds):
    o = _offer()
    for k in kinds:
        o.attributes.add().CopyFrom(_attr(k))
    return o


def _matcher(kind, how):
    return PL.ExactMatcher.create(attribute_to_string(_attr(kind))) if how == "exact" else \
        PL.RegexMatcher.create(REGEX[kind])


def _require(matcher, offer):
    return PL.RuleFactory(PL.AttributeRule).require(matcher).filter(offer, _pod(), []).is_passing()


@pytest.mark.parametrize("how", ["exact", "regex"])
def test_attribute_rule_matches_each_type_alone_and_together(how):
    for k in KINDS:
        assert _require(_matcher(k, how), _attr_offer(k)), k
        assert _require(_matcher(k, how), _attr_offer(*KINDS)), k


@pytest.mark.parametrize("how", ["exact", "regex"])
def test_attribute_rule_mismatches(how):
    assert [_require(_matcher(k, how), _attr_offer("scalar", "set")) for k in KINDS] == [False, True, False, True]
    assert [_require(_matcher(k, how), _attr_offer("ranges", "text")) for k in KINDS] == [True, False, True, False]


# ---------------------------------------------------------------------------------------
# PlacementUtils


def test_agent_placement_rule():
    assert PL.get_agent_placement_rule([], []) is None
    avoid = "NotRule{rule=OrRule{rules=[AgentRule{agentId=avoidme}, AgentRule{agentId=avoidme2}]}}"
    colocate = "OrRule{rules=[AgentRule{agentId=colocateme}, AgentRule{agentId=colocateme2}]}"
    assert repr(PL.get_agent_placement_rule(["avoidme", "avoidme2"], [])) == avoid
    assert repr(PL.get_agent_placement_rule([], ["colocateme", "colocateme2"])) == colocate
    assert repr(PL.get_agent_placement_rule(["avoidme", "avoidme2"], ["colocateme", "colocateme2"])) == \
        f"AndRule{{rules=[{avoid}, {colocate}]}}"


def _region():
    return PL.RegionRule(PL.ExactMatcher.create("region"))


def _zone():
    return PL.ZoneRule(PL.ExactMatcher.create("zone"))


def _attribute():
    return PL.AttributeRule(PL.ExactMatcher.create("attribute"))


@pytest.mark.parametrize("rule,references", [
    (None, False),
    (PL.PassthroughRule(), False),
    (_region(), True),
    (_zone(), False),
    (PL.OrRule([_region(), _zone()]), True),
    (PL.OrRule([_attribute(), _zone()]), False),
    (PL.AndRule([_attribute(), PL.OrRule([_region(), _zone()])]), True),
    (PL.AndRule([_attribute(), PL.OrRule([_attribute(), _zone()])]), False),
])
def test_references_region(rule, references):
    assert PL.references_region(SimpleNamespace(placement_rule=rule)) is references


def test_references_zone_through_not():
    assert PL.references_zone(SimpleNamespace(placement_rule=PL.NotRule(_zone())))
    assert not PL.references_zone(SimpleNamespace(placement_rule=PL.NotRule(_region())))
