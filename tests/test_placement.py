"""Placement rules and the Marathon constraint parser.

Behavior pinned against the reference's placement test suite
(sdk/scheduler/src/test/java/com/mesosphere/sdk/offer/evaluate/placement/*Test.java):
MarathonConstraintParserTest (split/escape tables, rule rendering per operator, invalid forms),
RoundRobinBy*RuleTest (rollout sequences with and without a distinct-key count), MaxPer*RuleTest,
TaskTypeRuleTest, And/Or/Not/Passthrough and IsLocalRegionRuleTest. Scenarios are written fresh
against this SDK's API; rule descriptions follow the reference's ``toString`` text.
"""
from types import SimpleNamespace

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.evaluate import placement as PL
from dcos_commons_amd.offer.taskdata.labels import TaskLabelWriter, scalar_attribute, text_attribute

POD = "hello"


def pod(type_="hello", index=99):
    return SimpleNamespace(pod=SimpleNamespace(type=type_), index=index, name=f"{type_}-{index}")


def offer(host="host1", agent=None, attrs=(), zone=None, region=None):
    o = P.Offer()
    o.id.value = f"offer-{host}"
    o.agent_id.value = agent or f"agent-{host}"
    o.framework_id.value = "fw"
    o.hostname = host
    for a in attrs:
        o.attributes.add().CopyFrom(a)
    if region is not None:
        o.domain.fault_domain.region.name = region
        o.domain.fault_domain.zone.name = zone or ""
    return o


def task(name, host="host1", type_="other", index=0, attrs=(), zone=None, region=None, agent=None):
    t = P.TaskInfo(name=name)
    t.task_id.value = name + "__id"
    o = offer(host, agent=agent, attrs=attrs, zone=zone, region=region)
    t.agent_id.CopyFrom(o.agent_id)
    w = TaskLabelWriter(t)
    w.set_hostname(o)
    w.set_type(type_)
    w.set_index(index)
    if attrs:
        w.set_offer_attributes(o)
    if zone is not None:
        w.set_zone(zone)
    if region is not None:
        w.set_region(region)
    t.labels.CopyFrom(w.to_proto())
    return t


def passes(rule, o, tasks=(), pi=None):
    return rule.filter(o, pi or pod(), list(tasks)).is_passing()


# ---------------------------------------------------------------------------------------
# constraint string splitting (MarathonConstraintParserTest.testSplitConstraints / testSplit*)


@pytest.mark.parametrize("raw,expected", [
    ("", [[""]]),
    ("a", [["a"]]),
    ('["a", "b", "c"]', [["a", "b", "c"]]),
    ('[["a", "b", "c"]]', [["a", "b", "c"]]),
    ('[["a", "b", "c"], ["d", "e"]]', [["a", "b", "c"], ["d", "e"]]),
    ('[["a"], []]', [["a"], []]),
    ("a:b:c,d:e,f:g:", [["a", "b", "c"], ["d", "e"], ["f", "g", ""]]),
    ("a:b:c,:d:e,:f:", [["a", "b", "c"], ["", "d", "e"], ["", "f", ""]]),
    (" a : b : c , : d : e , : f : ", [["a", "b", "c"], ["", "d", "e"], ["", "f", ""]]),
    ("::,:", [["", "", ""], ["", ""]]),
])
def test_split_constraints(raw, expected):
    assert PL.split_constraints(raw) == expected


@pytest.mark.parametrize("raw,expected", [
    ("hi,hey", ["hi", "hey"]),
    ("hi\\,hey", ["hi,hey"]),
    ("hi\\,,hey", ["hi,", "hey"]),
    ("hi,\\,hey", ["hi", ",hey"]),
    ("hi,,   ,  hey  ", ["hi", "", "", "hey"]),
])
def test_escaped_split(raw, expected):
    assert PL.escaped_split(raw, ",") == expected


# ---------------------------------------------------------------------------------------
# operator → rule rendering; every operator accepts the nested-JSON, flat-JSON and colon forms


def _forms(row):
    q = ", ".join(f'"{x}"' for x in row)
    return [f"[[{q}]]", f"[{q}]", ":".join(row)]


FILTER = "task-filter=RegexMatcher{pattern='hello-.*'}"


@pytest.mark.parametrize("row,expected", [
    (["hostname", "UNIQUE"], "MaxPerHostnameRule{max=1, " + FILTER + "}"),
    (["rack-id", "UNIQUE"], "AndRule{rules=[AttributeRule{matcher=RegexMatcher{pattern='rack-id:.*'}}, "
                            "MaxPerAttributeRule{max=1, matcher=RegexMatcher{pattern='rack-id:.*'}, " + FILTER + "}]}"),
    (["rack-id", "CLUSTER", "rack-1"], "AttributeRule{matcher=ExactMatcher{str='rack-id:rack-1'}}"),
    (["hostname", "CLUSTER", "a.specific.node.com"], "HostnameRule{matcher=ExactMatcher{str='a.specific.node.com'}}"),
    (["rack-id", "GROUP_BY"], "RoundRobinByAttributeRule{attribute=rack-id, attribute-count=Optional.empty, "
                              + FILTER + "}"),
    (["rack-id", "GROUP_BY", "3"], "RoundRobinByAttributeRule{attribute=rack-id, attribute-count=Optional[3], "
                                   + FILTER + "}"),
    (["zone", "GROUP_BY", "3"], "RoundRobinByAttributeRule{attribute=zone, attribute-count=Optional[3], "
                                + FILTER + "}"),
    (["hostname", "GROUP_BY"], "RoundRobinByHostnameRule{agent-count=Optional.empty, " + FILTER + "}"),
    (["hostname", "GROUP_BY", "3"], "RoundRobinByHostnameRule{agent-count=Optional[3], " + FILTER + "}"),
    (["rack-id", "LIKE", "rack-[1-3]"], "AttributeRule{matcher=RegexMatcher{pattern='rack-id:rack-[1-3]'}}"),
    (["hostname", "LIKE", "rack-[1-3]"], "HostnameRule{matcher=RegexMatcher{pattern='rack-[1-3]'}}"),
    (["foo", "IS", "bar"], "AttributeRule{matcher=ExactMatcher{str='foo:bar'}}"),
    (["@region", "IS", "bar"], "RegionRule{matcher=ExactMatcher{str='bar'}}"),
    (["@zone", "IS", "bar"], "ZoneRule{matcher=ExactMatcher{str='bar'}}"),
    (["@hostname", "IS", "bar"], "HostnameRule{matcher=ExactMatcher{str='bar'}}"),
    (["rack-id", "UNLIKE", "rack-[7-9]"], "NotRule{rule=AttributeRule{matcher=RegexMatcher{pattern='rack-id:rack-[7-9]'}}}"),
    (["hostname", "UNLIKE", "rack-[7-9]"], "NotRule{rule=HostnameRule{matcher=RegexMatcher{pattern='rack-[7-9]'}}}"),
    (["rack-id", "MAX_PER", "2"], "AndRule{rules=[AttributeRule{matcher=RegexMatcher{pattern='rack-id:.*'}}, "
                                  "MaxPerAttributeRule{max=2, matcher=RegexMatcher{pattern='rack-id:.*'}, " + FILTER + "}]}"),
    (["hostname", "MAX_PER", "2"], "MaxPerHostnameRule{max=2, " + FILTER + "}"),
])
def test_operator_rendering(row, expected):
    for form in _forms(row):
        assert repr(PL.parse_marathon_constraints(POD, form)) == expected, form


def test_many_operators_is_an_and_rule_in_order():
    colon = ("hostname:UNIQUE,rack-id:CLUSTER:rack-1,rack-id:GROUP_BY,rack-id:LIKE:rack-[1-3],"
             "rack-id:UNLIKE:rack-[7-9],rack-id:MAX_PER:2")
    js = ('[["hostname", "UNIQUE"], ["rack-id", "CLUSTER", "rack-1"], ["rack-id", "GROUP_BY"], '
          '["rack-id", "LIKE", "rack-[1-3]"], ["rack-id", "UNLIKE", "rack-[7-9]"],["rack-id", "MAX_PER", "2"]]')
    a, b = PL.parse_marathon_constraints(POD, colon), PL.parse_marathon_constraints(POD, js)
    assert repr(a) == repr(b)
    assert isinstance(a, PL.AndRule) and len(a.rules) == 6
    assert [type(r).__name__ for r in a.rules] == [
        "MaxPerHostnameRule", "AttributeRule", "RoundRobinByAttributeRule", "AttributeRule", "NotRule", "AndRule"]


def test_escaped_separators_in_regex():
    assert repr(PL.parse_marathon_constraints(POD, "rack-id:LIKE:rack-{1\\,3}")) == \
        "AttributeRule{matcher=RegexMatcher{pattern='rack-id:rack-{1,3}'}}"
    assert repr(PL.parse_marathon_constraints(POD, "rack-id:LIKE:foo\\:bar\\:baz")) == \
        "AttributeRule{matcher=RegexMatcher{pattern='rack-id:foo:bar:baz'}}"


@pytest.mark.parametrize("raw", ["", "[]"])
def test_empty_constraints_pass_through(raw):
    r = PL.parse_marathon_constraints(POD, raw)
    assert repr(r) == "PassthroughRule{}"
    assert passes(r, offer())


@pytest.mark.parametrize("raw", [
    '[[\\"hostname\\",\\"MAX_PER\\",\\"1\\"]]',          # over-escaped
    '[["rack-id", "MAX_PER", "2"]',                      # missing ']]'
    "rack-id:MAX_PER:,",                                 # missing last element
    "rack-id:GROUP_BY:foo",                              # non-integer count
    "rack-id:MAX_PER:foo",
    '["hostname","UNIQUE"],[["hostname","LIKE","10.0.3.6"]',  # trailing tokens
    '["hostname","UNIQUE"],[',
    '[["hostname","UNIQUE"],["hostname","LIKE","10.0.3.6"]',
    '[["hostname","UNIQUE"]],',
    "rack-id:CLUSTER", "rack-id:LIKE", "rack-id:UNLIKE", "rack-id:MAX_PER",  # missing parameter
    "rack-id:FOO:foo",                                   # unknown operator
    "rack-id:LIKE:foo:bar",                              # too many elements
])
def test_invalid_constraints_never_match(raw):
    r = PL.parse_marathon_constraints(POD, raw)
    assert isinstance(r, PL.InvalidPlacementRule), raw
    out = r.filter(offer(), pod(), [])
    assert not out.is_passing()
    # An invalid rule survives serialization (it is persisted inside the ServiceSpec).
    again = PL.placement_rule_from_dict(r.to_dict())
    assert isinstance(again, PL.InvalidPlacementRule)


# ---------------------------------------------------------------------------------------
# JSON round trip of every rule type (rules are persisted inside the ServiceSpec config)


def _all_rules():
    rx = PL.RegexMatcher.create("hello-.*")
    return [
        PL.PassthroughRule(),
        PL.HostnameRule(PL.ExactMatcher.create("h1")),
        PL.ZoneRule(PL.RegexMatcher.create("z.*")),
        PL.RegionRule(PL.AnyMatcher.create()),
        PL.AttributeRule(PL.ExactMatcher.create_attribute("rack", "r1")),
        PL.MaxPerHostnameRule(2, rx),
        PL.MaxPerZoneRule(1, rx),
        PL.MaxPerRegionRule(3, rx),
        PL.MaxPerAttributeRule(2, PL.RegexMatcher.create_attribute("rack", ".*"), rx),
        PL.RoundRobinByHostnameRule(3, rx),
        PL.RoundRobinByZoneRule(None, rx),
        PL.RoundRobinByRegionRule(2, rx),
        PL.RoundRobinByAttributeRule("rack", 4, rx),
        PL.TaskTypeRule.avoid("world"),
        PL.TaskTypeRule.colocate_with("hello"),
        PL.IsLocalRegionRule(),
        PL.AgentRule.require("a1"),
        PL.NotRule(PL.HostnameRule(PL.ExactMatcher.create("h2"))),
        PL.AndRule([PL.MaxPerHostnameRule(1, rx), PL.OrRule([PL.ZoneRule(PL.ExactMatcher.create("z1")),
                                                             PL.ZoneRule(PL.ExactMatcher.create("z2"))])]),
    ]


@pytest.mark.parametrize("rule", _all_rules(), ids=lambda r: type(r).__name__)
def test_rule_json_round_trip(rule):
    d = rule.to_dict()
    assert "@type" in d
    again = PL.placement_rule_from_dict(d)
    assert again == rule
    assert repr(again) == repr(rule)
    assert again.to_dict() == d


# ---------------------------------------------------------------------------------------
# field rules


def test_hostname_rule_require_and_avoid():
    req = PL.HostnameRuleFactory.require(PL.ExactMatcher.create("host1"))
    avoid = PL.HostnameRuleFactory.avoid(PL.ExactMatcher.create("host1"))
    assert passes(req, offer("host1")) and not passes(req, offer("host2"))
    assert not passes(avoid, offer("host1")) and passes(avoid, offer("host2"))
    rx = PL.HostnameRule(PL.RegexMatcher.create("host[12]"))
    assert passes(rx, offer("host2")) and not passes(rx, offer("host3"))
    # regex must match the whole string, as in Java's String.matches
    assert not passes(rx, offer("xhost1"))


def test_attribute_rule_matches_text_and_scalar_attributes():
    o = offer(attrs=[text_attribute("rack", "r1"), scalar_attribute("tier", 2.0)])
    assert passes(PL.AttributeRule(PL.ExactMatcher.create_attribute("rack", "r1")), o)
    assert not passes(PL.AttributeRule(PL.ExactMatcher.create_attribute("rack", "r2")), o)
    # scalar attributes are rendered with three decimals, as in AttributeStringUtils
    assert passes(PL.AttributeRule(PL.ExactMatcher.create("tier:2.000")), o)
    assert passes(PL.AttributeRule(PL.RegexMatcher.create("tier:2\\..*")), o)
    assert not passes(PL.AttributeRule(PL.ExactMatcher.create("rack")), offer())


def test_zone_and_region_rules_require_fault_domain():
    zr = PL.ZoneRule(PL.ExactMatcher.create("z1"))
    rr = PL.RegionRule(PL.ExactMatcher.create("r1"))
    assert not passes(zr, offer()) and not passes(rr, offer())
    o = offer(zone="z1", region="r1")
    assert passes(zr, o) and passes(rr, o)
    o2 = offer(zone="z2", region="r2")
    assert not passes(zr, o2) and not passes(rr, o2)


def test_agent_rule():
    o = offer("h", agent="a1")
    assert passes(PL.AgentRule.require("a1"), o)
    assert not passes(PL.AgentRule.require("a2"), o)
    assert not passes(PL.AgentRule.avoid("a1"), o)
    assert passes(PL.AgentRule.avoid("a2"), o)
    assert passes(PL.AgentRule.require("a2", "a1"), o)


def test_combinators():
    t, f = PL.PassthroughRule(), PL.NotRule(PL.PassthroughRule())
    o = offer()
    assert passes(t, o) and not passes(f, o)
    assert passes(PL.AndRule([t, t]), o) and not passes(PL.AndRule([t, f]), o)
    assert passes(PL.OrRule([f, t]), o) and not passes(PL.OrRule([f, f]), o)
    assert passes(PL.NotRule(PL.AndRule([t, f])), o)
    out = PL.AndRule([t, f]).filter(o, pod(), [])
    assert len(out.children) == 2 and [c.is_passing() for c in out.children] == [True, False]


def test_is_local_region_rule():
    rule = PL.IsLocalRegionRule()
    saved = PL.IsLocalRegionRule.local_domain
    try:
        PL.IsLocalRegionRule.set_local_domain(None)
        assert passes(rule, offer(region="remote", zone="z"))   # master reported no domain
        local = P.DomainInfo()
        local.fault_domain.region.name = "home"
        local.fault_domain.zone.name = "z1"
        PL.IsLocalRegionRule.set_local_domain(local)
        assert passes(rule, offer())                             # offer without region is local
        assert passes(rule, offer(region="home", zone="z2"))
        assert not passes(rule, offer(region="remote", zone="z1"))
    finally:
        PL.IsLocalRegionRule.set_local_domain(saved)


# ---------------------------------------------------------------------------------------
# MAX_PER


def test_max_per_hostname_counts_matching_tasks_only():
    rule = PL.MaxPerHostnameRule(2, PL.RegexMatcher.create("hello-.*"))
    tasks = [task("world-0-server", "host1"), task("world-1-server", "host1"), task("world-2-server", "host1")]
    assert passes(rule, offer("host1"), tasks)            # non-matching tasks ignored
    tasks.append(task("hello-0-server", "host1", "hello", 0))
    assert passes(rule, offer("host1"), tasks)
    tasks.append(task("hello-1-server", "host1", "hello", 1))
    assert not passes(rule, offer("host1"), tasks)        # two matching already there
    assert passes(rule, offer("host2"), tasks)
    # relaunching hello-1 itself: its own stale TaskInfo does not count against it
    assert passes(rule, offer("host1"), tasks, pod("hello", 1))


def test_unique_hostname_from_constraint_string():
    rule = PL.parse_marathon_constraints(POD, "hostname:UNIQUE")
    tasks = [task("hello-0-server", "host1", "hello", 0)]
    assert not passes(rule, offer("host1"), tasks)
    assert passes(rule, offer("host2"), tasks)
    assert passes(rule, offer("host1"), tasks, pod("hello", 0))


def test_max_per_attribute():
    rule = PL.parse_marathon_constraints(POD, "rack:MAX_PER:1")
    r1, r2 = [text_attribute("rack", "r1")], [text_attribute("rack", "r2")]
    tasks = [task("hello-0-server", "h1", "hello", 0, attrs=r1)]
    assert not passes(rule, offer("h9", attrs=r1), tasks)
    assert passes(rule, offer("h9", attrs=r2), tasks)
    # an agent without the attribute fails the AttributeRule half of the AND
    assert not passes(rule, offer("h9"), tasks)


def test_max_per_zone_and_region():
    zr = PL.MaxPerZoneRule(1, PL.RegexMatcher.create("hello-.*"))
    rr = PL.MaxPerRegionRule(2, PL.RegexMatcher.create("hello-.*"))
    tasks = [task("hello-0-server", "h1", "hello", 0, zone="z1", region="r1")]
    assert not passes(zr, offer("h2", zone="z1", region="r1"), tasks)
    assert passes(zr, offer("h2", zone="z2", region="r1"), tasks)
    assert not passes(zr, offer("h2"), tasks)                    # no zone at all
    assert passes(rr, offer("h2", zone="z1", region="r1"), tasks)
    tasks.append(task("hello-1-server", "h2", "hello", 1, zone="z2", region="r1"))
    assert not passes(rr, offer("h3", zone="z3", region="r1"), tasks)
    assert passes(rr, offer("h3", zone="z3", region="r2"), tasks)


def test_max_per_rejects_nonpositive_max():
    with pytest.raises(ValueError):
        PL.MaxPerHostnameRule(0)


# ---------------------------------------------------------------------------------------
# GROUP_BY (round robin) — the reference rollout sequences


def _rr_tasks():
    # pre-existing tasks that the task filter ([0-9]) ignores
    return [task(f"ignored{i}", h, "x", 100 + i) for i, h in
            enumerate(["host1", "host2", "host3", "host1", "host2"], 1)]


def _t(n, host):
    return task(n, host, "pod", int(n))


def test_round_robin_by_hostname_with_agent_count():
    rule = PL.RoundRobinByHostnameRule(3, PL.RegexMatcher.create("[0-9]"))
    tasks = _rr_tasks()
    ok = lambda h, pi=None: passes(rule, offer(h), tasks, pi)  # noqa: E731
    assert ok("host1")
    tasks.append(_t("1", "host1"))
    assert not ok("host1") and ok("host2") and ok("host3")
    tasks.append(_t("2", "host3"))
    assert ok("host1", pod("pod", 1)) and ok("host3", pod("pod", 2))  # relaunch in place
    assert not ok("host1") and ok("host2") and not ok("host3")
    tasks.append(_t("3", "host2"))
    assert ok("host1") and ok("host2") and ok("host3")
    tasks.append(_t("4", "host2"))
    assert ok("host1") and not ok("host2") and ok("host3")
    tasks.append(_t("5", "host3"))
    assert ok("host4")                       # an unexpected fourth host is still usable
    tasks.append(_t("6", "host4"))
    assert ok("host4")
    tasks.append(_t("7", "host4"))
    assert not ok("host2") and not ok("host3") and not ok("host4") and ok("host1")
    tasks.append(_t("8", "host1"))
    assert all(ok(h) for h in ("host1", "host2", "host3", "host4"))


def test_round_robin_by_hostname_without_agent_count():
    rule = PL.RoundRobinByHostnameRule(None, PL.RegexMatcher.create("[0-9]"))
    tasks = _rr_tasks()
    ok = lambda h: passes(rule, offer(h), tasks)  # noqa: E731
    assert ok("host1")
    tasks.append(_t("1", "host1"))
    assert ok("host1") and ok("host2") and ok("host3")   # other hosts unknown: anything goes
    tasks.append(_t("2", "host3"))
    assert ok("host1") and ok("host2") and ok("host3")
    tasks.append(_t("3", "host2"))
    tasks.append(_t("4", "host2"))
    assert ok("host1") and not ok("host2") and ok("host3")


def test_round_robin_by_zone_and_attribute():
    rz = PL.RoundRobinByZoneRule(2, PL.RegexMatcher.create("hello-.*"))
    tasks = [task("hello-0-server", "h1", "hello", 0, zone="z1", region="r")]
    assert not passes(rz, offer("h2", zone="z1", region="r"), tasks)
    assert passes(rz, offer("h2", zone="z2", region="r"), tasks)
    assert not passes(rz, offer("h2"), tasks)    # offer lacks the key

    ra = PL.RoundRobinByAttributeRule("rack", 2, PL.RegexMatcher.create("hello-.*"))
    a1, a2 = [text_attribute("rack", "a")], [text_attribute("rack", "b")]
    tasks = [task("hello-0-server", "h1", "hello", 0, attrs=a1)]
    assert not passes(ra, offer("h2", attrs=a1), tasks)
    assert passes(ra, offer("h2", attrs=a2), tasks)
    tasks.append(task("hello-1-server", "h2", "hello", 1, attrs=a2))
    assert passes(ra, offer("h3", attrs=a1), tasks) and passes(ra, offer("h3", attrs=a2), tasks)
    assert not passes(ra, offer("h3"), tasks)


# ---------------------------------------------------------------------------------------
# task-type affinity


def test_task_type_avoid():
    rule = PL.TaskTypeRule.avoid("world")
    assert passes(rule, offer("h1"), [])
    tasks = [task("world-0-server", "h1", "world", 0)]
    assert not passes(rule, offer("h1"), tasks)
    assert passes(rule, offer("h2"), tasks)
    # the task being relaunched does not avoid itself
    assert passes(rule, offer("h1"), tasks, pod("world", 0))


def test_task_type_colocate():
    rule = PL.TaskTypeRule.colocate_with("hello")
    assert passes(rule, offer("h1"), [])                # nothing to colocate with yet
    tasks = [task("hello-0-server", "h1", "hello", 0)]
    assert passes(rule, offer("h1"), tasks)
    assert not passes(rule, offer("h2"), tasks)


def test_agent_placement_rule_helper():
    assert PL.get_agent_placement_rule([], []) is None
    r = PL.get_agent_placement_rule(["a1"], [])
    assert not passes(r, offer("h", agent="a1")) and passes(r, offer("h", agent="a2"))
    r = PL.get_agent_placement_rule([], ["a1"])
    assert passes(r, offer("h", agent="a1")) and not passes(r, offer("h", agent="a2"))


def test_placement_field_references():
    assert PL.AndRule([PL.ZoneRule(PL.AnyMatcher.create()), PL.MaxPerHostnameRule(1)]).placement_fields() == [
        PL.PlacementField.ZONE, PL.PlacementField.HOSTNAME]
    spec = SimpleNamespace(placement_rule=PL.RoundRobinByRegionRule(2))
    assert PL.references_region(spec) and not PL.references_zone(spec)
    assert PL.references_zone(SimpleNamespace(placement_rule=PL.MaxPerZoneRule(1)))
    assert not PL.references_zone(SimpleNamespace(placement_rule=None))
