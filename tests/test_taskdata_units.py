"""Task-data units: attribute strings, VIP port labels, environment helpers and the task label
reader/writer.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/offer/taskdata/{AttributeStringUtilsTest,
AuxLabelAccessTest,EnvUtilsTest,TaskLabelReaderWriterTest}.java.
"""
import uuid

import pytest

import testutils as U
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.taskdata import labels as L


def _attr(t, name):
    return P.Attribute(type=t, name=name)


def _ranges(name, *pairs):
    a = _attr(P.Value.RANGES, name)
    for b, e in pairs:
        a.ranges.range.add(begin=b, end=e)
    return a


def _scalar(name, value=None):
    a = _attr(P.Value.SCALAR, name)
    a.scalar.value = 0.0 if value is None else value
    return a


def _set(name, *items):
    a = _attr(P.Value.SET, name)
    a.set.SetInParent()
    a.set.item.extend(items)
    return a


def _text(name, value=None):
    a = _attr(P.Value.TEXT, name)
    a.text.value = value or ""
    return a


@pytest.mark.parametrize("attr,expected", [
    (_ranges("ram", (1, 2)), "ram:[1-2]"),
    # Range bounds are uint64: the reference's negative cases (Java longs) cannot be built here.
    (_ranges("ports", (1, 2), (21000, 24000), (0, 0), (30000, 34000), (321, 123)),
     "ports:[1-2,21000-24000,0-0,30000-34000,321-123]"),
    (_ranges("ram", (0, 0)), "ram:[0-0]"),
    (_ranges("disk", (321, 123)), "disk:[321-123]"),
    (_ranges("", (321, 123)), ":[321-123]"),
    (_ranges("empty"), "empty:[]"),
    (_ranges(""), ":[]"),
])
def test_range_attribute_string(attr, expected):
    assert L.attribute_to_string(attr) == expected


@pytest.mark.parametrize("name,value,expected", [
    ("ram", 0, "ram:0.000"), ("ports", 0.0001, "ports:0.000"), ("ports", 0.0005, "ports:0.001"),
    ("rounddown", -1.99999, "rounddown:-2.000"), ("roundup1", 1.99999, "roundup1:2.000"),
    ("", 1.99999, ":2.000"), ("roundup2", 999999.99999, "roundup2:1000000.000"),
    ("empty", None, "empty:0.000"), ("", None, ":0.000"),
])
def test_scalar_attribute_string(name, value, expected):
    assert L.attribute_to_string(_scalar(name, value)) == expected


@pytest.mark.parametrize("attr,expected", [
    (_set("ram", ""), "ram:{}"), (_set("ports", "a", "b", "c"), "ports:{a,b,c}"),
    (_set("disk", "-1", "-2"), "disk:{-1,-2}"), (_set("", "-1", "-2"), ":{-1,-2}"),
    (_set("empty"), "empty:{}"), (_set(""), ":{}"),
])
def test_set_attribute_string(attr, expected):
    assert L.attribute_to_string(attr) == expected


@pytest.mark.parametrize("attr,expected", [
    (_text("ram", ":::"), "ram::::"), (_text("ram", "abc"), "ram:abc"), (_text("", "123"), ":123"),
    (_text("empty"), "empty:"), (_text(""), ":"),
])
def test_text_attribute_string(attr, expected):
    assert L.attribute_to_string(attr) == expected


def test_mixed_attribute_strings():
    attrs = []
    assert L.attributes_to_string(attrs) == ""
    attrs.append(_text("ram", ""))
    assert L.attributes_to_string(attrs) == "ram:"
    attrs.append(_set("ports", "a", "b", "c"))
    assert L.attributes_to_string(attrs) == "ram:;ports:{a,b,c}"
    attrs.append(_scalar("roundup1", 1.99999))
    assert L.attributes_to_string(attrs) == "ram:;ports:{a,b,c};roundup1:2.000"
    attrs.append(_ranges("disk", (321, 123)))
    assert L.attributes_to_string(attrs) == "ram:;ports:{a,b,c};roundup1:2.000;disk:[321-123]"


def test_split_attribute_string():
    assert L.attribute_string_list("") == []
    assert L.attribute_string_list(
        "cpus:24;gpus:2;mem:24576;disk:409600;ports:[21000-24000,30000-34000];bugs(debug_role):{a,b,c}") == [
        "cpus:24", "gpus:2", "mem:24576", "disk:409600", "ports:[21000-24000,30000-34000]",
        "bugs(debug_role):{a,b,c}"]
    assert L.attribute_string_list("rack:abc;zone:west;os:centos5;level:10;keys:[1000-1500]") == [
        "rack:abc", "zone:west", "os:centos5", "level:10", "keys:[1000-1500]"]


@pytest.mark.parametrize("s,name,value", [
    (":", "", ""), ("foo:", "foo", ""), (":bar", "", "bar"), ("foo:bar", "foo", "bar"),
    ("foo:bar:baz", "foo", "bar:baz"),
])
def test_split_join_single_attribute(s, name, value):
    assert L.attribute_split(s) == (name, value)
    assert L.attribute_join(name, value) == s


def test_split_single_attribute_fails():
    with pytest.raises(ValueError):
        L.attribute_split("foobar")


# ---------------------------------------------------------------------------------------
# VIP labels (AuxLabelAccess)


def _port():
    return P.Port(number=999)


def test_create_vip_label():
    port = _port()
    L.set_vip_labels(port, "vip", 5, [], lambda n: False)
    assert len(port.labels.labels) == 1
    label = port.labels.labels[0]
    assert label.key.startswith("VIP_") and label.value == "vip:5"
    assert L.get_vips_from_labels(port) == [("vip", 5)]


def test_create_vip_label_on_overlay():
    port = _port()
    L.set_vip_labels(port, "vip", 5, ["dcos"], lambda n: False)
    labels = [(l.key, l.value) for l in port.labels.labels]
    assert len(labels) == 2
    assert sum(1 for k, v in labels if k.startswith("VIP_") and v == "vip:5") == 1
    assert (L.VIP_OVERLAY_FLAG_KEY, L.VIP_OVERLAY_FLAG_VALUE) in labels
    assert L.get_vips_from_labels(port) == [("vip", 5)]


def test_vip_on_port_mapped_network_routes_by_host():
    port = _port()
    L.set_vip_labels(port, "vip", 5, ["mesos-bridge"], lambda n: n == "mesos-bridge")
    assert (L.VIP_OVERLAY_FLAG_KEY, L.VIP_BRIDGE_FLAG_VALUE) in [(l.key, l.value) for l in port.labels.labels]


def _with_label(key, value):
    port = _port()
    port.labels.labels.add(key=key, value=value)
    return port


@pytest.mark.parametrize("key,value", [("", ""), ("asdf", "ara"), ("VIP_0000", "ara"), ("VIP_0000", "ara:rar")])
def test_unparseable_vip_labels_are_ignored(key, value):
    assert L.get_vips_from_labels(_with_label(key, value)) == []


def test_parse_vip_label():
    assert L.get_vips_from_labels(_with_label("VIP_0000", "myvip:321")) == [("myvip", 321)]


# ---------------------------------------------------------------------------------------
# EnvUtils


def _reference_secret(path):
    s = P.Secret(type=P.Secret.REFERENCE)
    s.reference.name = path
    return s


def test_with_env_var_keeps_secrets():
    env = P.Environment()
    v = env.variables.add(name="SECRET_KEY", type=P.Environment.Variable.SECRET)
    v.secret.CopyFrom(_reference_secret("SECRET_PATH"))
    out = L.with_env_var(env, "TEST_KEY", "TEST_VALUE")
    assert len(out.variables) == 2
    by_name = {x.name: x for x in out.variables}
    assert by_name["SECRET_KEY"].secret == _reference_secret("SECRET_PATH")
    assert by_name["TEST_KEY"].value == "TEST_VALUE"


def test_with_env_var_overwrites_an_existing_key():
    env = P.Environment()
    env.variables.add(name="TEST_KEY", value="TEST_VALUE")
    out = L.with_env_var(env, "TEST_KEY", "TEST_NEW_VALUE")
    assert len(out.variables) == 1 and out.variables[0].value == "TEST_NEW_VALUE"


@pytest.mark.parametrize("raw,env", [("hello", "HELLO"), ("hello-world.1", "HELLO_WORLD_1"), ("a b", "A_B")])
def test_to_env_name(raw, env):
    assert L.to_env_name(raw) == env


# ---------------------------------------------------------------------------------------
# TaskLabelReader / TaskLabelWriter


def _task():
    t = P.TaskInfo(name="test-task-name")
    t.task_id.value = "test-task-id"
    t.agent_id.value = "test-agent-id"
    return t


def test_missing_target_configuration_fails():
    with pytest.raises(L.TaskException):
        L.TaskLabelReader(_task()).get_target_configuration()


def test_set_target_configuration():
    target = uuid.uuid4()
    t = _task()
    t.labels.CopyFrom(L.TaskLabelWriter(t).set_target_configuration(target).to_proto())
    assert L.TaskLabelReader(t).get_target_configuration() == target


def test_set_get_offer_attributes():
    offer = P.Offer(hostname=U.HOSTNAME)
    offer.id.CopyFrom(U.OFFER_ID)
    offer.framework_id.CopyFrom(U.FRAMEWORK_ID)
    offer.agent_id.CopyFrom(U.AGENT_ID)
    offer.attributes.extend([_ranges("1", (5, 6), (10, 12)), _scalar("2", 123.4567),
                             _set("3", "foo", "bar", "baz"), _ranges("4", (7, 8), (10, 12))])
    assert L.TaskLabelReader(_task()).get_offer_attribute_strings() == []
    t = _task()
    t.labels.CopyFrom(L.TaskLabelWriter(t).set_offer_attributes(offer).to_proto())
    assert L.TaskLabelReader(t).get_offer_attribute_strings() == [
        "1:[5-6,10-12]", "2:123.457", "3:{foo,bar,baz}", "4:[7-8,10-12]"]
    del offer.attributes[:]
    t.labels.CopyFrom(L.TaskLabelWriter(t).set_offer_attributes(offer).to_proto())
    assert L.TaskLabelReader(t).get_offer_attribute_strings() == []


def test_read_write_region_and_zone():
    assert L.TaskLabelReader(_task()).get_region() is None
    assert L.TaskLabelReader(_task()).get_zone() is None
    t = _task()
    fd = U.LOCAL_DOMAIN_INFO.fault_domain
    t.labels.CopyFrom(L.TaskLabelWriter(t).set_region(fd.region.name).set_zone(fd.zone.name).to_proto())
    assert L.TaskLabelReader(t).get_region() == U.LOCAL_REGION
    assert L.TaskLabelReader(t).get_zone() == U.ZONE


def test_missing_task_type_fails():
    with pytest.raises(L.TaskException):
        L.TaskLabelReader(_task()).get_type()


@pytest.mark.parametrize("task_type", ["foo", ""])
def test_set_get_task_type(task_type):
    t = _task()
    t.labels.CopyFrom(L.TaskLabelWriter(t).set_type(task_type).to_proto())
    assert L.TaskLabelReader(t).get_type() == task_type


def test_additional_labels():
    t = _task()
    t.labels.CopyFrom(L.TaskLabelWriter(t).set_additional_labels(
        {"label1": "label1-value", "label2": "label2-value"}).to_proto())
    m = L.labels_to_map(t.labels)
    assert m["label1"] == "label1-value" and m["label2"] == "label2-value"


def test_readiness_check_tagging():
    check = P.HealthCheck(delay_seconds=1.0, consecutive_failures=3)
    t = _task()
    t.labels.CopyFrom(L.TaskLabelWriter(t).set_readiness_check(check).to_proto())
    out = L.TaskLabelWriter(t).get_readiness_check()
    assert out.delay_seconds == 1.0
    assert out.consecutive_failures == 0  # readiness checks never kill the task
    assert L.TaskLabelReader(t).has_readiness_check_label()


def test_readiness_check_env_var():
    check = P.HealthCheck(delay_seconds=1.0)
    check.command.value = "true"
    t = _task()
    L.TaskLabelWriter(t).set_readiness_check(check).apply()
    L.TaskLabelWriter(t).set_readiness_check_envvar("KEY", "value").apply()
    assert L.get_env_var(L.TaskLabelReader(t).get_readiness_check().command.environment, "KEY") == "value"


def test_permanently_failed_and_footprint_flags():
    t = _task()
    assert not L.TaskLabelReader(t).is_permanently_failed()
    L.TaskLabelWriter(t).set_permanently_failed().set_launch_new_footprint(True).apply()
    r = L.TaskLabelReader(t)
    assert r.is_permanently_failed() and r.is_launch_new_footprint()
    L.TaskLabelWriter(t).clear_permanently_failed().set_launch_new_footprint(False).apply()
    r = L.TaskLabelReader(t)
    assert not r.is_permanently_failed() and not r.is_launch_new_footprint()


@pytest.mark.parametrize("labels,check_exit,expected", [
    ({}, None, True),                                               # no check at all
    ({L.READINESS_CHECK_LABEL: "x"}, None, False),                   # check pending
    ({L.READINESS_CHECK_LABEL: "x", "passed": "true"}, None, True),  # legacy passed label
    ({L.READINESS_CHECK_LABEL: "x"}, 0, True),                       # Mesos check status
    ({L.READINESS_CHECK_LABEL: "x"}, 1, False),
])
def test_readiness_check_succeeded(labels, check_exit, expected):
    t = _task()
    L.map_to_labels({k: v for k, v in labels.items() if k != "passed"}, t.labels)
    status = P.TaskStatus(state=P.TASK_RUNNING)
    status.task_id.CopyFrom(t.task_id)
    if "passed" in labels:
        status.labels.labels.add(key=L.READINESS_CHECK_PASSED_LABEL, value=labels["passed"])
    if check_exit is not None:
        status.check_status.command.exit_code = check_exit
    assert L.TaskLabelReader(t).is_readiness_check_succeeded(status) is expected
