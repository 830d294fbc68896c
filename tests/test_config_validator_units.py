"""Config validator cases from the reference's per-validator JUnit classes that ``test_config_validators``
does not already pin: user changes across pod sets, pod shrink/rename/decommission, pre-reserved
role changes, network-regime switches, capability-gated features, domain rules on old clusters and
invalid placement inside combinators.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/config/validate/{UserCannotChangeTest,
PodSpecsCannotShrinkTest,PreReservationCannotChangeTest,PodSpecsCannotChangeNetworkRegimeTest,
PodSpecsCannotUseUnsupportedFeaturesTest,DomainCapabilityValidatorTest,PlacementRuleIsValidTest}.java.
"""
import dataclasses

import pytest

from dcos_commons_amd.config import validate as V
from dcos_commons_amd.offer.evaluate import placement as PL
from test_config_validators import _task, caps, spec  # noqa: F401  (shared builders / fixture)


def _with_users(s, service_user, pod_users):
    pods = tuple(dataclasses.replace(p, user=u) for p, u in zip(s.pods, pod_users))
    return dataclasses.replace(s, user=service_user, pods=pods)


def _pods(*types):
    return spec({t: (1, "", _task()) for t in types})


# ---------------------------------------------------------------------------------------
# UserCannotChange


@pytest.mark.parametrize("old_user,new_user,errors", [
    ("user", "user", 0), ("user", "other", 1), (None, "user", 0), (None, None, 0),
])
def test_service_user(old_user, new_user, errors):
    old = _with_users(_pods("a"), old_user, [old_user])
    new = _with_users(_pods("a"), new_user, [old_user])
    assert len(V.UserCannotChange().validate(old, new)) == errors


@pytest.mark.parametrize("old_pod_users,new_pod_users,errors", [
    (["u"], ["u"], 0),
    (["u"], ["v"], 1),
    (["u"], [None], 1),                              # old pod set a user, new one does not
    ([None], ["u"], 1),                              # and the reverse
    ([None], [None], 0),
    (["u", "v"], ["v", "u"], 2),                     # every pod changes
    (["u", "u"], ["u", "v"], 1),                     # one user -> several
    (["u", "v"], ["u", "u"], 1),                     # several -> one
    ([None, None], ["u", None], 1),
    ([None, None], ["u", "v"], 2),
])
def test_pod_users(old_pod_users, new_pod_users, errors):
    old = _with_users(_pods("a", "b"), None, old_pod_users + [None] * (2 - len(old_pod_users)))
    new = _with_users(_pods("a", "b"), None, new_pod_users + [None] * (2 - len(new_pod_users)))
    assert len(V.UserCannotChange().validate(old, new)) == errors


def test_new_pod_types_may_set_any_user():
    old = _with_users(_pods("a"), "u", ["u"])
    new = _with_users(_pods("a", "b", "c"), "u", ["u", "x", "y"])
    assert V.UserCannotChange().validate(old, new) == []


def test_user_errors_are_fatal_and_name_the_users():
    old = _with_users(_pods("a"), "user", ["user"])
    new = _with_users(_pods("a"), "other", ["other"])
    errs = V.UserCannotChange().validate(old, new)
    assert len(errs) == 2 and all(e.fatal for e in errs)
    assert "from 'user' to 'other'" in errs[0].message


# ---------------------------------------------------------------------------------------
# PodSpecsCannotShrink


def _sized(*pods):
    """(type, count, allow_decommission) tuples."""
    return spec({t: (n, "allow-decommission: true\n" if allow else "", _task()) for t, n, allow in pods})


@pytest.mark.parametrize("old,new,errors", [
    ([("a", 2, False)], [("a", 2, False)], 0),                       # matching size
    ([("a", 2, False)], [("a", 2, False), ("b", 1, False)], 0),      # pod added
    ([("a", 2, False), ("b", 1, False)], [("a", 2, False)], 1),      # pod removed
    ([("a", 2, False), ("b", 1, True)], [("a", 2, False)], 0),       # decommissionable pod removed
    ([("a", 2, True)], [("c", 2, False)], 0),                        # decommissionable pod renamed
    ([("a", 2, False)], [("c", 2, False)], 1),                       # pod renamed
    ([("a", 2, False)], [("a", 1, False)], 1),                       # count reduced
    ([("a", 2, True)], [("a", 1, False)], 1),                        # only the source allowed it
    ([("a", 2, False)], [("a", 1, True)], 0),                        # the destination allows it
    ([("a", 2, True)], [("a", 1, True)], 0),
    ([("a", 2, False)], [("a", 3, False)], 0),                       # count increased
])
def test_pods_cannot_shrink(old, new, errors):
    assert len(V.PodSpecsCannotShrink().validate(_sized(*old), _sized(*new))) == errors


def test_duplicate_pod_types_and_first_deploy():
    new = _sized(("a", 1, False))
    dup = dataclasses.replace(new, pods=new.pods + new.pods)
    errs = V.PodSpecsCannotShrink().validate(new, dup)
    assert len(errs) == 1 and errs[0].message == "Duplicate pod types detected."
    assert V.PodSpecsCannotShrink().validate(None, dup) == []


# ---------------------------------------------------------------------------------------
# PreReservationCannotChange


def _reserved(*pods):
    """(type, pre-reserved role or None) tuples."""
    return spec({t: (1, f"pre-reserved-role: {r}\n" if r else "", _task()) for t, r in pods})


@pytest.mark.parametrize("old,new,errors", [
    (None, [("a", "slave_public")], 0),                                      # first deployment
    ([("a", "r1"), ("b", "r2")], [("a", "r1"), ("b", "r2")], 0),
    ([("a", "r1"), ("b", "r2")], [("b", "r2"), ("a", "r1")], 0),             # order does not matter
    ([("a", "r1")], [("c", "r3")], 0),                                       # replaced pod type
    ([("a", "r1"), ("b", "r2")], [("a", "changed"), ("b", "r2")], 1),
    ([("a", "r1"), ("b", "r2")], [("a", "r1"), ("b", "changed")], 1),
    ([("a", "r1"), ("b", "r2")], [("b", "r2")], 0),                          # pod removed
    ([("a", "r1"), ("b", "r2")], [("a", "r1")], 0),
    ([("a", "r1")], [("a", None)], 1),                                       # role removed
    ([("a", None)], [("a", "r1")], 1),                                       # role added
    ([("a", None)], [("a", None)], 0),
])
def test_pre_reservation_cannot_change(old, new, errors):
    old_spec = _reserved(*old) if old is not None else None
    assert len(V.PreReservationCannotChange().validate(old_spec, _reserved(*new))) == errors


# ---------------------------------------------------------------------------------------
# PodSpecsCannotChangeNetworkRegime


def _on(network):
    extra = f"networks:\n  {network}: {{}}\n" if network else ""
    return spec({"a": (1, extra, _task())})


@pytest.mark.parametrize("old,new,errors", [
    ("dcos", "dcos", 0), (None, None, 0), ("mesos-bridge", "mesos-bridge", 0),
    ("dcos", None, 1),                  # overlay -> host: gains a host-port requirement
    ("dcos", "mesos-bridge", 1),
    ("mesos-bridge", None, 0),          # bridge and host both use host ports
])
def test_network_regime(old, new, errors):
    assert len(V.PodSpecsCannotChangeNetworkRegime().validate(_on(old), _on(new))) == errors


# ---------------------------------------------------------------------------------------
# PodSpecsCannotUseUnsupportedFeatures


RLIMITS = "rlimits:\n  RLIMIT_NOFILE:\n    soft: 128000\n    hard: 128000\n"
SECRET_FILE = "secrets:\n  s:\n    secret: path/to/secret\n    file: secret-file\n"
SECRET_ENV = "secrets:\n  s:\n    secret: path/to/secret\n    env-key: SECRET_ENV\n"
PORT_MAP = "networks:\n  mesos-bridge:\n    host-ports: [4040]\n    container-ports: [8080]\n"


@pytest.mark.parametrize("extra,task_extra,override,errors", [
    ("", "", {}, 0),
    (RLIMITS, "", {}, 0),
    (RLIMITS, "", {"supports_rlimits": False}, 1),
    ("", "gpus: 1\n", {"supports_gpu_resource": False}, 1),
    ("", "gpus: 1\n", {"supports_gpu_resource": True}, 0),
    (PORT_MAP, "", {"supports_cni_networking": False}, 1),
    (SECRET_FILE, "", {"supports_file_based_secrets": False}, 1),
    (SECRET_FILE, "", {}, 0),
    (SECRET_ENV, "", {"supports_env_based_secrets": False}, 1),
    (SECRET_ENV, "", {}, 0),
])
def test_unsupported_features(caps, extra, task_extra, override, errors):  # noqa: F811
    caps(**override)
    s = spec({"a": (1, extra, _task(extra=task_extra))})
    assert len(V.PodSpecsCannotUseUnsupportedFeatures().validate(None, s)) == errors


# ---------------------------------------------------------------------------------------
# DomainCapabilityValidator


RULES = {
    "none": None,
    "attribute": PL.AttributeRule(PL.ExactMatcher.create("foo:bar")),
    "region": PL.RegionRule(PL.ExactMatcher.create("region")),
    "zone": PL.ZoneRule(PL.ExactMatcher.create("zone")),
    "both": PL.AndRule([PL.RegionRule(PL.ExactMatcher.create("r")), PL.ZoneRule(PL.ExactMatcher.create("z"))]),
}


@pytest.mark.parametrize("rule,old_cluster_errors", [
    ("none", 0), ("attribute", 0), ("region", 1), ("zone", 1), ("both", 2),
])
@pytest.mark.parametrize("domains", [False, True])
def test_domain_capability(caps, rule, old_cluster_errors, domains):  # noqa: F811
    caps(supports_domains=domains)
    s = spec()
    s = dataclasses.replace(s, pods=(dataclasses.replace(s.pods[0], placement_rule=RULES[rule]),))
    errs = V.DomainCapabilityValidator().validate(None, s)
    assert len(errs) == (0 if domains else old_cluster_errors)
    for e in errs:
        assert e.message.startswith("The PlacementRule for PodSpec 'hello' may not reference ")


# ---------------------------------------------------------------------------------------
# PlacementRuleIsValid


INVALID = PL.InvalidPlacementRule("bad", "parse error")
VALID = PL.HostnameRule(PL.ExactMatcher.create("h"))


@pytest.mark.parametrize("rule,errors", [
    (None, 0),
    (PL.AndRule([VALID, VALID]), 0), (PL.AndRule([VALID, INVALID]), 1),
    (PL.OrRule([VALID, VALID]), 0), (PL.OrRule([INVALID, VALID]), 1),
    (INVALID, 1),
])
def test_placement_rule_is_valid(rule, errors):
    s = spec()
    s = dataclasses.replace(s, pods=(dataclasses.replace(s.pods[0], placement_rule=rule),))
    assert len(V.PlacementRuleIsValid().validate(None, s)) == errors
