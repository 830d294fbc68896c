"""Logger naming and FRAMEWORK_LOG_LEVEL (reference: offer/LoggingUtils.java, log4j2.xml)."""
import logging

from dcos_commons_amd.utils import logging_utils as L


def test_namespaced_logger_stays_in_package_hierarchy():
    plain = L.get_logger("dcos_commons_amd.offer.evaluate.offer_evaluator")
    tagged = L.get_logger("dcos_commons_amd.offer.evaluate.offer_evaluator", "svc-a")
    assert plain.name == "dcos_commons_amd.offer.evaluate.offer_evaluator"
    assert tagged.name == "dcos_commons_amd.offer.evaluate.offer_evaluator(svc-a)"
    assert L.get_logger("x", "  ").name == "x"
    logging.getLogger("dcos_commons_amd.offer").setLevel(logging.ERROR)
    try:
        assert tagged.getEffectiveLevel() == logging.ERROR  # package-level config applies
    finally:
        logging.getLogger("dcos_commons_amd.offer").setLevel(logging.NOTSET)


def test_configure_reads_framework_log_level():
    root = logging.getLogger()
    old = root.level
    try:
        assert L.configure({"FRAMEWORK_LOG_LEVEL": "debug"}) == logging.DEBUG
        assert root.level == logging.DEBUG
        assert L.configure({"FRAMEWORK_LOG_LEVEL": "LOUD"}) == logging.INFO
        assert L.configure({}) == logging.INFO
    finally:
        root.setLevel(old)


def test_multi_service_components_tag_their_loggers():
    from dcos_commons_amd.scheduler.plan.plan_scheduler import PlanScheduler

    assert PlanScheduler(None, None, namespace="svc-b").logger.name.endswith("plan_scheduler(svc-b)")
    assert PlanScheduler(None, None).logger.name == "dcos_commons_amd.scheduler.plan.plan_scheduler"
