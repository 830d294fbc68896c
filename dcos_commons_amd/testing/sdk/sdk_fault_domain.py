"""Fault-domain name checks (reference: testing/sdk_fault_domain.py); the local cluster uses
AWS-style names (``us-west-2`` / ``us-west-2a``) by default."""
from __future__ import annotations

import re

_AWS_REGION = re.compile(r"^[a-z]{2}(-gov)?-[a-z]+-\d$")
_AWS_ZONE = re.compile(r"^[a-z]{2}(-gov)?-[a-z]+-\d[a-z]$")


def is_valid_aws_region(region: str) -> bool:
    return bool(_AWS_REGION.match(region or ""))


def is_valid_aws_zone(region: str, zone: str) -> bool:
    return is_valid_aws_region(region) and bool(_AWS_ZONE.match(zone or "")) and zone.startswith(region)


def is_valid_region(region: str) -> bool:
    return is_valid_aws_region(region)


def is_valid_zone(zone: str) -> bool:
    return bool(_AWS_ZONE.match(zone or ""))
