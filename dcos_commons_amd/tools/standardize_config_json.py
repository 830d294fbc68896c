"""Put a package's ``config.json`` options into the standard order.

Reference: tools/standardize_config_json.py. ``properties.service.properties`` is ordered
``name, user, service_account, service_account_secret, virtual_network_enabled,
virtual_network_name, virtual_network_plugin_labels, mesos_api_version, log_level``, then every
other key alphabetically, then ``security``; inside each option schema ``description, type,
enum, default`` come first and ``properties`` last. Further sections are ordered by the
``standardize_config_json.sections`` head/tail lists of an optional ``sdk-tools.json``.

Usage: ``python -m dcos_commons_amd.tools.standardize_config_json --service-config-json
config.json [--sdk-tools-config sdk-tools.json] [--check]`` (``--check`` only reports whether
the file is already standard: exit 1 if not).
"""
from __future__ import annotations

import argparse
import collections
import difflib
import json
import os
import sys
from typing import Callable, Optional, Sequence

SERVICE_HEAD = ("name", "user", "service_account", "service_account_secret", "virtual_network_enabled",
                "virtual_network_name", "virtual_network_plugin_labels", "mesos_api_version", "log_level")
SERVICE_TAIL = ("security",)
PROPERTY_HEAD = ("description", "type", "enum", "default")
PROPERTY_TAIL = ("properties",)


def reorder(original, head: Sequence[str] = (), tail: Sequence[str] = (),
            mapper: Callable = lambda x: x):
    if not isinstance(original, dict):
        return original
    out = collections.OrderedDict()
    for k in head:
        if k in original:
            out[k] = mapper(original[k])
    for k in sorted(k for k in original if k not in head and k not in tail):
        out[k] = mapper(original[k])
    for k in tail:
        if k in original:
            out[k] = mapper(original[k])
    return out


def reorder_property(schema):
    return reorder(schema, PROPERTY_HEAD, PROPERTY_TAIL)


def standardize(contents: dict, tools_config: Optional[dict] = None) -> dict:
    out = json.loads(json.dumps(contents), object_pairs_hook=collections.OrderedDict)
    props = out.get("properties", {})
    if "service" in props and "properties" in props["service"]:
        props["service"]["properties"] = reorder(props["service"]["properties"], SERVICE_HEAD, SERVICE_TAIL,
                                                 reorder_property)
    for section, ht in (tools_config or {}).get("sections", {}).items():
        if section in props and "properties" in props[section]:
            props[section]["properties"] = reorder(props[section]["properties"], ht.get("head") or (),
                                                   ht.get("tail") or (), reorder_property)
    return out


def render(contents: dict) -> str:
    return json.dumps(contents, indent=2) + "\n"


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="Standardizes the ordering of sections in SDK config.json files.")
    ap.add_argument("--service-config-json", required=True)
    ap.add_argument("--sdk-tools-config", default=None)
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args(argv)
    if not os.path.isfile(args.service_config_json):
        print(f"'{args.service_config_json}' is not a file, was expecting an SDK service configuration file")
        return 1
    tools_cfg = {}
    if args.sdk_tools_config:
        if not os.path.isfile(args.sdk_tools_config):
            print(f"'{args.sdk_tools_config}' is not a file, was expecting an SDK Tools configuration file")
            return 1
        with open(args.sdk_tools_config, "r", encoding="utf-8") as f:
            tools_cfg = json.load(f).get("standardize_config_json", {})
    with open(args.service_config_json, "r", encoding="utf-8") as f:
        original_text = f.read()
    original = json.loads(original_text, object_pairs_hook=collections.OrderedDict)
    new_text = render(standardize(original, tools_cfg))
    diff = list(difflib.unified_diff(render(original).split("\n"), new_text.split("\n"), lineterm=""))
    print("\n".join(diff) if diff else "No changes")
    if args.check:
        return 1 if diff else 0
    with open(args.service_config_json, "w", encoding="utf-8") as f:
        f.write(new_text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
