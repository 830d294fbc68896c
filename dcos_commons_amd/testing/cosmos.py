"""Universe package rendering: package options -> Marathon app -> scheduler environment.

Reference: sdk/testing/src/main/java/com/mesosphere/sdk/testing/CosmosRenderer.java. A framework's
``universe/`` directory holds ``config.json`` (a JSON schema whose ``default`` values are the
package options), ``resource.json`` (artifact URLs) and ``marathon.json.mustache`` (the scheduler's
Marathon app). Rendering flattens the option defaults to dotted keys (``service.user``), overlays
``resource.*`` entries, the caller's options and build/tooling parameters, renders the Marathon
template strictly and returns its ``env`` plus ``PORT<i>``/``PORT_<NAME>`` for declared ports
(Marathon injects those; port 0 simulates an ephemeral port).

Also used outside tests: ``render_scheduler_environment`` is what ``python -m
dcos_commons_amd.models.<framework>`` uses to turn ``--option k=v`` flags into a scheduler env.
"""
from __future__ import annotations

import json
import os
import random
from typing import Dict, List, Mapping, Optional

from dcos_commons_amd.specification.yaml import template_utils as T

RESOURCE_TEMPLATE_PARAMS = {
    "artifact-dir": "https://test-url/artifacts",
    "jre-url": "https://test-url/jre.tgz",
    "scheduler-jre-url": "https://test-url/jre.tgz",
    "libmesos-bundle-url": "https://test-url/libmesos-bundle.tgz",
    "dcos-sdk-version": "99.99.99-SNAPSHOT",
}
MARATHON_TEMPLATE_PARAMS = {
    "package-name": "test-pkg",
    "package-version": "0.0.1-beta",
    "package-build-time-epoch-ms": "0",
    "package-build-time-str": "Today",
}


def _read(path: str) -> str:
    with open(path, "r", encoding="utf-8") as f:
        return f.read()


def _scalar(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (dict, list)):
        return json.dumps(v, separators=(",", ":"))
    return str(v)


def flatten_property_tree(path: str, node: Mapping, out: Dict[str, str]) -> None:
    if "default" in node:
        # quotes are re-escaped because the value is substituted into a JSON string
        out[path] = _scalar(node["default"]).replace('"', '\\"')
    if node.get("type") == "object" and isinstance(node.get("properties"), Mapping):
        for key, child in node["properties"].items():
            flatten_property_tree(f"{path}.{key}" if path else key, child, out)


def flatten_tree(path: str, node: Mapping, out: Dict[str, str]) -> None:
    for key, val in node.items():
        p = f"{path}.{key}" if path else key
        if isinstance(val, Mapping):
            flatten_tree(p, val, out)
        else:
            out[p] = _scalar(val)


def option_defaults(universe_dir: str, build_params: Optional[Mapping[str, str]] = None) -> Dict[str, str]:
    cfg = json.loads(T.render_mustache_throw_if_missing(
        "universe/config.json", _read(os.path.join(universe_dir, "config.json")), dict(build_params or {})))
    out: Dict[str, str] = {}
    flatten_property_tree("", cfg, out)
    return out


def render_marathon_app(universe_dir: str, options: Optional[Mapping[str, str]] = None,
                        build_params: Optional[Mapping[str, str]] = None,
                        package_params: Optional[Mapping[str, str]] = None) -> Dict:
    """``package_params`` override the test package coordinates (``package-name``,
    ``package-version``, ...) that otherwise default to ``MARATHON_TEMPLATE_PARAMS``."""
    build_params = dict(build_params or {})
    params = option_defaults(universe_dir, build_params)
    resource_path = os.path.join(universe_dir, "resource.json")
    if os.path.exists(resource_path):
        rp = dict(build_params)
        rp.update(RESOURCE_TEMPLATE_PARAMS)
        missing: List[T.MissingValue] = []
        rendered = T.render_mustache("universe/resource.json", _read(resource_path), rp, missing)
        missing = [m for m in missing if not m.name.startswith("sha256:")]
        T.validate_missing_values("universe/resource.json", rp, missing)
        flatten_tree("resource", json.loads(rendered), params)
    # caller options land inside JSON strings too: escape quotes like the defaults (arrays and
    # objects are rendered as raw JSON values, e.g. the scheduler's ``constraints``)
    params.update({k: _scalar(v) if isinstance(v, (list, dict)) else _scalar(v).replace('"', '\\"')
                   for k, v in (options or {}).items()})
    params.update(build_params)
    params.update(MARATHON_TEMPLATE_PARAMS)
    params.update(package_params or {})
    text = T.render_mustache_throw_if_missing("universe/marathon.json.mustache",
                                              _read(os.path.join(universe_dir, "marathon.json.mustache")), params)
    return json.loads(text)


def render_scheduler_environment(universe_dir: str, options: Optional[Mapping[str, str]] = None,
                                 build_params: Optional[Mapping[str, str]] = None,
                                 rng: Optional[random.Random] = None) -> Dict[str, str]:
    app = render_marathon_app(universe_dir, options, build_params)
    env = {k: _scalar(v) for k, v in (app.get("env") or {}).items() if not isinstance(v, Mapping)}
    rng = rng or random.Random()
    for i, port in enumerate(app.get("portDefinitions") or []):
        val = int(port.get("port", 0)) or rng.randrange(32768, 61000)
        env[f"PORT{i}"] = str(val)
        if port.get("name"):
            env[f"PORT_{port['name'].upper()}"] = str(val)
    return dict(sorted(env.items()))
