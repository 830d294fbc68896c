"""Configuration value types and (de)serialization helpers.

Reference: sdk/.../config/{Configuration,ConfigurationFactory,ConfigurationComparator,
StringConfiguration,RecoveryConfiguration,SerializationUtils,YAMLConfigurationLoader}.java.

* ``StringConfiguration`` -- the simplest ``ConfigStore`` payload (bytes are the UTF-8 string);
* ``RecoveryConfiguration`` -- the legacy recovery knobs (``recover-in-place-grace-period-secs``,
  ``min-delay-between-recoveries-secs``, ``enable-replacement``);
* ``to_json_string``/``from_json_string``/``to_yaml_string``/``from_yaml_string`` -- the JSON
  written the way Jackson's pretty printer writes it (``"key" : value``, two-space indent), so
  configs and API payloads diff cleanly against the reference's;
* ``load_config_from_env`` -- reads a YAML file after substituting ``${VAR}`` (and
  ``${VAR:-default}``) from the environment, ``$${VAR}`` escaping; unknown variables stay as
  written (commons-lang StrSubstitutor semantics).
"""
from __future__ import annotations

import dataclasses
import json
import logging
import os
import re
from typing import Any, Callable, Dict, Mapping, Optional, Type, TypeVar

import yaml

LOGGER = logging.getLogger(__name__)
T = TypeVar("T")


class Configuration:
    """A ConfigStore payload: ``get_bytes`` is what is persisted, ``to_json_string`` what is shown."""

    def get_bytes(self) -> bytes:
        raise NotImplementedError

    def to_json_string(self) -> str:
        raise NotImplementedError


class StringConfiguration(Configuration):
    def __init__(self, config: str):
        self.config = config

    def get_bytes(self) -> bytes:
        return self.config.encode("utf-8")

    def to_json_string(self) -> str:
        return '{ "string": "%s" }' % self.config.replace('"', '\\"')

    def __eq__(self, other):
        return isinstance(other, StringConfiguration) and self.config == other.config

    def __hash__(self):
        return hash(self.config)

    def __repr__(self):
        return f"StringConfiguration({self.config!r})"

    class Factory:
        def parse(self, data: bytes) -> "StringConfiguration":
            return StringConfiguration(data.decode("utf-8"))

    class Comparator:
        def equals(self, first: "StringConfiguration", second: "StringConfiguration") -> bool:
            return first == second


@dataclasses.dataclass
class RecoveryConfiguration:
    grace_period_secs: int = 0
    recover_delay_secs: int = 0
    enable_replacement: bool = False

    _KEYS = (("grace_period_secs", "recover-in-place-grace-period-secs"),
             ("recover_delay_secs", "min-delay-between-recoveries-secs"),
             ("enable_replacement", "enable-replacement"))

    def is_replacement_enabled(self) -> bool:
        return self.enable_replacement

    def to_dict(self) -> Dict[str, Any]:
        return {k: getattr(self, a) for a, k in self._KEYS}

    @staticmethod
    def from_dict(d: Mapping[str, Any]) -> "RecoveryConfiguration":
        return RecoveryConfiguration(int(d.get("recover-in-place-grace-period-secs") or 0),
                                     int(d.get("min-delay-between-recoveries-secs") or 0),
                                     bool(d.get("enable-replacement") or False))


def _plain(value: Any) -> Any:
    """Objects with ``to_dict`` (specs, configs) or dataclasses become plain JSON values."""
    if hasattr(value, "to_dict"):
        return _plain(value.to_dict())
    if dataclasses.is_dataclass(value) and not isinstance(value, type):
        return _plain(dataclasses.asdict(value))
    if isinstance(value, Mapping):
        return {str(k): _plain(v) for k, v in value.items()}
    if isinstance(value, (list, tuple, set, frozenset)):
        return [_plain(v) for v in value]
    return value


def to_json_string(value: Any) -> str:
    """Jackson ``writerWithDefaultPrettyPrinter`` layout: ``{\\n  "key" : value\\n}``."""
    return _jackson(_plain(value), 0)


def _jackson(v: Any, depth: int) -> str:
    pad, inner = "  " * depth, "  " * (depth + 1)
    if isinstance(v, dict):
        if not v:
            return "{ }"
        items = [f'{inner}{json.dumps(k)} : {_jackson(x, depth + 1)}' for k, x in v.items()]
        return "{\n" + ",\n".join(items) + "\n" + pad + "}"
    if isinstance(v, list):
        if not v:
            return "[ ]"
        return "[ " + ", ".join(_jackson(x, depth + 1) for x in v) + " ]"
    return json.dumps(v)


def from_json_string(text: str, cls: Optional[Type[T]] = None) -> Any:
    data = json.loads(text)
    return _typed(data, cls)


def to_yaml_string(value: Any) -> str:
    return yaml.safe_dump(_plain(value), default_flow_style=False, sort_keys=False)


def to_yaml_string_or_empty(value: Any) -> str:
    try:
        return to_yaml_string(value)
    except Exception:  # noqa: BLE001 -- SerializationUtils.toYamlStringOrEmpty
        return ""


def from_yaml_string(text: str, cls: Optional[Type[T]] = None) -> Any:
    return _typed(yaml.safe_load(text), cls)


def _typed(data: Any, cls: Optional[Type[T]]) -> Any:
    if cls is None:
        return data
    if hasattr(cls, "from_dict"):
        return cls.from_dict(data)
    if dataclasses.is_dataclass(cls):
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k.replace("-", "_"): v for k, v in data.items() if k.replace("-", "_") in names})
    return cls(data)


_VAR = re.compile(r"\$(\$?)\{([^{}]+)\}")


def substitute_env(text: str, env: Optional[Mapping[str, str]] = None) -> str:
    """``${VAR}`` / ``${VAR:-default}`` from ``env`` (default: the process environment); ``$${VAR}``
    is an escaped literal; variables that resolve to nothing are left as written. Substituted
    values are themselves substituted (StrSubstitutor.setEnableSubstitutionInVariables)."""
    env = os.environ if env is None else env

    def repl(m: "re.Match") -> str:
        if m.group(1):  # escaped
            return "${" + m.group(2) + "}"
        name, _, default = m.group(2).partition(":-")
        value = env.get(name)
        if value is None:
            value = default if ":-" in m.group(2) else None
        if value is None:
            return m.group(0)
        return substitute_env(value, env) if "${" in value else value

    return _VAR.sub(repl, text)


def load_config_from_env(cls: Optional[Type[T]], path: str, env: Optional[Mapping[str, str]] = None) -> Any:
    """YAMLConfigurationLoader.loadConfigFromEnv: env-substituted YAML file -> ``cls``."""
    LOGGER.info("Parsing configuration file from %s", path)
    with open(os.path.abspath(path), "r", encoding="utf-8") as f:
        text = f.read()
    return from_yaml_string(substitute_env(text, env), cls)


ConfigurationFactory = Callable[[bytes], Configuration]
