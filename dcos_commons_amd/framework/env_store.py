"""Typed access to the scheduler environment (reference sdk/.../framework/EnvStore.java)."""
from __future__ import annotations

import os
from typing import Dict, List, Mapping, Optional


class ConfigException(RuntimeError):
    pass


class EnvStore:
    def __init__(self, env: Optional[Mapping[str, str]] = None):
        self._env: Dict[str, str] = dict(os.environ if env is None else env)

    @staticmethod
    def from_env() -> "EnvStore":
        return EnvStore(os.environ)

    @staticmethod
    def from_map(m: Mapping[str, str]) -> "EnvStore":
        return EnvStore(m)

    def as_map(self) -> Dict[str, str]:
        return dict(self._env)

    def is_present(self, key: str) -> bool:
        return key in self._env

    def get_required(self, key: str) -> str:
        v = self._env.get(key)
        if v is None:
            raise ConfigException(f"Missing required environment variable: {key}")
        return v

    def get_optional(self, key: str, default: Optional[str]) -> Optional[str]:
        return self._env.get(key, default)

    def get_optional_non_empty(self, key: str, default: str) -> str:
        v = self._env.get(key)
        return v if v else default

    def _num(self, key: str, conv, default):
        v = self._env.get(key)
        if v is None:
            return default
        try:
            return conv(v)
        except ValueError:
            raise ConfigException(f"Failed to parse env {key}={v!r}")

    def get_required_int(self, key: str) -> int:
        return int(self.get_required(key))

    def get_required_long(self, key: str) -> int:
        return int(self.get_required(key))

    def get_optional_int(self, key: str, default: int) -> int:
        return self._num(key, int, default)

    def get_optional_long(self, key: str, default: int) -> int:
        return self._num(key, int, default)

    def get_optional_double(self, key: str, default: float) -> float:
        return self._num(key, float, default)

    def get_optional_boolean(self, key: str, default: bool) -> bool:
        v = self._env.get(key)
        if v is None:
            return default
        return v.strip().lower() in ("true", "1", "yes")

    def get_optional_string_list(self, key: str, default: List[str]) -> List[str]:
        v = self._env.get(key)
        if not v:
            return list(default)
        return [s.strip() for s in v.split(",") if s.strip()]
