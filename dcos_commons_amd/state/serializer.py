"""Property value (de)serializers.

Reference: sdk/.../state/Serializer.java, state/JsonSerializer.java (Jackson object <-> UTF-8 JSON
bytes; a parse failure is an IOException) and http/types/PropertyDeserializer.java +
StringPropertyDeserializer.java (what ``GET /v1/state/properties/{key}`` shows: the stored bytes as
a UTF-8 string, unchanged).
"""
from __future__ import annotations

import json
from typing import Any, Optional, Type


class JsonSerializer:
    """Values <-> compact UTF-8 JSON bytes. ``deserialize`` raises ``ValueError`` on bytes that
    are not JSON or, with ``cls``, that do not decode to that type."""

    def serialize(self, value: Any) -> bytes:
        return json.dumps(value, separators=(",", ":")).encode("utf-8")

    def deserialize(self, data: bytes, cls: Optional[Type] = None) -> Any:
        try:
            text = data.decode("utf-8") if isinstance(data, (bytes, bytearray)) else data
            value = json.loads(text)
        except (UnicodeDecodeError, json.JSONDecodeError) as e:
            raise ValueError(f"Failed to deserialize JSON: {e}") from e
        if cls is not None:
            # bool is an int subclass in Python, JSON booleans are not numbers in Jackson
            if cls is int and isinstance(value, bool) or not isinstance(value, cls):
                raise ValueError(f"JSON value {value!r} is not a {cls.__name__}")
        return value


class PropertyDeserializer:
    """Renders a stored property for the state API (PropertyDeserializer.java)."""

    def to_json_string(self, key: str, value: bytes) -> str:
        raise NotImplementedError

    def __call__(self, key: str, value: bytes) -> str:
        return self.to_json_string(key, value)


class StringPropertyDeserializer(PropertyDeserializer):
    """The stored bytes as a UTF-8 string (StringPropertyDeserializer.java)."""

    def to_json_string(self, key: str, value: bytes) -> str:
        if value is None:
            return ""
        return value.decode("utf-8", errors="replace") if isinstance(value, (bytes, bytearray)) else str(value)
