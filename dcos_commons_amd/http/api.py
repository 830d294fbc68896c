"""Minimal routing core for the scheduler's REST API.

The reference serves JAX-RS resources on Jetty (sdk/.../framework/ApiServer.java:40-120,
http/ResponseUtils.java). Here every resource object exposes ``routes()`` -> list of
``Route(method, template, handler)``; handlers take a ``Request`` and return a ``Response``.
The same dispatch table is used by the threaded HTTP server and, socket-free, by tests and the
simulation harness (``Router.dispatch``).
"""
from __future__ import annotations

import functools
import json
import re
import urllib.parse
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple, Union

JSON = "application/json"
TEXT = "text/plain"
HTML = "text/html"


@dataclass
class Request:
    method: str
    path: str
    query: Dict[str, str] = field(default_factory=dict)
    body: bytes = b""
    headers: Dict[str, str] = field(default_factory=dict)
    params: Dict[str, str] = field(default_factory=dict)

    def q(self, name: str, default: Optional[str] = None) -> Optional[str]:
        return self.query.get(name, default)

    def q_bool(self, name: str) -> bool:
        return (self.query.get(name) or "").lower() == "true"

    def text(self) -> str:
        return self.body.decode("utf-8") if self.body else ""

    def json(self):
        return json.loads(self.text()) if self.body else None


@dataclass
class Response:
    status: int = 200
    body: Union[bytes, str, dict, list, None] = None
    content_type: str = JSON

    def payload(self) -> bytes:
        if self.body is None:
            return b""
        if isinstance(self.body, bytes):
            return self.body
        if isinstance(self.body, str):
            return self.body.encode("utf-8")
        return to_json_text(self.body).encode("utf-8")

    def json(self):
        if isinstance(self.body, (dict, list)):
            return self.body
        return json.loads(self.payload() or b"null")


def to_json_text(value, indent: int = 2, _cur: int = 0) -> str:
    """The layout of org.json's ``toString(2)`` that the reference's ResponseUtils writes: a
    one-entry object or one-element array stays on one line, longer ones put each entry on its
    own indented line (ResponseUtils.java jsonOkResponse)."""
    if isinstance(value, dict):
        if not value:
            return "{}"
        if len(value) == 1:
            (k, v), = value.items()
            return "{" + json.dumps(str(k)) + ": " + to_json_text(v, indent, _cur) + "}"
        pad = _cur + indent
        return "{\n" + ",\n".join(" " * pad + json.dumps(str(k)) + ": " + to_json_text(v, indent, pad)
                                  for k, v in value.items()) + "\n" + " " * _cur + "}"
    if isinstance(value, (list, tuple)):
        if not value:
            return "[]"
        if len(value) == 1:
            return "[" + to_json_text(value[0], indent, _cur) + "]"
        pad = _cur + indent
        return "[\n" + ",\n".join(" " * pad + to_json_text(v, indent, pad) for v in value) + "\n" + " " * _cur + "]"
    return json.dumps(value)


def read_data(stream, declared_size: Optional[int], size_limit: int) -> bytes:
    """RequestUtils.readData: ``size_limit <= 0`` means unlimited. A declared size over the limit
    fails before the stream is touched; the stream itself is read to at most one byte past the
    limit, whatever size was declared."""
    if stream is None:
        raise ValueError("Missing payload")
    if size_limit <= 0:
        return stream.read()
    if declared_size is not None and declared_size > size_limit:
        raise ValueError(f"Stream exceeds {size_limit} byte size limit")
    data = stream.read(size_limit + 1)
    if len(data) > size_limit:
        raise ValueError(f"Stream exceeds {size_limit} byte size limit")
    return data


def json_ok(body, status: int = 200) -> Response:
    return Response(status, body, JSON)


def plain(text: str, status: int = 200) -> Response:
    return Response(status, text, TEXT)


def html(text: str, status: int = 200) -> Response:
    return Response(status, text, HTML)


def not_found(item: str) -> Response:
    return plain(f"{item} not found", 404)


def status_only(status: int) -> Response:
    return Response(status, None, TEXT)


def already_reported() -> Response:
    return plain("Command has already been reported or completed", 208)


def command_result(cmd: str) -> dict:
    return {"message": f"Received cmd: {cmd}"}


@dataclass
class Route:
    method: str
    template: str
    handler: Callable[[Request], Response]
    regex: "re.Pattern" = None

    def __post_init__(self):
        self.regex = _route_regex(self.template)


@functools.lru_cache(maxsize=1024)
def _route_regex(template: str) -> "re.Pattern":
    """``/v1/plans/{plan}`` -> compiled matcher (cached: every scheduler start builds the same
    few hundred routes)."""
    pattern = re.sub(r"\{(\w+):path\}", r"(?P<\1>.+)", template.rstrip("/") or "/")
    pattern = re.sub(r"\{(\w+)\}", r"(?P<\1>[^/]+)", pattern)
    return re.compile("^" + pattern + "/?$")


class Router:
    def __init__(self, resources=()):
        self.routes: List[Route] = []
        for r in resources:
            self.add(r)

    def add(self, resource) -> None:
        self.routes.extend(resource.routes())

    def match(self, method: str, path: str) -> Tuple[Optional[Route], Dict[str, str], bool]:
        path_matched = False
        for r in self.routes:
            m = r.regex.match(path)
            if m is None:
                continue
            path_matched = True
            if r.method == method:
                return r, {k: urllib.parse.unquote(v) for k, v in m.groupdict().items()}, True
        return None, {}, path_matched

    def dispatch(self, method: str, path_and_query: str, body: bytes = b"",
                 headers: Optional[Dict[str, str]] = None) -> Response:
        parsed = urllib.parse.urlsplit(path_and_query)
        query = {k: v[-1] for k, v in urllib.parse.parse_qs(parsed.query, keep_blank_values=True).items()}
        route, params, path_matched = self.match(method.upper(), parsed.path)
        if route is None:
            return status_only(405 if path_matched else 404)
        req = Request(method.upper(), parsed.path, query, body or b"", dict(headers or {}), params)
        try:
            return route.handler(req)
        except Exception as e:  # noqa: BLE001
            import logging

            logging.getLogger(__name__).exception("Request %s %s failed", method, path_and_query)
            return plain(f"Internal error: {e}", 500)

    def get(self, path: str) -> Response:
        return self.dispatch("GET", path)

    def post(self, path: str, body=b"") -> Response:
        if isinstance(body, (dict, list)):
            body = json.dumps(body).encode()
        elif isinstance(body, str):
            body = body.encode()
        return self.dispatch("POST", path, body)

    def put(self, path: str, body=b"", headers=None) -> Response:
        if isinstance(body, str):
            body = body.encode()
        return self.dispatch("PUT", path, body, headers)
