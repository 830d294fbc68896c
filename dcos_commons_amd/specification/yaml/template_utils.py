"""Strict Mustache renderer for ``svc.yml`` and task config templates.

Reference: sdk/.../specification/yaml/TemplateUtils.java:45-185 (mustache.java with a
``MissingValueBinding`` that records ``NAME@L<line>`` for every unresolved ``{{value}}``).
Semantics implemented here (no mustache library exists in this image):

* ``{{name}}`` HTML-escaped (mustache.java escapes ``& < > " ' ` =``), ``{{{name}}}`` and
  ``{{& name}}`` raw;
* sections ``{{#name}}..{{/name}}`` and inverted ``{{^name}}..{{/name}}``, comments
  ``{{! ..}}``, delimiter changes ``{{=<% %>=}}``; standalone tag lines are removed;
* env values equal (case-insensitively) to ``true``/``false`` are booleans, so
  ``{{#ENABLE_X}}`` works as a flag; empty strings are falsy;
* missing *value* tags are collected (with their 1-based line) and rendered empty; strict mode
  raises :class:`MustacheError` listing them.

The same grammar is implemented in C++ for the in-task ``bootstrap`` helper
(``native/bootstrap/mustache.hpp``).
"""
from __future__ import annotations

import collections.abc
import re
from dataclasses import dataclass
from typing import Any, Dict, List, Mapping, Optional, Tuple


class MustacheError(ValueError):
    pass


@dataclass(frozen=True)
class MissingValue:
    name: str
    line: int

    def __str__(self):
        return f"{self.name}@L{self.line}"

    __repr__ = __str__


_ESCAPES = {"&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;", "'": "&#39;", "`": "&#x60;", "=": "&#x3D;"}
_ESC_RE = re.compile(r"[&<>\"'`=]")


def html_escape(s: str) -> str:
    return _ESC_RE.sub(lambda m: _ESCAPES[m.group(0)], s)


# token kinds
_TEXT, _VAR, _RAW, _SECTION, _INVERTED, _CLOSE, _COMMENT, _PARTIAL, _DELIM = range(9)
_STANDALONE_KINDS = (_SECTION, _INVERTED, _CLOSE, _COMMENT, _PARTIAL, _DELIM)


def _tokenize(template: str) -> List[Tuple[int, str, int]]:
    """Returns a list of (kind, value, line) tokens with standalone-line whitespace removed."""
    otag, ctag = "{{", "}}"
    pos = 0
    raw_tokens: List[list] = []  # [kind, value, start, end, line]
    n = len(template)
    line, counted_to = 1, 0  # line of ``counted_to``, advanced incrementally (not rescanned per tag)
    while pos < n:
        start = template.find(otag, pos)
        if start < 0:
            raw_tokens.append([_TEXT, template[pos:], pos, n, 0])
            break
        if start > pos:
            raw_tokens.append([_TEXT, template[pos:start], pos, start, 0])
        line += template.count("\n", counted_to, start)
        counted_to = start
        inner_start = start + len(otag)
        if otag == "{{" and template.startswith("{", inner_start):
            end = template.find("}" + ctag, inner_start)
            if end < 0:
                raise MustacheError(f"Unclosed tag at line {line}")
            raw_tokens.append([_RAW, template[inner_start + 1:end].strip(), start, end + 1 + len(ctag), line])
            pos = end + 1 + len(ctag)
            continue
        end = template.find(ctag, inner_start)
        if end < 0:
            raise MustacheError(f"Unclosed tag at line {line}")
        body = template[inner_start:end]
        pos = end + len(ctag)
        sigil = body[:1]
        if sigil == "#":
            tok = [_SECTION, body[1:].strip()]
        elif sigil == "^":
            tok = [_INVERTED, body[1:].strip()]
        elif sigil == "/":
            tok = [_CLOSE, body[1:].strip()]
        elif sigil == "!":
            tok = [_COMMENT, ""]
        elif sigil == ">":
            tok = [_PARTIAL, body[1:].strip()]
        elif sigil == "&":
            tok = [_RAW, body[1:].strip()]
        elif sigil == "=" and body.endswith("="):
            parts = body[1:-1].strip().split()
            if len(parts) != 2:
                raise MustacheError(f"Invalid delimiter change at line {line}")
            otag, ctag = parts
            tok = [_DELIM, ""]
        else:
            tok = [_VAR, body.strip()]
        raw_tokens.append(tok + [start, pos, line])

    # standalone detection: a non-value tag alone on its line (only whitespace around it)
    out: List[Tuple[int, str, int]] = []
    for i, t in enumerate(raw_tokens):
        kind = t[0]
        if kind in _STANDALONE_KINDS:
            ls = template.rfind("\n", 0, t[2]) + 1
            le = template.find("\n", t[3])
            le_eff = n if le < 0 else le
            before = template[ls:t[2]]
            after = template[t[3]:le_eff]
            if before.strip() == "" and after.strip() == "":
                # make sure no other tag shares the line (tokens are in position order, so only
                # the neighbours up to the line's bounds need looking at)
                alone = True
                j = i - 1
                while alone and j >= 0 and raw_tokens[j][2] >= ls:
                    alone = raw_tokens[j][0] == _TEXT
                    j -= 1
                j = i + 1
                while alone and j < len(raw_tokens) and raw_tokens[j][2] < le_eff + 1:
                    alone = raw_tokens[j][0] == _TEXT
                    j += 1
                if alone:
                    t.append((ls, le_eff + 1 if le >= 0 else le_eff))
    # rebuild text tokens honoring removed ranges
    removed = [t[5] for t in raw_tokens if len(t) > 5]
    for t in raw_tokens:
        if t[0] == _TEXT:
            s, e = t[2], t[3]
            pieces = []
            cur = s
            for rs, re_ in removed:
                if re_ <= cur or rs >= e:
                    continue
                if rs > cur:
                    pieces.append(template[cur:rs])
                cur = max(cur, re_)
            if cur < e:
                pieces.append(template[cur:e])
            txt = "".join(pieces)
            if txt:
                out.append((_TEXT, txt, 0))
        else:
            out.append((t[0], t[1], t[4]))
    return out


def _parse(tokens, i=0, closing: Optional[str] = None):
    nodes = []
    while i < len(tokens):
        kind, val, line = tokens[i]
        if kind == _CLOSE:
            if val != closing:
                raise MustacheError(f"Unexpected closing tag {{{{/{val}}}}} at line {line}")
            return nodes, i + 1
        if kind in (_SECTION, _INVERTED):
            children, i = _parse(tokens, i + 1, val)
            nodes.append((kind, val, line, children))
            continue
        if kind in (_COMMENT, _DELIM, _PARTIAL):
            i += 1
            continue
        nodes.append((kind, val, line, None))
        i += 1
    if closing is not None:
        raise MustacheError(f"Unclosed section {{{{#{closing}}}}}")
    return nodes, i


_MISSING = object()


def _is_map(x) -> bool:
    # a plain dict first: typing.Mapping's isinstance goes through the ABC machinery on every
    # variable of every template (~200 lookups in an hdfs-site.xml)
    return type(x) is dict or isinstance(x, collections.abc.Mapping)


def _lookup(stack: List[Any], name: str):
    if name == ".":
        return stack[-1]
    if "." in name:
        # jmustache (non-standards mode) tries the whole key first: Universe options are
        # flattened to keys like "service.user" (CosmosRenderer.flattenPropertyTree).
        for ctx in reversed(stack):
            if _is_map(ctx) and name in ctx:
                return ctx[name]
    parts = name.split(".")
    for ctx in reversed(stack):
        if _is_map(ctx) and parts[0] in ctx:
            v = ctx[parts[0]]
            for p in parts[1:]:
                if _is_map(v) and p in v:
                    v = v[p]
                else:
                    return _MISSING
            return v
    return _MISSING


def _to_str(v) -> str:
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float) and v.is_integer():
        return str(v)
    return str(v)


def _truthy(v) -> bool:
    if v is _MISSING or v is None or v is False:
        return False
    if isinstance(v, (list, tuple)) and not v:
        return False
    if isinstance(v, str) and v == "":
        return False
    return True


def _render(nodes, stack, out: List[str], missing: List[MissingValue]) -> None:
    for kind, val, line, children in nodes:
        if kind == _TEXT:
            out.append(val)
        elif kind in (_VAR, _RAW):
            v = _lookup(stack, val)
            if v is _MISSING:
                missing.append(MissingValue(val, line))
                continue
            if v is None:
                continue
            s = _to_str(v)
            out.append(html_escape(s) if kind == _VAR else s)
        elif kind == _SECTION:
            v = _lookup(stack, val)
            if not _truthy(v):
                continue
            if isinstance(v, (list, tuple)):
                for item in v:
                    _render(children, stack + [item], out, missing)
            elif _is_map(v):
                _render(children, stack + [v], out, missing)
            else:
                _render(children, stack, out, missing)
        elif kind == _INVERTED:
            v = _lookup(stack, val)
            if not _truthy(v):
                _render(children, stack, out, missing)


def _coerce_env(values: Mapping[str, Any]) -> Dict[str, Any]:
    out = {}
    for k, v in values.items():
        if isinstance(v, str) and v.lower() in ("true", "false"):
            out[k] = v.lower() == "true"
        else:
            out[k] = v
    return out


# parsed templates by content: a scheduler renders the same svc.yml and config templates on every
# start, config update and (for tasks' config files) validation pass
_PARSED: Dict[str, list] = {}
_PARSED_MAX = 256


def _parsed(content: str) -> list:
    nodes = _PARSED.get(content)
    if nodes is None:
        nodes, _ = _parse(_tokenize(content))
        if len(_PARSED) >= _PARSED_MAX:
            _PARSED.clear()
        _PARSED[content] = nodes
    return nodes


def render_mustache(template_name: str, content: str, values: Mapping[str, Any],
                    missing_values: Optional[List[MissingValue]] = None) -> str:
    nodes = _parsed(content)
    out: List[str] = []
    missing: List[MissingValue] = [] if missing_values is None else missing_values
    _render(nodes, [_coerce_env(values)], out, missing)
    return "".join(out)


def validate_missing_values(template_name: str, values: Mapping[str, Any], missing: List[MissingValue]) -> None:
    if missing:
        ordered = dict(sorted(values.items()))
        raise MustacheError(
            f"Missing {len(missing)} value{'' if len(missing) == 1 else 's'} when rendering {template_name}:\n"
            f"- Missing values: {missing}\n- Provided values: {ordered}")


def render_mustache_throw_if_missing(template_name: str, content: str, values: Mapping[str, Any]) -> str:
    missing: List[MissingValue] = []
    rendered = render_mustache(template_name, content, values, missing)
    validate_missing_values(template_name, values, missing)
    return rendered
