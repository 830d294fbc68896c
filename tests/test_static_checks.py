"""Static checks over the package source, the counterpart of the reference's lint tier
(``gradle/quality.gradle`` checkstyle/findbugs, ``.pylintrc``, ``.flake8``, ``mypy.ini``; SURVEY.md
§4 "Static checks"). No linter is installed in this image, so the checks that catch real defects
are done on the AST here:

* every module parses;
* no unused imports (outside package ``__init__`` re-export modules);
* no bare ``except:`` (it also swallows ``KeyboardInterrupt``/``SystemExit``);
* no mutable default arguments (``[]``, ``{}``, ``set()``), which are shared across calls;
* no ``print(`` in library code outside CLIs, benchmarks, tools and the test harness.
"""
import ast
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dcos_commons_amd")
# modules whose job is to print (CLIs, benchmark drivers, packaging tools, the cluster stand-in)
PRINTING = ("benchmarks", "tools", "testing", "models", "__main__", "build")


def _modules():
    out = []
    for dp, dn, fn in os.walk(PKG):
        dn[:] = [d for d in dn if d != "__pycache__"]
        out.extend(os.path.join(dp, f) for f in fn if f.endswith(".py"))
    return sorted(out)


MODULES = _modules()


def _tree(path):
    with open(path, encoding="utf-8") as f:
        return ast.parse(f.read(), path)


def _rel(path):
    return os.path.relpath(path, ROOT)


def test_every_module_parses():
    for p in MODULES:
        _tree(p)


def _string_tokens(tree):
    """Names mentioned in string constants (quoted annotations, ``__all__`` entries)."""
    out = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Constant) and isinstance(node.value, str):
            text = node.value
            for ch in "[],.()|:":
                text = text.replace(ch, " ")
            out.update(t.strip("'\"") for t in text.split())
    return out


def unused_imports(tree):
    imported = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            for a in node.names:
                imported[(a.asname or a.name).split(".")[0]] = node.lineno
        elif isinstance(node, ast.ImportFrom) and node.module != "__future__":
            for a in node.names:
                if a.name != "*":
                    imported[a.asname or a.name] = node.lineno
    used = {n.id for n in ast.walk(tree) if isinstance(n, ast.Name)} | _string_tokens(tree)
    return sorted((line, name) for name, line in imported.items() if name not in used)


def test_no_unused_imports():
    problems = []
    for p in MODULES:
        if os.path.basename(p) == "__init__.py":
            continue  # package modules re-export what they import
        problems += [f"{_rel(p)}:{line}: unused import {name}" for line, name in unused_imports(_tree(p))]
    assert not problems, "\n".join(problems)


def test_no_bare_except():
    problems = [f"{_rel(p)}:{n.lineno}: bare except" for p in MODULES for n in ast.walk(_tree(p))
                if isinstance(n, ast.ExceptHandler) and n.type is None]
    assert not problems, "\n".join(problems)


def _mutable(node):
    return isinstance(node, (ast.List, ast.Dict, ast.Set)) or (
        isinstance(node, ast.Call) and isinstance(node.func, ast.Name) and node.func.id in ("list", "dict", "set")
        and not node.args and not node.keywords)


def test_no_mutable_default_arguments():
    problems = []
    for p in MODULES:
        for n in ast.walk(_tree(p)):
            if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
                for d in list(n.args.defaults) + [d for d in n.args.kw_defaults if d is not None]:
                    if _mutable(d):
                        problems.append(f"{_rel(p)}:{d.lineno}: mutable default argument")
    assert not problems, "\n".join(problems)


def test_no_print_in_library_code():
    problems = []
    for p in MODULES:
        rel = _rel(p)
        if any(part in rel.split(os.sep) or rel.endswith(part + ".py") for part in PRINTING):
            continue
        tree = _tree(p)
        mains = {n.lineno for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == "main"}
        for n in ast.walk(tree):
            if isinstance(n, ast.Call) and isinstance(n.func, ast.Name) and n.func.id == "print":
                problems.append(f"{rel}:{n.lineno}: print()")
        if mains:
            problems = [x for x in problems if not x.startswith(rel + ":")]  # a module with a CLI main()
    assert not problems, "\n".join(problems)


@pytest.mark.parametrize("src,expected", [
    ("import os\n", [(1, "os")]),
    ("import os\nos.getcwd()\n", []),
    ("from typing import List\nx: 'List[int]' = []\n", []),
    ("from a import b as c\n", [(1, "c")]),
])
def test_unused_import_detector(src, expected):
    assert unused_imports(ast.parse(src)) == expected
