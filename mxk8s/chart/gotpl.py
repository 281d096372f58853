"""A small Go ``text/template`` + Helm-function engine for offline chart rendering.

``helm`` is not available in the build environment (and has no network), so
``charts/amd-gpu-stack`` is rendered by this engine for tests, for the static
manifests in ``deploy/`` and for ``mxk8s render``.  It implements the subset
of Go templates the chart uses — and the chart uses nothing else, so the same
templates work unchanged with real ``helm install`` (the reference's install
path, /root/reference/README.md:264-272):

* actions ``{{ }}`` with ``{{-`` / ``-}}`` whitespace trimming, comments
* ``if / else if / else / end``, ``range`` (with ``$k, $v :=``), ``with``,
  ``define`` / ``template`` / ``include``, ``$var :=`` and ``$var =``
* pipelines ``a | f x | g`` (the piped value is the last argument), parens
* Helm/Sprig functions: default quote squote toYaml toJson nindent indent int
  toString eq ne lt gt le ge not and or empty required fail printf trim
  trimSuffix trimPrefix lower upper replace contains hasKey list dict ternary
  trunc kindIs b64enc join
"""
from __future__ import annotations

import base64
import json
import re
from typing import Any

import yaml


class TemplateError(Exception):
    pass


class FailError(TemplateError):
    """Raised by the ``fail`` / ``required`` functions (Helm aborts the install)."""


# --------------------------------------------------------------------------
# lexing: split text into literal chunks and actions
# --------------------------------------------------------------------------

_ACTION = re.compile(r"\{\{(-?)\s*(.*?)\s*(-?)\}\}", re.S)


def _split(src: str):
    out = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        out.append(("text", text))
        out.append(("action", m.group(2), m.group(1) == "-", m.group(3) == "-"))
        pos = m.end()
    out.append(("text", src[pos:]))
    # apply trim markers
    for i, item in enumerate(out):
        if item[0] != "action":
            continue
        if item[2] and i > 0 and out[i - 1][0] == "text":
            out[i - 1] = ("text", out[i - 1][1].rstrip(" \t\r\n"))
        if item[3] and i + 1 < len(out) and out[i + 1][0] == "text":
            out[i + 1] = ("text", out[i + 1][1].lstrip(" \t\r\n"))
    return [x for x in out if not (x[0] == "text" and x[1] == "")]


_TOKEN = re.compile(r'''\s*(?:
    (?P<str>"(?:[^"\\]|\\.)*"|`[^`]*`) |
    (?P<num>-?\d+(?:\.\d+)?) |
    (?P<op>:=|=|\||\(|\)|,) |
    (?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*) |
    (?P<field>(?:\.[A-Za-z0-9_]+)+|\.) |
    (?P<ident>[A-Za-z_][A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)
)''', re.X)


def _tokens(s: str):
    pos, out = 0, []
    s = s.strip()
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise TemplateError(f"cannot tokenize {s[pos:]!r}")
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
        pos = m.end()
    return out


# --------------------------------------------------------------------------
# parsing
# --------------------------------------------------------------------------

class Node:
    pass


class Text(Node):
    def __init__(self, s):
        self.s = s


class Action(Node):
    def __init__(self, pipe, assign=None, declare=False):
        self.pipe, self.assign, self.declare = pipe, assign, declare


class If(Node):
    def __init__(self):
        self.branches = []   # [(pipe, body)]
        self.else_body = None


class Range(Node):
    def __init__(self, pipe, kvar, vvar, body):
        self.pipe, self.kvar, self.vvar, self.body = pipe, kvar, vvar, body
        self.else_body = None


class With(Node):
    def __init__(self, pipe, body):
        self.pipe, self.body = pipe, body
        self.else_body = None


class TemplateCall(Node):
    def __init__(self, name, pipe):
        self.name, self.pipe = name, pipe


def _parse_pipe(toks):
    """toks -> list of commands; each command = list of operands."""
    cmds, cur, depth, group = [], [], 0, []
    i = 0
    while i < len(toks):
        kind, val = toks[i]
        if kind == "op" and val == "(":
            # collect a parenthesized sub-pipeline
            depth, j = 1, i + 1
            while j < len(toks) and depth:
                if toks[j] == ("op", "("):
                    depth += 1
                elif toks[j] == ("op", ")"):
                    depth -= 1
                j += 1
            cur.append(("pipe", _parse_pipe(toks[i + 1:j - 1])))
            i = j
            continue
        if kind == "op" and val == "|":
            cmds.append(cur)
            cur = []
        else:
            cur.append((kind, val))
        i += 1
    cmds.append(cur)
    del group
    return cmds


def _parse_assign(toks):
    # $a := pipe   |   $a, $b := pipe (range)   |   $a = pipe
    if len(toks) >= 3 and toks[0][0] == "var" and toks[1] in (("op", ":="), ("op", "=")):
        return toks[0][1], None, toks[1][1] == ":=", toks[2:]
    if (len(toks) >= 5 and toks[0][0] == "var" and toks[1] == ("op", ",")
            and toks[2][0] == "var" and toks[3] == ("op", ":=")):
        return toks[0][1], toks[2][1], True, toks[4:]
    return None, None, False, toks


def parse(src: str, defines: dict) -> list:
    items = _split(src)
    pos = 0

    def block(stop):
        nonlocal pos
        body = []
        while pos < len(items):
            it = items[pos]
            if it[0] == "text":
                body.append(Text(it[1]))
                pos += 1
                continue
            a = it[1]
            if a.startswith("/*"):
                pos += 1
                continue
            word = a.split(None, 1)[0] if a else ""
            rest = a[len(word):].strip()
            if word in stop:
                return body, word, rest
            pos += 1
            if word == "if":
                node = If()
                cond = _parse_pipe(_tokens(rest))
                while True:
                    b, w, r = block({"else", "end"})
                    node.branches.append((cond, b))
                    pos += 1
                    if w == "end":
                        break
                    if r.startswith("if"):
                        cond = _parse_pipe(_tokens(r[2:]))
                        continue
                    node.else_body, w2, _ = block({"end"})
                    pos += 1
                    break
                body.append(node)
            elif word == "range":
                v1, v2, _, toks = _parse_assign(_tokens(rest))
                kvar, vvar = (v1, v2) if v2 else (None, v1)
                b, w, _ = block({"else", "end"})
                pos += 1
                node = Range(_parse_pipe(toks), kvar, vvar, b)
                if w == "else":
                    node.else_body, _, _ = block({"end"})
                    pos += 1
                body.append(node)
            elif word == "with":
                b, w, _ = block({"else", "end"})
                pos += 1
                node = With(_parse_pipe(_tokens(rest)), b)
                if w == "else":
                    node.else_body, _, _ = block({"end"})
                    pos += 1
                body.append(node)
            elif word == "define":
                name = json.loads(rest)
                b, _, _ = block({"end"})
                pos += 1
                defines[name] = b
            elif word == "template":
                toks = _tokens(rest)
                name = json.loads(toks[0][1])
                body.append(TemplateCall(name, _parse_pipe(toks[1:]) if len(toks) > 1 else None))
            elif word in ("end", "else"):
                raise TemplateError(f"unexpected {{{{{word}}}}}")
            else:
                v, _, decl, toks = _parse_assign(_tokens(a))
                body.append(Action(_parse_pipe(toks), v, decl))
        if stop:
            raise TemplateError(f"missing {{{{end}}}} (expected one of {sorted(stop)})")
        return body, None, None

    body, _, _ = block(set())
    return body


# --------------------------------------------------------------------------
# evaluation
# --------------------------------------------------------------------------

def _truthy(v) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, dict, tuple)):
        return len(v) > 0
    return True


def _to_yaml(v) -> str:
    if v is None:
        return "null"
    s = yaml.safe_dump(v, default_flow_style=False, sort_keys=True).rstrip("\n")
    if s.endswith("\n..."):
        s = s[:-4].rstrip("\n")
    return s


def _indent(n, s):
    pad = " " * int(n)
    return "\n".join(pad + line if line else line for line in str(s).split("\n"))


def _go_str(v) -> str:
    if v is None:
        return "<no value>"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if isinstance(v, (dict, list)):
        return json.dumps(v)
    return str(v)


def _printf(fmt, *args):
    conv = []
    for a in args:
        conv.append(a)
    py = re.sub(r"%v", "%s", fmt)
    return py % tuple(_go_str(a) if isinstance(a, (bool, type(None))) else a for a in conv)


def _required(msg, v):
    if not _truthy(v) and v != 0:
        raise FailError(msg)
    return v


def _fail(msg):
    raise FailError(msg)


def _dict(*kv):
    return {kv[i]: kv[i + 1] for i in range(0, len(kv), 2)}


FUNCS = {
    "default": lambda d, v=None: v if _truthy(v) else d,
    "quote": lambda *v: " ".join(json.dumps(_go_str(x)) for x in v),
    "squote": lambda *v: " ".join("'" + _go_str(x) + "'" for x in v),
    "toYaml": _to_yaml,
    "toJson": lambda v: json.dumps(v, sort_keys=True),
    "nindent": lambda n, s: "\n" + _indent(n, s),
    "indent": _indent,
    "int": lambda v: int(float(v)) if v not in (None, "") else 0,
    "toString": _go_str,
    "eq": lambda a, *b: any(a == x for x in b),
    "ne": lambda a, b: a != b,
    "lt": lambda a, b: a < b,
    "gt": lambda a, b: a > b,
    "le": lambda a, b: a <= b,
    "ge": lambda a, b: a >= b,
    "not": lambda v: not _truthy(v),
    "and": lambda *v: next((x for x in v if not _truthy(x)), v[-1]),
    "or": lambda *v: next((x for x in v if _truthy(x)), v[-1]),
    "empty": lambda v: not _truthy(v),
    "required": _required,
    "fail": _fail,
    "printf": _printf,
    "trim": lambda s: str(s).strip(),
    "trimSuffix": lambda suf, s: s[:-len(suf)] if suf and str(s).endswith(suf) else s,
    "trimPrefix": lambda pre, s: s[len(pre):] if pre and str(s).startswith(pre) else s,
    "lower": lambda s: str(s).lower(),
    "upper": lambda s: str(s).upper(),
    "replace": lambda old, new, s: str(s).replace(old, new),
    "contains": lambda sub, s: sub in str(s),
    "hasKey": lambda d, k: isinstance(d, dict) and k in d,
    "list": lambda *v: list(v),
    "dict": _dict,
    "ternary": lambda a, b, c: a if _truthy(c) else b,
    "trunc": lambda n, s: str(s)[:int(n)] if int(n) >= 0 else str(s)[int(n):],
    "kindIs": lambda kind, v: {"map": dict, "slice": list, "string": str, "bool": bool,
                               "int": int, "float64": float}.get(kind, type(None)) is type(v)
    if kind != "int" else isinstance(v, int) and not isinstance(v, bool),
    "b64enc": lambda s: base64.b64encode(str(s).encode()).decode(),
    "join": lambda sep, v: sep.join(_go_str(x) for x in v),
}


class _Scope:
    def __init__(self, dot, root, variables=None):
        self.dot, self.root = dot, root
        self.vars = variables if variables is not None else {"$": root}


def _field(obj, path: str):
    for part in [p for p in path.split(".") if p]:
        if isinstance(obj, dict):
            obj = obj.get(part)
        elif obj is None:
            return None
        else:
            obj = getattr(obj, part, None)
    return obj


class Engine:
    def __init__(self):
        self.defines: dict = {}

    def add(self, src: str) -> list:
        return parse(src, self.defines)

    def render_nodes(self, nodes, scope) -> str:
        out = []
        for n in nodes:
            if isinstance(n, Text):
                out.append(n.s)
            elif isinstance(n, Action):
                v = self.pipe(n.pipe, scope)
                if n.assign:
                    scope.vars[n.assign] = v
                else:
                    out.append(_go_str(v))
            elif isinstance(n, If):
                done = False
                for cond, body in n.branches:
                    if _truthy(self.pipe(cond, scope)):
                        out.append(self.render_nodes(body, scope))
                        done = True
                        break
                if not done and n.else_body is not None:
                    out.append(self.render_nodes(n.else_body, scope))
            elif isinstance(n, With):
                v = self.pipe(n.pipe, scope)
                if _truthy(v):
                    out.append(self.render_nodes(n.body, _Scope(v, scope.root, dict(scope.vars))))
                elif n.else_body is not None:
                    out.append(self.render_nodes(n.else_body, scope))
            elif isinstance(n, Range):
                v = self.pipe(n.pipe, scope)
                items = sorted(v.items()) if isinstance(v, dict) else list(enumerate(v or []))
                if not items and n.else_body is not None:
                    out.append(self.render_nodes(n.else_body, scope))
                for k, val in items:
                    vs = dict(scope.vars)
                    if n.kvar:
                        vs[n.kvar] = k
                    if n.vvar:
                        vs[n.vvar] = val
                    out.append(self.render_nodes(n.body, _Scope(val, scope.root, vs)))
            elif isinstance(n, TemplateCall):
                dot = self.pipe(n.pipe, scope) if n.pipe else None
                out.append(self.include(n.name, dot, scope.root))
        return "".join(out)

    def include(self, name, dot, root) -> str:
        if name not in self.defines:
            raise TemplateError(f"template {name!r} not defined")
        return self.render_nodes(self.defines[name], _Scope(dot, root))

    def operand(self, tok, scope):
        kind, val = tok
        if kind == "pipe":
            return self.pipe(val, scope)
        if kind == "str":
            return json.loads(val) if val.startswith('"') else val[1:-1]
        if kind == "num":
            return float(val) if "." in val else int(val)
        if kind == "field":
            return scope.dot if val == "." else _field(scope.dot, val)
        if kind == "var":
            name, _, path = val.partition(".")
            if name not in scope.vars:
                raise TemplateError(f"undefined variable {name}")
            return _field(scope.vars[name], path) if path else scope.vars[name]
        if kind == "ident":
            if val in ("true", "false"):
                return val == "true"
            if val == "nil":
                return None
            return ("func", val)
        raise TemplateError(f"bad operand {tok}")

    def command(self, cmd, scope, piped=None, has_piped=False):
        if not cmd:
            raise TemplateError("empty command")
        head = self.operand(cmd[0], scope)
        if isinstance(head, tuple) and head and head[0] == "func":
            name = head[1]
            args = [self.operand(t, scope) for t in cmd[1:]]
            if has_piped:
                args.append(piped)
            if name == "include":
                return self.include(args[0], args[1] if len(args) > 1 else None, scope.root)
            if name == "tpl":
                eng = Engine()
                eng.defines = self.defines
                return eng.render_nodes(eng.add(args[0]), _Scope(args[1], scope.root))
            fn = FUNCS.get(name)
            if fn is None:
                raise TemplateError(f"function {name!r} not defined")
            try:
                return fn(*args)
            except FailError:
                raise
            except TypeError as e:
                raise TemplateError(f"{name}: {e}") from e
        if len(cmd) > 1 or has_piped:
            raise TemplateError(f"cannot call non-function {cmd[0][1]}")
        return head

    def pipe(self, cmds, scope):
        v, has = None, False
        for c in cmds:
            v = self.command(c, scope, v, has)
            has = True
        return v


def render_string(src: str, values: dict, release=None, chart=None, helpers: str = "") -> str:
    eng = Engine()
    if helpers:
        eng.add(helpers)
    nodes = eng.add(src)
    root = {"Values": values, "Release": release or {}, "Chart": chart or {},
            "Capabilities": {"KubeVersion": {"Version": "v1.34.0"}}}
    return eng.render_nodes(nodes, _Scope(root, root))
