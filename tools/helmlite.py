#!/usr/bin/env python3
"""helmlite — an offline renderer for the Go-template subset our Helm charts use.

There is no ``helm`` binary in the build/test environment, so chart tests render
with this instead; when ``helm`` exists, ``render_chart(...,
prefer_helm=True)`` shells out to ``helm template`` instead.

Supported: text/actions with ``{{-``/``-}}`` trimming, comments, pipelines,
parenthesised sub-pipelines, variables (``$x := ...``, ``$x = ...``, ``$``),
field chains on dicts and variables, ``if/else if/else``, ``range`` (with
``$i, $v :=`` and ``else``), ``with``/``else``, ``define``/``include``/``template``,
and the Sprig/Helm functions listed in ``FUNCS``.
"""
from __future__ import annotations

import base64
import json
import os
import re
import sys

import yaml

# ---------------------------------------------------------------- lexing
_ACTION = re.compile(r"\{\{(-?)(.*?)(-?)\}\}", re.S)


def _lex(src: str):
    """-> list of ("text", str) | ("action", str)"""
    out = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1) == "-":
            text = text.rstrip(" \t\r\n")
        out.append(["text", text])
        out.append(["action", m.group(2).strip(), m.group(3) == "-"])
        pos = m.end()
    out.append(["text", src[pos:]])
    # apply right-trim markers
    res = []
    trim_next = False
    for tok in out:
        if tok[0] == "text":
            t = tok[1].lstrip(" \t\r\n") if trim_next else tok[1]
            trim_next = False
            if t:
                res.append(("text", t))
        else:
            res.append(("action", tok[1]))
            trim_next = tok[2]
    return res


_TOK = re.compile(r"""
    (?P<str>"(?:\\.|[^"\\])*") |
    (?P<raw>`[^`]*`) |
    (?P<num>-?\d+(?:\.\d+)?) |
    (?P<decl>:=) |
    (?P<assign>=) |
    (?P<pipe>\|) |
    (?P<lp>\() | (?P<rp>\)) |
    (?P<comma>,) |
    (?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*) |
    (?P<field>(?:\.[A-Za-z0-9_]+)+|\.) |
    (?P<ident>[A-Za-z_][A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*) |
    (?P<ws>\s+)
""", re.X)


def _tokens(s: str):
    pos, out = 0, []
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m:
            raise SyntaxError(f"bad template expression near {s[pos:pos + 20]!r}")
        pos = m.end()
        k = m.lastgroup
        if k != "ws":
            out.append((k, m.group(k), m.start()))
    return out


# ---------------------------------------------------------------- parsing
class Node:
    pass


class Text(Node):
    def __init__(self, s):
        self.s = s


class Action(Node):
    def __init__(self, expr):
        self.expr = expr


class Block(Node):
    def __init__(self, kind, expr, body, orelse=None):
        self.kind, self.expr, self.body, self.orelse = kind, expr, body, orelse


class Define(Node):
    def __init__(self, name, body):
        self.name, self.body = name, body


def _parse(tokens, i=0, stop=("end",)):
    body = []
    while i < len(tokens):
        kind, val = tokens[i][0], tokens[i][1]
        if kind == "text":
            body.append(Text(val))
            i += 1
            continue
        if val.startswith("/*"):
            i += 1
            continue
        word = val.split(None, 1)[0] if val else ""
        rest = val[len(word):].strip()
        if word in ("end", "else") and word in stop or (word == "else" and "else" in stop):
            return body, i, val
        if word in ("if", "range", "with"):
            sub, j, term = _parse(tokens, i + 1, ("end", "else"))
            node = Block(word, rest, sub)
            cur = node
            while term.startswith("else"):
                erest = term[4:].strip()
                if erest.startswith("if ") or erest.startswith("with "):
                    w2 = erest.split(None, 1)
                    sub2, j, term = _parse(tokens, j + 1, ("end", "else"))
                    nb = Block(w2[0], w2[1], sub2)
                    cur.orelse = [nb]
                    cur = nb
                else:
                    sub2, j, term = _parse(tokens, j + 1, ("end",))
                    cur.orelse = sub2
            body.append(node)
            i = j + 1
            continue
        if word == "define":
            sub, j, _ = _parse(tokens, i + 1, ("end",))
            body.append(Define(json.loads(rest), sub))
            i = j + 1
            continue
        if word == "block":
            raise SyntaxError("block not supported")
        body.append(Action(val))
        i += 1
    if stop:
        raise SyntaxError("unterminated block: missing {{ end }}")
    return body, i, ""


# ---------------------------------------------------------------- evaluation
class Ctx:
    def __init__(self, dot, root, vars_, tpls):
        self.dot, self.root, self.vars, self.tpls = dot, root, vars_, tpls

    def child(self, dot=None):
        return Ctx(self.dot if dot is None else dot, self.root, dict(self.vars), self.tpls)


def _truthy(v):
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, dict, tuple)):
        return len(v) > 0
    return True


def _get(obj, path):
    for p in path:
        if p == "":
            continue
        if isinstance(obj, dict):
            obj = obj.get(p)
        elif obj is None:
            return None
        else:
            obj = getattr(obj, p, None)
    return obj


def _to_yaml(v):
    if v is None:
        return "null"
    s = yaml.safe_dump(v, default_flow_style=False, sort_keys=True, width=10**9)
    s = s.rstrip("\n")
    if s.endswith("\n..."):
        s = s[:-4].rstrip("\n")
    return s


def _indent(n, s):
    pad = " " * int(n)
    return "\n".join(pad + ln if ln else ln for ln in str(s).split("\n"))


def _printf(fmt, *args):
    fmt = re.sub(r"%v|%s|%d", "%s", fmt)
    return fmt % tuple("" if a is None else a for a in args)


def _required(msg, v):
    if v is None or v == "":
        raise ValueError(msg)
    return v


def _fail(msg):
    raise ValueError(msg)


FUNCS = {
    "default": lambda d, v=None: v if _truthy(v) else d,
    "quote": lambda *a: " ".join(json.dumps("" if x is None else str(x)) for x in a),
    "squote": lambda *a: " ".join("'" + ("" if x is None else str(x)) + "'" for x in a),
    "toYaml": _to_yaml,
    "toJson": lambda v: json.dumps(v, separators=(",", ":")),
    "indent": _indent,
    "nindent": lambda n, s: "\n" + _indent(n, s),
    "printf": _printf,
    "print": lambda *a: "".join(str(x) for x in a),
    "trunc": lambda n, s: str(s)[:int(n)] if int(n) >= 0 else str(s)[int(n):],
    "trimSuffix": lambda suf, s: s[: -len(suf)] if suf and str(s).endswith(suf) else s,
    "trimPrefix": lambda pre, s: s[len(pre):] if pre and str(s).startswith(pre) else s,
    "trim": lambda s: str(s).strip(),
    "lower": lambda s: str(s).lower(),
    "upper": lambda s: str(s).upper(),
    "replace": lambda old, new, s: str(s).replace(old, new),
    "contains": lambda sub, s: sub in str(s),
    "hasPrefix": lambda pre, s: str(s).startswith(pre),
    "hasSuffix": lambda suf, s: str(s).endswith(suf),
    "eq": lambda a, *b: any(a == x for x in b),
    "ne": lambda a, b: a != b,
    "lt": lambda a, b: a < b, "le": lambda a, b: a <= b,
    "gt": lambda a, b: a > b, "ge": lambda a, b: a >= b,
    "and": lambda *a: next((x for x in a if not _truthy(x)), a[-1]),
    "or": lambda *a: next((x for x in a if _truthy(x)), a[-1]),
    "not": lambda a: not _truthy(a),
    "len": lambda a: len(a) if a is not None else 0,
    "index": lambda obj, *keys: _index(obj, keys),
    "list": lambda *a: list(a),
    "dict": lambda *a: {a[i]: a[i + 1] for i in range(0, len(a), 2)},
    "required": _required,
    "fail": _fail,
    "empty": lambda v: not _truthy(v),
    "b64enc": lambda s: base64.b64encode(str(s).encode()).decode(),
    "int": lambda v: int(v or 0),
    "float64": lambda v: float(v or 0),
    "toString": lambda v: "" if v is None else str(v),
    "join": lambda sep, xs: sep.join(str(x) for x in (xs or [])),
    "ternary": lambda a, b, c: a if _truthy(c) else b,
    "hasKey": lambda d, k: isinstance(d, dict) and k in d,
    "kindIs": lambda k, v: {"map": dict, "slice": list, "string": str, "bool": bool}.get(k, object) is type(v),
    "add": lambda *a: sum(int(x) for x in a),
    "sub": lambda a, b: int(a) - int(b),
    "mul": lambda a, b: int(a) * int(b),
    "max": lambda *a: max(a), "min": lambda *a: min(a),
    "first": lambda xs: xs[0] if xs else None,
    "last": lambda xs: xs[-1] if xs else None,
    "keys": lambda d: sorted(d.keys()),
    "sha256sum": lambda s: __import__("hashlib").sha256(str(s).encode()).hexdigest(),
}


def _index(obj, keys):
    for k in keys:
        if isinstance(obj, dict):
            obj = obj.get(k)
        elif isinstance(obj, (list, tuple)):
            if not 0 <= int(k) < len(obj):
                raise IndexError(f"index out of range: {k}")
            obj = obj[int(k)]
        else:
            return None
    return obj


class Renderer:
    def __init__(self, templates: dict[str, str]):
        self.defs: dict[str, list] = {}
        self.trees = {}
        for name, src in templates.items():
            tree, _, _ = _parse(_lex(src), 0, ())
            self.trees[name] = tree
            self._collect(tree)

    def _collect(self, tree):
        for n in tree:
            if isinstance(n, Define):
                self.defs[n.name] = n.body

    # -- expression evaluation
    def _operand(self, toks, i, ctx):
        k, v = toks[i][0], toks[i][1]
        if k == "str":
            return json.loads(v), i + 1
        if k == "raw":
            return v[1:-1], i + 1
        if k == "num":
            return (float(v) if "." in v else int(v)), i + 1
        if k == "field":
            return (ctx.dot if v == "." else _get(ctx.dot, v[1:].split("."))), i + 1
        if k == "var":
            name, _, rest = v.partition(".")
            base = ctx.root if name == "$" else ctx.vars.get(name)
            if name != "$" and name not in ctx.vars:
                raise NameError(f"undefined variable {name}")
            return (_get(base, rest.split(".")) if rest else base), i + 1
        if k == "lp":
            val, j = self._pipeline(toks, i + 1, ctx)
            if j >= len(toks) or toks[j][0] != "rp":
                raise SyntaxError("missing )")
            j += 1
            # `(expr).field` only when the field is glued to the closing paren
            if j < len(toks) and toks[j][0] == "field" and toks[j][1] != "." and \
                    toks[j][2] == toks[j - 1][2] + 1:
                val = _get(val, toks[j][1][1:].split("."))
                j += 1
            return val, j
        if k == "ident":
            if v in ("true", "false"):
                return v == "true", i + 1
            if v == "nil":
                return None, i + 1
        raise SyntaxError(f"unexpected token {v!r}")

    def _command(self, toks, i, ctx, piped=_truthy):
        k, v = toks[i][0], toks[i][1]
        if k == "ident" and v not in ("true", "false", "nil"):
            fn = v
            args = []
            i += 1
            while i < len(toks) and toks[i][0] not in ("pipe", "rp"):
                a, i = self._operand(toks, i, ctx)
                args.append(a)
            return (fn, args), i
        val, i = self._operand(toks, i, ctx)
        # field access on a parenthesised value: (expr).field
        return (None, [val]), i

    def _call(self, fn, args, ctx):
        if fn in ("include", "template"):
            name, dot = args[0], (args[1] if len(args) > 1 else None)
            if name not in self.defs:
                raise KeyError(f"template {name!r} not defined")
            return self._render(self.defs[name], ctx.child(dot))
        if fn == "tpl":
            return Renderer({"_tpl": args[0]})._render(Renderer({"_tpl": args[0]}).trees["_tpl"],
                                                      ctx.child(args[1]))
        if fn not in FUNCS:
            raise NameError(f"function {fn!r} not supported by helmlite")
        return FUNCS[fn](*args)

    def _pipeline(self, toks, i, ctx):
        val = None
        first = True
        while i < len(toks):
            (fn, args), i = self._command(toks, i, ctx)
            if not first:
                args = args + [val]
            if fn is None:
                val = args[0] if first else args[-1]
            else:
                val = self._call(fn, args, ctx)
            first = False
            if i < len(toks) and toks[i][0] == "pipe":
                i += 1
                continue
            break
        return val, i

    def _eval(self, expr, ctx):
        toks = _tokens(expr)
        if len(toks) >= 2 and toks[0][0] == "var" and toks[1][0] in ("decl", "assign"):
            val, _ = self._pipeline(toks, 2, ctx)
            ctx.vars[toks[0][1]] = val
            return None, True
        val, j = self._pipeline(toks, 0, ctx)
        if j != len(toks):
            raise SyntaxError(f"trailing tokens in {expr!r}")
        return val, False

    def _render(self, tree, ctx) -> str:
        out = []
        for n in tree:
            if isinstance(n, Text):
                out.append(n.s)
            elif isinstance(n, Define):
                continue
            elif isinstance(n, Action):
                val, is_assign = self._eval(n.expr, ctx)
                if not is_assign:
                    out.append(_fmt(val))
            elif isinstance(n, Block):
                out.append(self._block(n, ctx))
        return "".join(out)

    def _block(self, n, ctx):
        if n.kind == "if":
            val, _ = self._eval(n.expr, ctx)
            if _truthy(val):
                return self._render(n.body, ctx)
            return self._render(n.orelse or [], ctx)
        if n.kind == "with":
            val, _ = self._eval(n.expr, ctx)
            if _truthy(val):
                return self._render(n.body, ctx.child(val))
            return self._render(n.orelse or [], ctx)
        # range
        toks = _tokens(n.expr)
        names = []
        if "decl" in [t[0] for t in toks]:
            d = [t[0] for t in toks].index("decl")
            names = [t[1] for t in toks[:d] if t[0] == "var"]
            toks = toks[d + 1:]
        coll, _ = self._pipeline(toks, 0, ctx)
        if not _truthy(coll):
            return self._render(n.orelse or [], ctx)
        items = coll.items() if isinstance(coll, dict) else enumerate(coll) if not isinstance(coll, int) \
            else enumerate(range(coll))
        if isinstance(coll, dict):
            items = sorted(coll.items())
        out = []
        for k, v in items:
            c = ctx.child(v)
            if len(names) == 1:
                c.vars[names[0]] = v
            elif len(names) == 2:
                c.vars[names[0]], c.vars[names[1]] = k, v
            out.append(self._render(n.body, c))
        return "".join(out)

    def render(self, name, values, release=None, chart=None) -> str:
        root = {"Values": values, "Release": release or {}, "Chart": chart or {},
                "Capabilities": {"KubeVersion": {"Version": "v1.31.0"}}, "Template": {"Name": name}}
        return self._render(self.trees[name], Ctx(root, root, {}, self.defs))


def _fmt(v):
    if v is None:
        return "<no value>"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if isinstance(v, (dict, list)):
        return _go_repr(v)
    return str(v)


def _go_repr(v):
    if isinstance(v, dict):
        return "map[" + " ".join(f"{k}:{_go_repr(x)}" for k, x in sorted(v.items())) + "]"
    if isinstance(v, list):
        return "[" + " ".join(_go_repr(x) for x in v) + "]"
    return _fmt(v)


def deep_merge(a: dict, b: dict) -> dict:
    out = dict(a)
    for k, v in (b or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = deep_merge(out[k], v)
        else:
            out[k] = v
    return out


def render_chart(chart_dir: str, values: dict | None = None, release: str = "release",
                 namespace: str = "default", prefer_helm: bool = False) -> dict[str, str]:
    """Render every template of a chart -> {template path: text}."""
    if prefer_helm and _which("helm"):
        return _helm_template(chart_dir, values, release, namespace)
    with open(os.path.join(chart_dir, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        vals = yaml.safe_load(f) or {}
    vals = deep_merge(vals, values or {})
    tdir = os.path.join(chart_dir, "templates")
    srcs = {}
    for fn in sorted(os.listdir(tdir)):
        if fn.endswith((".yaml", ".yml", ".tpl", ".txt")):
            with open(os.path.join(tdir, fn)) as f:
                srcs[fn] = f.read()
    r = Renderer(srcs)
    chart_obj = {"Name": chart.get("name"), "Version": chart.get("version"),
                 "AppVersion": chart.get("appVersion", "")}
    rel = {"Name": release, "Namespace": namespace, "Service": "Helm", "IsInstall": True}
    out = {}
    for fn in srcs:
        if fn.startswith("_") or fn.endswith(".tpl"):
            continue
        out[fn] = r.render(fn, vals, rel, chart_obj)
    return out


def manifests(rendered: dict[str, str]) -> list[dict]:
    docs = []
    for fn, text in rendered.items():
        for d in yaml.safe_load_all(text):
            if d:
                d.setdefault("__source", fn)
                docs.append(d)
    return docs


def _which(b):
    from shutil import which

    return which(b)


def _helm_template(chart_dir, values, release, namespace):
    import subprocess
    import tempfile

    with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as f:
        yaml.safe_dump(values or {}, f)
    out = subprocess.check_output(["helm", "template", release, chart_dir, "-n", namespace, "-f", f.name],
                                  text=True)
    return {"helm": out}


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="render a chart offline (helm template subset)")
    ap.add_argument("chart")
    ap.add_argument("-f", "--values", action="append", default=[])
    ap.add_argument("--release", default="release")
    ap.add_argument("-n", "--namespace", default="default")
    a = ap.parse_args(argv)
    vals = {}
    for p in a.values:
        with open(p) as f:
            vals = deep_merge(vals, yaml.safe_load(f) or {})
    for fn, text in render_chart(a.chart, vals, a.release, a.namespace).items():
        if text.strip():
            print(f"---\n# Source: {os.path.basename(a.chart)}/templates/{fn}")
            print(text.strip("\n"))


if __name__ == "__main__":
    sys.exit(main())
