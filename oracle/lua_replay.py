"""Execute the reference's own Lua scripts against a mock Redis (TEST INFRASTRUCTURE).

The reference's decision logic is Lua embedded in C# raw string literals, run by a
Redis server (TB:181-238, A:221-270).  No Lua VM, Redis or .NET exists in this image
(SURVEY.md §8c), so this module contains:

  * ``extract_script``  -- pulls the ``$$\"\"\"...\"\"\"`` literal of a C# method out of a
    reference source file, applies the C# raw-string de-indentation, the ``{{hole}}``
    interpolation (invariant culture, shortest round-trip doubles) and SE.Redis
    ``LuaScript.Prepare``'s ``@Param`` -> ``ARGV[i]`` rewrite;
  * a Lua 5.1 subset interpreter (tokenizer, recursive-descent parser, tree walker)
    with Lua 5.1 number semantics: IEEE binary64, string->number coercion in
    arithmetic (strtod), ``tostring`` = "%.14g", ``math.max/min`` argument order;
  * ``MockRedis``: ``TIME`` (injected microseconds), ``HGETALL``/``HSET`` (hash values
    stored as strings, Lua numbers formatted with round-trip precision as Redis does),
    ``EXPIRE`` with passive expiry on the ms command-time snapshot, and the Lua ->
    RESP reply conversion (number -> integer by truncation, false -> nil, true -> 1);
  * the C# reply parsing of TB:64-81 and A:440-443.

It reads /root/reference only when generating fixtures (tests/golden/make_golden.py);
nothing on the GPU box or in the product path imports it.
"""
from __future__ import annotations

import math
import re
from typing import Any, Dict, List, Optional

# ============================================================== C# literal extraction


def extract_script(cs_path: str, method: str) -> str:
    """Return the raw text of the ``$$\"\"\"`` literal returned by ``method`` (unformatted)."""
    src = open(cs_path, encoding="utf-8-sig").read()
    m = re.search(r"\b" + re.escape(method) + r"\s*\([^)]*\)\s*=>", src)
    if not m:
        raise ValueError(f"{method} not found in {cs_path}")
    start = src.index('$$"""', m.end())
    body_start = src.index("\n", start) + 1
    end = src.index('"""', body_start)
    body = src[body_start:end]
    # C# raw string literal: the closing delimiter's indentation is removed from every line.
    lines = body.split("\n")
    closing_indent = lines[-1]
    assert closing_indent.strip() == "", "closing \"\"\" must be on its own line"
    out = []
    for ln in lines[:-1]:
        if ln.strip() == "":
            out.append("")
        else:
            assert ln.startswith(closing_indent), "raw string line less indented than the closing quotes"
            out.append(ln[len(closing_indent):])
    return "\n".join(out)


def csharp_double_to_string(x: float) -> str:
    """.NET Core 3.0+ ``double.ToString()`` (shortest round-trip, invariant culture)."""
    if math.isinf(x):
        return "∞" if x > 0 else "-∞"
    if math.isnan(x):
        return "NaN"
    if x == int(x) and abs(x) < 1e15:
        return str(int(x))
    r = repr(x)
    if "e" in r:
        mant, exp = r.split("e")
        e = int(exp)
        return f"{mant}E{'+' if e >= 0 else '-'}{abs(e):02d}"
    return r


def prepare_script(template: str, holes: Dict[str, Any], params: List[str]) -> str:
    """C# ``{{name}}`` interpolation then ``LuaScript.Prepare``'s ``@Param`` -> ``ARGV[i]``."""
    def fmt(v):
        if isinstance(v, float):
            return csharp_double_to_string(v)
        return str(v)

    text = template
    for k, v in holes.items():
        text = text.replace("{{" + k + "}}", fmt(v))
    if "{{" in text:
        raise ValueError("unfilled interpolation hole")
    for i, name in enumerate(params, start=1):
        text = re.sub(r"@" + name + r"\b", f"ARGV[{i}]", text)
    return text


# ============================================================== Lua 5.1 subset: lexer

_TOKEN = re.compile(r"""
    (?P<ws>\s+) |
    (?P<comment>--[^\n]*) |
    (?P<num>0[xX][0-9a-fA-F]+|(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?) |
    (?P<str>'(?:[^'\\]|\\.)*'|"(?:[^"\\]|\\.)*") |
    (?P<name>[A-Za-z_][A-Za-z_0-9]*) |
    (?P<op>\.\.\.|\.\.|==|~=|<=|>=|[-+*/%^#<>=(){}\[\];:,.])
""", re.X)

KEYWORDS = {"and", "break", "do", "else", "elseif", "end", "false", "for", "function", "if", "in",
            "local", "nil", "not", "or", "repeat", "return", "then", "true", "until", "while"}


def tokenize(src: str):
    toks, pos = [], 0
    while pos < len(src):
        m = _TOKEN.match(src, pos)
        if not m:
            raise SyntaxError(f"lua: unexpected character {src[pos]!r} at {pos}")
        pos = m.end()
        kind = m.lastgroup
        if kind in ("ws", "comment"):
            continue
        val = m.group(kind)
        if kind == "name" and val in KEYWORDS:
            kind = "kw"
        toks.append((kind, val))
    toks.append(("eof", None))
    return toks


# ============================================================== parser -> tuples AST

_BINPRI = {"or": (1, 1), "and": (2, 2), "<": (3, 3), ">": (3, 3), "<=": (3, 3), ">=": (3, 3),
           "~=": (3, 3), "==": (3, 3), "..": (5, 4), "+": (6, 6), "-": (6, 6), "*": (7, 7),
           "/": (7, 7), "%": (7, 7), "^": (10, 9)}
_UNARY_PRI = 8


class Parser:
    def __init__(self, src: str):
        self.t = tokenize(src)
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k]

    def check(self, kind, val=None):
        tk = self.peek()
        return tk[0] == kind and (val is None or tk[1] == val)

    def accept(self, kind, val=None):
        if self.check(kind, val):
            self.i += 1
            return True
        return False

    def expect(self, kind, val=None):
        tk = self.peek()
        if not self.check(kind, val):
            raise SyntaxError(f"lua: expected {val or kind}, got {tk}")
        self.i += 1
        return tk[1]

    def chunk(self):
        body = self.block()
        self.expect("eof")
        return body

    def block(self):
        stmts = []
        while not (self.check("eof") or self.check("kw", "end") or self.check("kw", "else")
                   or self.check("kw", "elseif") or self.check("kw", "until")):
            if self.check("kw", "return"):
                self.i += 1
                exprs = [] if (self.check("kw", "end") or self.check("eof") or self.check("op", ";")) \
                    else self.exprlist()
                self.accept("op", ";")
                stmts.append(("return", exprs))
                break
            st = self.statement()
            if st is not None:
                stmts.append(st)
        return stmts

    def statement(self):
        if self.accept("op", ";"):
            return None
        if self.accept("kw", "local"):
            if self.accept("kw", "function"):
                name = self.expect("name")
                return ("local", [name], [self.funcbody()])
            names = [self.expect("name")]
            while self.accept("op", ","):
                names.append(self.expect("name"))
            exprs = self.exprlist() if self.accept("op", "=") else []
            return ("local", names, exprs)
        if self.accept("kw", "if"):
            clauses = []
            cond = self.expr()
            self.expect("kw", "then")
            clauses.append((cond, self.block()))
            els = None
            while True:
                if self.accept("kw", "elseif"):
                    c = self.expr()
                    self.expect("kw", "then")
                    clauses.append((c, self.block()))
                elif self.accept("kw", "else"):
                    els = self.block()
                else:
                    break
            self.expect("kw", "end")
            return ("if", clauses, els)
        if self.accept("kw", "for"):
            n1 = self.expect("name")
            if self.accept("op", "="):
                a = self.expr(); self.expect("op", ",")
                b = self.expr()
                c = self.expr() if self.accept("op", ",") else ("num", 1.0)
                self.expect("kw", "do"); body = self.block(); self.expect("kw", "end")
                return ("fornum", n1, a, b, c, body)
            names = [n1]
            while self.accept("op", ","):
                names.append(self.expect("name"))
            self.expect("kw", "in")
            exprs = self.exprlist()
            self.expect("kw", "do"); body = self.block(); self.expect("kw", "end")
            return ("forin", names, exprs, body)
        if self.accept("kw", "do"):
            body = self.block(); self.expect("kw", "end")
            return ("do", body)
        # expression statement: assignment or call
        target = self.suffixedexp()
        if self.check("op", "=") or self.check("op", ","):
            targets = [target]
            while self.accept("op", ","):
                targets.append(self.suffixedexp())
            self.expect("op", "=")
            return ("assign", targets, self.exprlist())
        if target[0] != "call":
            raise SyntaxError("lua: syntax error (expression statement must be a call)")
        return ("callstat", target)

    def exprlist(self):
        exprs = [self.expr()]
        while self.accept("op", ","):
            exprs.append(self.expr())
        return exprs

    def primaryexp(self):
        if self.check("name"):
            return ("name", self.expect("name"))
        if self.accept("op", "("):
            e = self.expr()
            self.expect("op", ")")
            return ("paren", e)
        raise SyntaxError(f"lua: unexpected {self.peek()}")

    def suffixedexp(self):
        e = self.primaryexp()
        while True:
            if self.accept("op", "."):
                e = ("index", e, ("str", self.expect("name")))
            elif self.accept("op", "["):
                k = self.expr(); self.expect("op", "]")
                e = ("index", e, k)
            elif self.check("op", "("):
                self.i += 1
                args = [] if self.check("op", ")") else self.exprlist()
                self.expect("op", ")")
                e = ("call", e, args)
            elif self.check("op", "{") or self.check("str"):
                args = [self.simpleexp()]
                e = ("call", e, args)
            else:
                return e

    def funcbody(self):
        self.expect("op", "(")
        params = []
        if not self.check("op", ")"):
            params.append(self.expect("name"))
            while self.accept("op", ","):
                params.append(self.expect("name"))
        self.expect("op", ")")
        body = self.block()
        self.expect("kw", "end")
        return ("function", params, body)

    def simpleexp(self):
        tk = self.peek()
        if tk[0] == "num":
            self.i += 1
            return ("num", lua_str2number(tk[1]))
        if tk[0] == "str":
            self.i += 1
            return ("str", unescape(tk[1][1:-1]))
        if self.accept("kw", "nil"):
            return ("nil",)
        if self.accept("kw", "true"):
            return ("true",)
        if self.accept("kw", "false"):
            return ("false",)
        if self.accept("kw", "function"):
            return self.funcbody()
        if self.accept("op", "{"):
            items = []  # ("pos", e) | ("key", kexpr, vexpr)
            while not self.check("op", "}"):
                if self.check("name") and self.peek(1) == ("op", "="):
                    k = self.expect("name"); self.expect("op", "=")
                    items.append(("key", ("str", k), self.expr()))
                elif self.accept("op", "["):
                    k = self.expr(); self.expect("op", "]"); self.expect("op", "=")
                    items.append(("key", k, self.expr()))
                else:
                    items.append(("pos", self.expr()))
                if not (self.accept("op", ",") or self.accept("op", ";")):
                    break
            self.expect("op", "}")
            return ("table", items)
        return self.suffixedexp()

    def expr(self, limit=0):
        if self.check("kw", "not") or self.check("op", "-") or self.check("op", "#"):
            op = self.peek()[1]
            self.i += 1
            left = ("unop", op, self.expr(_UNARY_PRI))
        else:
            left = self.simpleexp()
        while True:
            tk = self.peek()
            op = tk[1] if tk[0] in ("op", "kw") else None
            if op not in _BINPRI or _BINPRI[op][0] <= limit:
                return left
            self.i += 1
            right = self.expr(_BINPRI[op][1])
            left = ("binop", op, left, right)


def unescape(s: str) -> str:
    return re.sub(r"\\(.)", lambda m: {"n": "\n", "t": "\t", "\\": "\\", "'": "'", '"': '"'}.get(
        m.group(1), m.group(1)), s)


# ============================================================== Lua values & semantics


class LuaTable:
    def __init__(self):
        self.h: Dict[Any, Any] = {}

    def get(self, k):
        if isinstance(k, float) and k.is_integer():
            k = float(k)
        return self.h.get(k)

    def set(self, k, v):
        if k is None:
            raise LuaError("table index is nil")
        if v is None:
            self.h.pop(k, None)
        else:
            self.h[k] = v

    def length(self) -> int:
        n = 0
        while (float(n + 1)) in self.h:
            n += 1
        return n


class LuaFunction:
    def __init__(self, params, body, env):
        self.params, self.body, self.env = params, body, env


class LuaError(RuntimeError):
    pass


def lua_str2number(s: str) -> Optional[float]:
    """``luaO_str2d``: strtod (decimal or 0x hex), surrounding whitespace allowed."""
    t = s.strip()
    try:
        if re.fullmatch(r"0[xX][0-9a-fA-F]+", t):
            return float(int(t, 16))
        if re.fullmatch(r"[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?", t) or \
                t.lower() in ("inf", "-inf", "+inf", "nan", "infinity", "-infinity"):
            return float(t)
    except ValueError:
        return None
    return None


def lua_tostring(v) -> str:
    if v is None:
        return "nil"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float):
        if math.isinf(v):
            return "inf" if v > 0 else "-inf"
        if math.isnan(v):
            return "nan" if math.copysign(1, v) > 0 else "-nan"
        return "%.14g" % v                     # LUA_NUMBER_FMT
    if isinstance(v, str):
        return v
    return f"table: {id(v):#x}"


def tonum_arith(v):
    if isinstance(v, float):
        return v
    if isinstance(v, str):
        n = lua_str2number(v)
        if n is not None:
            return n
    raise LuaError(f"attempt to perform arithmetic on a {type_name(v)} value")


def type_name(v):
    if v is None:
        return "nil"
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, float):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, LuaTable):
        return "table"
    return "function"


def truthy(v) -> bool:
    return not (v is None or v is False)


class _Return(Exception):
    def __init__(self, values):
        self.values = values


class Env:
    def __init__(self, parent=None):
        self.vars: Dict[str, Any] = {}
        self.parent = parent

    def lookup(self, name):
        e = self
        while e is not None:
            if name in e.vars:
                return e
            e = e.parent
        return None


class Interpreter:
    def __init__(self, globals_: Dict[str, Any]):
        self.G = Env()
        self.G.vars.update(globals_)

    def run(self, ast):
        try:
            self.exec_block(ast, Env(self.G))
        except _Return as r:
            return r.values
        return []

    # ---------------------------------------------------------------- statements
    def exec_block(self, stmts, env):
        for st in stmts:
            self.exec_stmt(st, env)

    def exec_stmt(self, st, env):
        kind = st[0]
        if kind == "local":
            vals = self.eval_list(st[2], env)
            for i, name in enumerate(st[1]):
                env.vars[name] = vals[i] if i < len(vals) else None
        elif kind == "assign":
            vals = self.eval_list(st[2], env)
            for i, tgt in enumerate(st[1]):
                self.assign(tgt, vals[i] if i < len(vals) else None, env)
        elif kind == "callstat":
            self.eval(st[1], env, multi=True)
        elif kind == "if":
            for cond, body in st[1]:
                if truthy(self.eval(cond, env)):
                    self.exec_block(body, Env(env))
                    return
            if st[2] is not None:
                self.exec_block(st[2], Env(env))
        elif kind == "forin":
            f, s, var = (self.eval_list(st[2], env) + [None, None, None])[:3]
            while True:
                vals = self.call(f, [s, var])
                vals = vals + [None] * (len(st[1]) - len(vals))
                if vals[0] is None:
                    break
                var = vals[0]
                inner = Env(env)
                for n, v in zip(st[1], vals):
                    inner.vars[n] = v
                self.exec_block(st[3], inner)
        elif kind == "fornum":
            a, b, c = (tonum_arith(self.eval(x, env)) for x in st[2:5])
            i = a
            while (c > 0 and i <= b) or (c <= 0 and i >= b):
                inner = Env(env)
                inner.vars[st[1]] = i
                self.exec_block(st[5], inner)
                i = i + c
        elif kind == "do":
            self.exec_block(st[1], Env(env))
        elif kind == "return":
            raise _Return(self.eval_list(st[1], env))
        else:
            raise LuaError(f"unsupported statement {kind}")

    def assign(self, tgt, val, env):
        if tgt[0] == "name":
            e = env.lookup(tgt[1])
            (e if e is not None else self.G).vars[tgt[1]] = val
        elif tgt[0] == "index":
            t = self.eval(tgt[1], env)
            if not isinstance(t, LuaTable):
                raise LuaError(f"attempt to index a {type_name(t)} value")
            t.set(self.key(self.eval(tgt[2], env)), val)
        else:
            raise LuaError("cannot assign")

    @staticmethod
    def key(k):
        return float(k) if isinstance(k, float) else k

    # ---------------------------------------------------------------- expressions
    def eval_list(self, exprs, env):
        out = []
        for i, e in enumerate(exprs):
            if i == len(exprs) - 1 and e[0] == "call":
                out.extend(self.eval(e, env, multi=True))
            else:
                out.append(self.eval(e, env))
        return out

    def eval(self, e, env, multi=False):
        k = e[0]
        if k == "num":
            return e[1]
        if k == "str":
            return e[1]
        if k == "nil":
            return None
        if k == "true":
            return True
        if k == "false":
            return False
        if k == "name":
            en = env.lookup(e[1])
            return en.vars[e[1]] if en is not None else None
        if k == "paren":
            return self.eval(e[1], env)
        if k == "index":
            t = self.eval(e[1], env)
            if isinstance(t, LuaTable):
                return t.get(self.key(self.eval(e[2], env)))
            raise LuaError(f"attempt to index a {type_name(t)} value")
        if k == "call":
            f = self.eval(e[1], env)
            args = self.eval_list(e[2], env)
            res = self.call(f, args)
            return res if multi else (res[0] if res else None)
        if k == "function":
            return LuaFunction(e[1], e[2], env)
        if k == "table":
            t = LuaTable()
            n = 0
            for idx, item in enumerate(e[1]):
                if item[0] == "pos":
                    if idx == len(e[1]) - 1 and item[1][0] == "call":
                        vals = self.eval(item[1], env, multi=True)
                    else:
                        vals = [self.eval(item[1], env)]
                    for v in vals:
                        n += 1
                        t.set(float(n), v)
                else:
                    t.set(self.key(self.eval(item[1], env)), self.eval(item[2], env))
            return t
        if k == "unop":
            v = self.eval(e[2], env)
            if e[1] == "not":
                return not truthy(v)
            if e[1] == "-":
                return -tonum_arith(v)
            if e[1] == "#":
                if isinstance(v, str):
                    return float(len(v.encode()))
                if isinstance(v, LuaTable):
                    return float(v.length())
                raise LuaError(f"attempt to get length of a {type_name(v)} value")
        if k == "binop":
            op = e[1]
            if op == "and":
                a = self.eval(e[2], env)
                return self.eval(e[3], env) if truthy(a) else a
            if op == "or":
                a = self.eval(e[2], env)
                return a if truthy(a) else self.eval(e[3], env)
            a, b = self.eval(e[2], env), self.eval(e[3], env)
            return binop(op, a, b)
        raise LuaError(f"unsupported expression {k}")

    def call(self, f, args):
        if callable(f) and not isinstance(f, LuaFunction):
            r = f(*args)
            return list(r) if isinstance(r, tuple) else [r]
        if isinstance(f, LuaFunction):
            env = Env(f.env)
            for i, p in enumerate(f.params):
                env.vars[p] = args[i] if i < len(args) else None
            try:
                self.exec_block(f.body, env)
            except _Return as r:
                return r.values
            return []
        raise LuaError(f"attempt to call a {type_name(f)} value")


def binop(op, a, b):
    if op in ("+", "-", "*", "/", "%", "^"):
        x, y = tonum_arith(a), tonum_arith(b)
        if op == "+":
            return x + y
        if op == "-":
            return x - y
        if op == "*":
            return x * y
        if op == "/":
            if y == 0.0:
                if x == 0.0 or math.isnan(x):
                    return math.nan
                return math.copysign(math.inf, x) * math.copysign(1.0, y)
            return x / y
        if op == "%":
            return x - math.floor(x / y) * y     # luai_nummod
        return math.pow(x, y)
    if op == "..":
        def s(v):
            if isinstance(v, (str, float)) and not isinstance(v, bool):
                return lua_tostring(v)
            raise LuaError(f"attempt to concatenate a {type_name(v)} value")
        return s(a) + s(b)
    if op == "==":
        return type_name(a) == type_name(b) and a == b
    if op == "~=":
        return not (type_name(a) == type_name(b) and a == b)
    # order comparisons: numbers with numbers, strings with strings, else error
    if isinstance(a, float) and isinstance(b, float) and not isinstance(a, bool) and not isinstance(b, bool):
        pass
    elif isinstance(a, str) and isinstance(b, str):
        pass
    else:
        raise LuaError(f"attempt to compare {type_name(a)} with {type_name(b)}")
    if op == "<":
        return a < b
    if op == "<=":
        return a <= b
    if op == ">":
        return a > b
    return a >= b


# ============================================================== Lua standard library


def _math_max(*args):
    dmax = tonum_check(args[0])
    for a in args[1:]:
        d = tonum_check(a)
        if d > dmax:
            dmax = d
    return dmax


def _math_min(*args):
    dmin = tonum_check(args[0])
    for a in args[1:]:
        d = tonum_check(a)
        if d < dmin:
            dmin = d
    return dmin


def tonum_check(v):  # luaL_checknumber: numbers and numeric strings
    return tonum_arith(v)


def _tonumber(v, base=None):
    if isinstance(v, float) and not isinstance(v, bool):
        return v
    if isinstance(v, str):
        return lua_str2number(v)
    return None


def _ipairs(t):
    def it(tbl, i):
        i = i + 1.0
        v = tbl.get(i)
        return (None,) if v is None else (i, v)
    return it, t, 0.0


def stdlib() -> Dict[str, Any]:
    m = LuaTable()
    m.set("max", _math_max)
    m.set("min", _math_min)
    m.set("ceil", lambda x: float(math.ceil(tonum_check(x))))
    m.set("floor", lambda x: float(math.floor(tonum_check(x))))
    return {"math": m, "tonumber": _tonumber, "tostring": lua_tostring, "ipairs": _ipairs,
            "type": type_name}


# ============================================================== mock Redis


def redis_format_number(x: float) -> str:
    """Lua number -> Redis command argument (script_lua.c): integers via ll2string, other
    values with round-trip precision (fpconv_dtoa in Redis 7, "%.17g" before)."""
    if math.isfinite(x) and x == int(x) and -2**63 <= x < 2**63:
        return str(int(x))
    return repr(x)


class MockRedis:
    """Key space of hashes with TTLs; time is injected per script call (``now_us``)."""

    def __init__(self):
        self.hashes: Dict[str, Dict[str, str]] = {}
        self.expire_at_ms: Dict[str, int] = {}
        self.now_us = 0

    @property
    def now_ms(self):
        return self.now_us // 1000

    def _expire_if_needed(self, key):
        at = self.expire_at_ms.get(key)
        if at is not None and self.now_ms > at:
            self.hashes.pop(key, None)
            self.expire_at_ms.pop(key, None)

    def call(self, cmd, *args):
        cmd = str(cmd).upper()
        sargs = [a if isinstance(a, str) else redis_format_number(a) for a in args]
        if cmd == "TIME":
            sec, usec = divmod(self.now_us, 1_000_000)
            t = LuaTable()
            t.set(1.0, str(sec))
            t.set(2.0, str(usec))
            return t
        if cmd == "HGETALL":
            key = sargs[0]
            self._expire_if_needed(key)
            t = LuaTable()
            i = 0.0
            for f, v in self.hashes.get(key, {}).items():
                t.set(i + 1, f)
                t.set(i + 2, v)
                i += 2
            return t
        if cmd == "HSET":
            key = sargs[0]
            self._expire_if_needed(key)
            h = self.hashes.setdefault(key, {})
            added = 0
            for f, v in zip(sargs[1::2], sargs[2::2]):
                added += f not in h
                h[f] = v
            return float(added)
        if cmd == "EXPIRE":
            key, secs = sargs[0], int(sargs[1])
            self._expire_if_needed(key)
            if key not in self.hashes:
                return 0.0
            self.expire_at_ms[key] = self.now_ms + secs * 1000
            return 1.0
        raise LuaError(f"unsupported redis command {cmd}")


def lua_to_resp(v):
    """Redis' Lua -> RESP reply conversion (script_lua.c luaReplyToRedisReply)."""
    if isinstance(v, bool):
        return 1 if v else None
    if isinstance(v, float):
        return int(v)                      # (long long) cast: truncation
    if isinstance(v, str):
        return v.encode()
    if v is None:
        return None
    if isinstance(v, LuaTable):
        out, i = [], 1.0
        while True:
            e = v.get(i)
            if e is None:
                break
            out.append(lua_to_resp(e))
            i += 1
        return out
    raise LuaError("unsupported reply type")


class ScriptRunner:
    """One prepared script (C# interpolation + ARGV rewrite) executed per call."""

    def __init__(self, script_text: str, redis: MockRedis):
        self.ast = Parser(script_text).chunk()
        self.redis = redis

    def evaluate(self, argv: List[str], now_us: int):
        self.redis.now_us = now_us
        rt = LuaTable()
        rt.set("call", self.redis.call)
        g = stdlib()
        argv_t = LuaTable()
        for i, a in enumerate(argv, start=1):
            argv_t.set(float(i), a)
        g.update({"redis": rt, "ARGV": argv_t, "KEYS": LuaTable()})
        vals = Interpreter(g).run(self.ast)
        return lua_to_resp(vals[0] if vals else None)


# ============================================================== the reference's scripts

REF_ROOT = "/root/reference/DistributedRateLimiting.Redis"
TB_CS = REF_ROOT + "/TokenBucket/RedisTokenBucketRateLimiter.cs"
APPROX_CS = REF_ROOT + "/ApproximateTokenBucket/RedisApproximateTokenBucketRateLimiter.cs"


class ReferenceTokenBucket:
    """``RedisTokenBucketRateLimiter.WaitAsyncCore`` (TB:58-82) over the mock Redis, per key
    (``BucketId = InstanceName + resourceID``, PTB:42)."""

    def __init__(self, capacity: int, fill_rate: float, cs_path: str = TB_CS):
        tmpl = extract_script(cs_path, "GetAcquireLuaScript")
        text = prepare_script(tmpl, {"capacity": capacity, "fillRate": fill_rate},
                              ["BucketId", "PermitCount"])
        self.redis = MockRedis()
        self.runner = ScriptRunner(text, self.redis)

    def acquire(self, key: int, permits: int, ts_us: int):
        raw = self.runner.evaluate([f"tb:{key}", str(permits)], ts_us)   # TB:63
        result = [0 if x is None else int(x) for x in raw]              # (int[])rawResult, nil->0
        if len(result) == 0:
            return False, 0                                             # TB:65-69
        remaining = result[1] if len(result) >= 2 else 0                # TB:71-74
        return result[0] == 1, remaining                                # TB:76-81

    def state(self, key: int, now_us: Optional[int] = None):
        k = f"tb:{key}"
        if now_us is not None:
            self.redis.now_us = now_us
            self.redis._expire_if_needed(k)
        h = self.redis.hashes.get(k)
        if h is None:
            return None
        return float(h["v"]), float(h["t"])


class ReferenceApproxSync:
    """The ApproximateTokenBucket global-tier sync script (A:221-270) and the C# reply
    parse (A:440-443)."""

    def __init__(self, decay_rate: float, cs_path: str = APPROX_CS):
        tmpl = extract_script(cs_path, "GetAcquireLuaScript")
        text = prepare_script(tmpl, {"decayRate": decay_rate}, ["BucketId", "LocalCount"])
        self.redis = MockRedis()
        self.runner = ScriptRunner(text, self.redis)

    def sync(self, bucket: str, local_count: int, now_us: int):
        raw = self.runner.evaluate([bucket, str(local_count)], now_us)   # A:439
        global_score = int(raw[0])                                       # (int)resultArray[0]
        period = float(raw[1].decode())                                  # (double)resultArray[1]
        return global_score, period, raw[1].decode()

    def state(self, bucket: str):
        h = self.redis.hashes.get(bucket)
        if h is None:
            return None
        return {k: float(v) for k, v in h.items()}
