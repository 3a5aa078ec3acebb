"""Restricted evaluator for the reference's index strings (``prior_ind``, ``test_ind``,
``train_ind``).

The MATLAB scripts do ``if (ischar(ind)) ind = eval(ind); end`` (process_qsos.m:7-9,53-55,
learn_qso_model.m:16-18) on strings such as (README.md:242-253)

    prior_catalog.in_dr9 & prior_catalog.los_inds(dla_catalog_name) & (prior_catalog.filter_flags == 0)
    (catalog.filter_flags == 0)

Here those strings are parsed by a small recursive-descent parser over exactly that grammar and
evaluated on numpy arrays; nothing is handed to Python's ``eval``.  Grammar (MATLAB precedence,
lowest first):

    expr    := andand ( '||' andand )*
    andand  := or ( '&&' or )*
    or      := and ( '|' and )*
    and     := cmp ( '&' cmp )*
    cmp     := unary ( ('==' | '~=' | '!=' | '<' | '<=' | '>' | '>=') unary )?
    unary   := ('~' | '!' | '-') unary | postfix
    postfix := atom ( '.' NAME | '(' expr ')' )*
    atom    := NAME | NUMBER | 'string' | "string" | 'true' | 'false' | '(' expr ')'

``NAME`` resolves only against the keyword arguments the caller passes (the loaded catalogue
structs and ``dla_catalog_name``); ``struct.field`` reads a variable of a loaded ``.mat`` dict,
and ``map(key)`` looks a key up in a ``containers.Map`` variable (a dict here, matv73.py).
Anything else -- attribute names starting with ``_``, unknown names, calls on non-maps, other
characters -- raises ``IndexExpressionError``.
"""
from __future__ import annotations

import re

import numpy as np


class IndexExpressionError(ValueError):
    """The string is not a valid index expression over the given names."""


_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<num>(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?)
  | (?P<name>[A-Za-z][A-Za-z0-9_]*)
  | (?P<str>'(?:[^']|'')*'|"(?:[^"]|"")*")
  | (?P<op>&&|\|\||==|~=|!=|<=|>=|[&|~!<>().,-])
""", re.VERBOSE)


def _tokenize(s: str):
    pos, out = 0, []
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise IndexExpressionError(f"unexpected character {s[pos]!r} at {pos} in {s!r}")
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        text = m.group(kind)
        if kind == "str":
            q = text[0]
            text = text[1:-1].replace(q + q, q)
        out.append((kind, text))
    out.append(("end", ""))
    return out


def _column(v):
    """A loaded MATLAB column/row vector as a 1-D array (scalars and matrices unchanged)."""
    if isinstance(v, dict):
        return v
    a = np.asarray(v)
    return a.ravel() if a.ndim == 2 and 1 in a.shape else a


class _Map:
    """A ``containers.Map`` variable (stored as a struct keyed by name): ``map(key)``."""

    def __init__(self, d: dict):
        self.d = d

    def lookup(self, key):
        if not isinstance(key, str):
            raise IndexExpressionError("containers.Map keys are strings")
        if key not in self.d:
            raise IndexExpressionError(f"no key {key!r} in map")
        v = self.d[key]
        if isinstance(v, np.ndarray) and v.dtype == object:
            return list(v.ravel(order="F"))
        return _column(v)


class _Struct:
    def __init__(self, d: dict):
        self.d = d

    def field(self, name):
        if name.startswith("_") or name not in self.d:
            raise IndexExpressionError(f"no field {name!r}")
        v = self.d[name]
        return _Map(v) if isinstance(v, dict) else _column(v)


def _wrap(v):
    return _Struct(v) if isinstance(v, dict) else v


class _Parser:
    def __init__(self, text: str, names: dict):
        self.toks = _tokenize(text)
        self.i = 0
        self.names = names

    def peek(self):
        return self.toks[self.i]

    def take(self, text=None):
        tok = self.toks[self.i]
        if text is not None and tok[1] != text:
            raise IndexExpressionError(f"expected {text!r}, got {tok[1]!r}")
        self.i += 1
        return tok

    def parse(self):
        v = self.expr()
        if self.peek()[0] != "end":
            raise IndexExpressionError(f"unexpected {self.peek()[1]!r}")
        return v

    def _binary(self, ops, sub, fn):
        v = sub()
        while self.peek()[0] == "op" and self.peek()[1] in ops:
            self.take()
            v = fn(_arr(v), _arr(sub()))
        return v

    def expr(self):
        return self._binary(("||",), self.andand, np.logical_or)

    def andand(self):
        return self._binary(("&&",), self.or_, np.logical_and)

    def or_(self):
        return self._binary(("|",), self.and_, np.logical_or)

    def and_(self):
        return self._binary(("&",), self.cmp, np.logical_and)

    _CMP = {"==": np.equal, "~=": np.not_equal, "!=": np.not_equal, "<": np.less,
            "<=": np.less_equal, ">": np.greater, ">=": np.greater_equal}

    def cmp(self):
        v = self.unary()
        kind, text = self.peek()
        if kind == "op" and text in self._CMP:
            self.take()
            v = self._CMP[text](_arr(v), _arr(self.unary()))
        return v

    def unary(self):
        kind, text = self.peek()
        if kind == "op" and text in ("~", "!"):
            self.take()
            return np.logical_not(_arr(self.unary()))
        if kind == "op" and text == "-":
            self.take()
            return -_arr(self.unary())
        return self.postfix()

    def postfix(self):
        v = self.atom()
        while True:
            kind, text = self.peek()
            if (kind, text) == ("op", "."):
                self.take()
                k2, name = self.take()
                if k2 != "name":
                    raise IndexExpressionError(f"field name expected after '.', got {name!r}")
                if not isinstance(v, _Struct):
                    raise IndexExpressionError(f"'.{name}' on a non-struct")
                v = v.field(name)
            elif (kind, text) == ("op", "("):
                self.take()
                key = self.expr()
                self.take(")")
                if not isinstance(v, _Map):
                    raise IndexExpressionError("only containers.Map variables can be called")
                v = v.lookup(key)
            else:
                return v

    def atom(self):
        kind, text = self.take()
        if kind == "num":
            return float(text)
        if kind == "str":
            return text
        if kind == "name":
            if text == "true":
                return True
            if text == "false":
                return False
            if text not in self.names:
                raise IndexExpressionError(f"unknown name {text!r}")
            return _wrap(self.names[text])
        if (kind, text) == ("op", "("):
            v = self.expr()
            self.take(")")
            return v
        raise IndexExpressionError(f"unexpected {text!r}")


def _arr(v):
    if isinstance(v, (_Struct, _Map)):
        raise IndexExpressionError("a struct or map is not a value")
    if isinstance(v, list):
        raise IndexExpressionError("a cell array is not a logical value")
    return np.asarray(v)


def evaluate_index_string(text: str, **names) -> np.ndarray:
    """Evaluate one index string over ``names`` (dicts are structs, nested dicts Maps)."""
    v = _Parser(text, names).parse()
    return _arr(v)
