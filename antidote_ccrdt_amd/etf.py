"""Erlang external term format (ETF) codec for to_binary/1 and from_binary/1.

Every reference module implements to_binary/1 as term_to_binary(State) and
from_binary/1 as {ok, binary_to_term(Bin)} (e.g. src/antidote_ccrdt_topk_rmv.erl
:156-163, src/antidote_ccrdt_average.erl:103-111).  The mirrors encode the
state term the reference would hold, so a BEAM node decodes the bytes into a
state its own module accepts, and decode whatever shape ERTS produced
(Q16: semantic round trip, not byte identity).

Term mapping (see terms.py): int <-> integer (small/int32/big), Atom <-> atom,
tuple <-> tuple, dict <-> map, list <-> list, bytes <-> binary, float <->
float, GbSet <-> gb_sets {Size, Tree}, ErlSet <-> sets (encoded as the OTP >= 24
map form #{E => []}; the record form of older OTP releases is decoded).
"""
from __future__ import annotations

import struct

VERSION = 131
NEW_FLOAT, SMALL_INT, INT, ATOM, SMALL_TUPLE, LARGE_TUPLE = 70, 97, 98, 100, 104, 105
NIL, STRING, LIST, BINARY, SMALL_BIG, LARGE_BIG, MAP = 106, 107, 108, 109, 110, 111, 116
SMALL_ATOM, ATOM_UTF8, SMALL_ATOM_UTF8 = 115, 118, 119


class Atom(str):
    """An Erlang atom (a str subclass so it compares and hashes like its name)."""

    def __repr__(self):
        return f"Atom({str(self)!r})"


class GbSet(frozenset):
    """A gb_sets set (encoded as the balanced {Size, Tree} of gb_sets:from_ordset/1)."""


class ErlSet(frozenset):
    """A sets set."""


class EtfError(ValueError):
    """badarg of binary_to_term/1."""


# ------------------------------------------------------------------ term order
def _rank(t) -> int:
    # number < atom < reference < fun < port < pid < tuple < map < nil < list < bitstring
    if isinstance(t, bool):
        return 1
    if isinstance(t, (int, float)):
        return 0
    if isinstance(t, Atom) or t is None:
        return 1
    if isinstance(t, tuple):
        return 6
    if isinstance(t, dict):
        return 7
    if isinstance(t, list):
        return 8 if not t else 9
    if isinstance(t, (bytes, bytearray)):
        return 10
    raise TypeError(f"no Erlang term order for {type(t).__name__}")


class _Ord:
    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t

    def __lt__(self, o):
        return compare(self.t, o.t) < 0


def compare(a, b) -> int:
    """Erlang term order (-1, 0, 1) of two terms."""
    ra, rb = _rank(a), _rank(b)
    if ra != rb:
        return -1 if ra < rb else 1
    if ra == 0:
        return (a > b) - (a < b)
    if ra == 1:
        sa, sb = _atom_name(a), _atom_name(b)
        return (sa > sb) - (sa < sb)
    if ra == 6:
        if len(a) != len(b):
            return -1 if len(a) < len(b) else 1
        for x, y in zip(a, b):
            c = compare(x, y)
            if c:
                return c
        return 0
    if ra == 7:  # maps: size, then keys in order, then values
        if len(a) != len(b):
            return -1 if len(a) < len(b) else 1
        ka, kb = sorted(a, key=_Ord), sorted(b, key=_Ord)
        for x, y in zip(ka, kb):
            c = compare(x, y)
            if c:
                return c
        for x, y in zip(ka, kb):
            c = compare(a[x], b[y])
            if c:
                return c
        return 0
    if ra in (8, 9):
        for x, y in zip(a, b):
            c = compare(x, y)
            if c:
                return c
        return (len(a) > len(b)) - (len(a) < len(b))
    return (bytes(a) > bytes(b)) - (bytes(a) < bytes(b))


def _atom_name(a) -> str:
    if a is None:  # the mirrors' None is Erlang's nil ({nil, nil, nil} = Min of an empty state)
        return "nil"
    if isinstance(a, bool):
        return "true" if a else "false"
    return str(a)


def ordset(items) -> list:
    """ordsets:from_list/1: sorted by term order, duplicates removed."""
    out = []
    for x in sorted(items, key=_Ord):
        if not out or compare(out[-1], x) != 0:
            out.append(x)
    return out


# -------------------------------------------------------------------- encoder
def _gb_tree(items: list):
    """gb_sets:from_ordset/1's balance_list/2: {Key, Smaller, Bigger} | nil."""
    it = iter(items)

    def bal(n):
        if n == 0:
            return Atom("nil")
        if n == 1:
            return (next(it), Atom("nil"), Atom("nil"))
        m = n - 1
        s2 = m // 2
        s1 = m - s2
        t1 = bal(s1)
        k = next(it)
        t2 = bal(s2)
        return (k, t1, t2)

    return (len(items), bal(len(items)))


def _enc(t, out: bytearray) -> None:
    if isinstance(t, bool) or t is None or isinstance(t, Atom):
        b = _atom_name(t).encode("utf-8")
        if len(b) > 255:
            raise EtfError("atom too long")
        out += bytes((SMALL_ATOM_UTF8, len(b))) + b
    elif isinstance(t, int):
        if 0 <= t <= 255:
            out += bytes((SMALL_INT, t))
        elif -(1 << 31) <= t < (1 << 31):
            out += bytes((INT,)) + struct.pack(">i", t)
        else:
            mag = abs(t)
            n = (mag.bit_length() + 7) // 8
            body = mag.to_bytes(n, "little")
            if n <= 255:
                out += bytes((SMALL_BIG, n, 1 if t < 0 else 0)) + body
            else:
                out += bytes((LARGE_BIG,)) + struct.pack(">I", n) + bytes((1 if t < 0 else 0,)) + body
    elif isinstance(t, float):
        out += bytes((NEW_FLOAT,)) + struct.pack(">d", t)
    elif isinstance(t, GbSet):
        _enc(_gb_tree(ordset(t)), out)
    elif isinstance(t, ErlSet):
        _enc({e: [] for e in ordset(t)}, out)
    elif isinstance(t, tuple):
        if len(t) <= 255:
            out += bytes((SMALL_TUPLE, len(t)))
        else:
            out += bytes((LARGE_TUPLE,)) + struct.pack(">I", len(t))
        for x in t:
            _enc(x, out)
    elif isinstance(t, dict):
        out += bytes((MAP,)) + struct.pack(">I", len(t))
        for k in sorted(t, key=_Ord):  # any order decodes; sorted = deterministic
            _enc(k, out)
            _enc(t[k], out)
    elif isinstance(t, list):
        if not t:
            out += bytes((NIL,))
        else:
            out += bytes((LIST,)) + struct.pack(">I", len(t))
            for x in t:
                _enc(x, out)
            out += bytes((NIL,))
    elif isinstance(t, (bytes, bytearray)):
        out += bytes((BINARY,)) + struct.pack(">I", len(t)) + bytes(t)
    else:
        raise TypeError(f"cannot encode {type(t).__name__} as an Erlang term")


def term_to_binary(t) -> bytes:
    out = bytearray((VERSION,))
    _enc(t, out)
    return bytes(out)


# -------------------------------------------------------------------- decoder
class _Reader:
    def __init__(self, b: bytes):
        self.b, self.i = memoryview(b), 0

    def take(self, n: int) -> bytes:
        if self.i + n > len(self.b):
            raise EtfError("truncated term")
        v = bytes(self.b[self.i:self.i + n])
        self.i += n
        return v

    def u8(self) -> int:
        return self.take(1)[0]

    def u16(self) -> int:
        return struct.unpack(">H", self.take(2))[0]

    def u32(self) -> int:
        return struct.unpack(">I", self.take(4))[0]


def _atom(name: str):
    return {"true": True, "false": False}.get(name, Atom(name))


def _dec(r: _Reader):
    tag = r.u8()
    if tag == SMALL_INT:
        return r.u8()
    if tag == INT:
        return struct.unpack(">i", r.take(4))[0]
    if tag in (SMALL_BIG, LARGE_BIG):
        n = r.u8() if tag == SMALL_BIG else r.u32()
        sign = r.u8()
        v = int.from_bytes(r.take(n), "little")
        return -v if sign else v
    if tag == NEW_FLOAT:
        return struct.unpack(">d", r.take(8))[0]
    if tag in (ATOM, ATOM_UTF8):
        return _atom(r.take(r.u16()).decode("utf-8" if tag == ATOM_UTF8 else "latin-1"))
    if tag in (SMALL_ATOM, SMALL_ATOM_UTF8):
        return _atom(r.take(r.u8()).decode("utf-8" if tag == SMALL_ATOM_UTF8 else "latin-1"))
    if tag in (SMALL_TUPLE, LARGE_TUPLE):
        n = r.u8() if tag == SMALL_TUPLE else r.u32()
        return tuple(_dec(r) for _ in range(n))
    if tag == NIL:
        return []
    if tag == STRING:  # list of bytes 0..255
        return list(r.take(r.u16()))
    if tag == LIST:
        n = r.u32()
        items = [_dec(r) for _ in range(n)]
        tail = _dec(r)
        if tail != []:
            raise EtfError("improper list")
        return items
    if tag == BINARY:
        return r.take(r.u32())
    if tag == MAP:
        n = r.u32()
        out = {}
        for _ in range(n):
            k = _dec(r)
            out[_hashable(k)] = _dec(r)
        return out
    raise EtfError(f"unsupported external term tag {tag}")


def _hashable(k):
    if isinstance(k, list):
        return tuple(k)
    if isinstance(k, dict):
        raise EtfError("map keys that are maps are not supported")
    return k


def binary_to_term(b: bytes):
    r = _Reader(bytes(b))
    if r.u8() != VERSION:
        raise EtfError("not an external term (version byte)")
    t = _dec(r)
    if r.i != len(r.b):
        raise EtfError("trailing bytes after the term")
    return t


# ------------------------------------------------ sets as the modules hold them
def gb_set_items(t) -> list:
    """Elements of a decoded gb_sets term {Size, Tree} (in-order walk)."""
    if not (isinstance(t, tuple) and len(t) == 2 and isinstance(t[0], int)):
        raise EtfError("not a gb_sets term")
    out, stack, node = [], [], t[1]
    while stack or node != Atom("nil"):
        while node != Atom("nil"):
            if not (isinstance(node, tuple) and len(node) == 3):
                raise EtfError("not a gb_sets tree node")
            stack.append(node)
            node = node[1]
        node = stack.pop()
        out.append(node[0])
        node = node[2]
    if len(out) != t[0]:
        raise EtfError("gb_sets size does not match its tree")
    return out


def sets_items(t) -> list:
    """Elements of a decoded sets term: the OTP >= 24 map form #{E => []} or
    the record form {set, Size, N, MaxN, BSize, ExpSize, ConSize, Empty, Segs}."""
    if isinstance(t, dict):
        return list(t)
    if isinstance(t, tuple) and len(t) == 9 and t[0] == Atom("set"):
        out = []
        for seg in t[8]:
            for bucket in seg:
                out.extend(bucket)
        if len(out) != t[1]:
            raise EtfError("sets size does not match its segments")
        return out
    raise EtfError("not a sets term")
