"""Data-only reader for R's serialization format (``.rda`` / ``.RData`` from ``save()``, ``.rds``).

The reference persists every stage as R objects: the analysis container
(``composite_code/rnotebook/data/sesetfilt_degseahack_targetaml.rda``, loaded at
`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:409-415`), the biomaRt annotation
(``dfens_v95hg38_bmart.rda``, `composite_code/rnotebook/seobjects/make_seobj_targetaml.R:104-157`)
and the per-model result lists (``svm4reps_resultslist.rda`` ``:673``, ``lasso_resultslist.rda``
``:778``, ``rf_noboost_2k5k10ktrees_allresultslist.rda`` ``:1069``, ``xgb_resultslist.rda``
``:1239``). This module decodes that format byte by byte -- XDR (big-endian) streams of format
version 2 or 3, gzip / bzip2 / xz compressed or plain -- into inert Python values. Nothing in the
file is ever evaluated: R functions, promises, byte code and language objects become inert
``RLanguage`` placeholders (their bytes are consumed and discarded, never run), and environments
are decoded only as data (their variable frame), never as scopes. ``strict=True`` refuses such
objects outright instead (RDataError). Reference-class containers (Bioconductor ``Assays``), model
fits with formula environments and the like do hold functions, which is why the default decodes
past them.

Value mapping:
  NULL -> None;  logical -> RVector(bool / int with NA);  integer -> RVector(int32);
  double -> RVector(float64);  complex -> RVector(complex128);  character -> RVector(list of str
  or None);  list (VECSXP) -> RList;  pairlist -> RPairList;  S4 object -> RS4 (slots = attrs);
  environment -> REnvironment;  symbol -> RSymbol;  raw -> RVector(uint8).
Every R value keeps its attributes (``.attrs``: names, dim, dimnames, class, levels, row.names,
S4 slots ...). Helpers turn the common shapes into numpy / pandas: ``as_array``, ``as_frame``,
``factor_labels``, ``names``.

The ALTREP encodings R >= 3.5 writes for compact sequences, deferred strings and wrappers are
expanded to plain vectors.
"""
from __future__ import annotations

import bz2
import gzip
import lzma
import struct
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

NA_INTEGER = -2147483648

# SEXP types
NILSXP, SYMSXP, LISTSXP, CLOSXP, ENVSXP, PROMSXP, LANGSXP = 0, 1, 2, 3, 4, 5, 6
SPECIALSXP, BUILTINSXP, CHARSXP, LGLSXP, INTSXP, REALSXP, CPLXSXP = 7, 8, 9, 10, 13, 14, 15
STRSXP, DOTSXP, VECSXP, EXPRSXP, BCODESXP, EXTPTRSXP, WEAKREFSXP = 16, 17, 19, 20, 21, 22, 23
RAWSXP, S4SXP = 24, 25
# serialization pseudo-types
REFSXP, NILVALUE_SXP, GLOBALENV_SXP, UNBOUNDVALUE_SXP, MISSINGARG_SXP = 255, 254, 253, 252, 251
BASENAMESPACE_SXP, NAMESPACESXP, PACKAGESXP, PERSISTSXP = 250, 249, 248, 247
CLASSREFSXP, GENERICREFSXP, BCREPDEF, EMPTYENV_SXP, BASEENV_SXP = 246, 245, 244, 242, 241
ATTRLANGSXP, ATTRLISTSXP, ALTREP_SXP, BCREPREF = 240, 239, 238, 243

UTF8_MASK, LATIN1_MASK, BYTES_MASK, ASCII_MASK = 1 << 3, 1 << 2, 1 << 1, 1 << 6


import threading as _threading

_STACK_LOCK = _threading.Lock()


class RDataError(ValueError):
    pass


class RObj:
    """Base: every decoded R value carries its attributes."""
    __slots__ = ("attrs",)

    def __init__(self, attrs: Optional[Dict[str, Any]] = None):
        self.attrs = attrs or {}

    @property
    def rclass(self) -> List[str]:
        c = self.attrs.get("class")
        return list(c.values) if isinstance(c, RVector) else []


class RVector(RObj):
    """Atomic vector: ``values`` is a numpy array (a list of str/None for character)."""
    __slots__ = ("values", "rtype")

    def __init__(self, values, rtype: int, attrs=None):
        super().__init__(attrs)
        self.values = values
        self.rtype = rtype

    def __len__(self):
        return len(self.values)

    def __repr__(self):
        v = self.values
        head = list(v[:4]) if len(v) > 4 else list(v)
        return f"RVector(type={self.rtype}, n={len(v)}, {head}{'...' if len(v) > 4 else ''})"


class RList(RObj):
    """Generic vector (R list / expression)."""
    __slots__ = ("items",)

    def __init__(self, items: List[Any], attrs=None):
        super().__init__(attrs)
        self.items = items

    def __len__(self):
        return len(self.items)

    def __getitem__(self, k):
        if isinstance(k, str):
            nm = names(self)
            if nm is None or k not in nm:
                raise KeyError(k)
            return self.items[nm.index(k)]
        return self.items[k]

    def keys(self) -> List[str]:
        return names(self) or []

    def __repr__(self):
        return f"RList(n={len(self.items)}, names={(names(self) or [])[:8]})"


class RPairList(RObj):
    """Pairlist: ordered (tag, value) pairs (tags may be None)."""
    __slots__ = ("pairs",)

    def __init__(self, pairs: List[Tuple[Optional[str], Any]], attrs=None):
        super().__init__(attrs)
        self.pairs = pairs

    def as_dict(self) -> Dict[str, Any]:
        return {k: v for k, v in self.pairs if k is not None}

    def __repr__(self):
        return f"RPairList({[k for k, _ in self.pairs][:8]})"


class RS4(RObj):
    """S4 object: slots are its attributes (``class`` names the S4 class)."""
    __slots__ = ()

    def slot(self, name: str):
        return self.attrs.get(name)

    def __repr__(self):
        return f"RS4(class={self.rclass}, slots={[k for k in self.attrs if k != 'class']})"


class REnvironment(RObj):
    """Environment decoded as data: its variable frame (never used as a scope)."""
    __slots__ = ("frame", "locked")

    def __init__(self):
        super().__init__(None)
        self.frame: Dict[str, Any] = {}
        self.locked = False

    def __repr__(self):
        return f"REnvironment({list(self.frame)[:8]})"


class RSymbol:
    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name

    def __repr__(self):
        return f"RSymbol({self.name})"


class RLanguage(RObj):
    """Inert placeholder for a function, call, promise or external pointer (never evaluated)."""
    __slots__ = ("kind",)

    def __init__(self, kind: str, attrs=None):
        super().__init__(attrs)
        self.kind = kind

    def __repr__(self):
        return f"RLanguage({self.kind})"


class RSpecial:
    """A marker value (global env, base namespace, missing argument, ...)."""
    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name

    def __repr__(self):
        return f"RSpecial({self.name})"


def _decompress(raw: bytes) -> bytes:
    if raw[:2] == b"\x1f\x8b":
        return gzip.decompress(raw)
    if raw[:3] == b"BZh":
        return bz2.decompress(raw)
    if raw[:6] == b"\xfd7zXZ\x00":
        return lzma.decompress(raw)
    return raw


# Limits for untrusted input: nesting depth of items (a Python frame chain per level, so a
# crafted deeply nested stream raises RDataError instead of exhausting the C stack) and the
# number of elements an ALTREP compact sequence may expand to (its length is file-supplied and
# costs no stream bytes).
MAX_DEPTH = 8192     # model formulas nest one call level per term: a 1984-gene terms object ~2000
MAX_EXPANDED_ELEMENTS = 1 << 27


class _Reader:
    def __init__(self, buf: bytes, strict: bool = False):
        self.b = memoryview(buf)
        self.p = 0
        self.refs: List[Any] = []
        self.strict = strict
        self.depth = 0

    def _code(self, what: str) -> None:
        if self.strict:
            raise RDataError(f"{what} in the stream: refused (strict data-only mode)")

    # ---------------------------------------------------------------- primitives (XDR)
    def _take(self, n: int) -> memoryview:
        if self.p + n > len(self.b):
            raise RDataError("truncated R serialization stream")
        v = self.b[self.p:self.p + n]
        self.p += n
        return v

    def int(self) -> int:
        return struct.unpack(">i", self._take(4))[0]

    def length(self) -> int:
        n = self.int()
        if n == -1:   # long vector
            hi, lo = self.int(), self.int()
            n = (hi << 32) + (lo & 0xFFFFFFFF)
        if n < 0:
            raise RDataError(f"bad vector length {n}")
        return n

    def header(self) -> None:
        fmt = bytes(self._take(2))
        if fmt != b"X\n":
            raise RDataError(f"only XDR (binary, big-endian) streams are supported, got {fmt!r}")
        version = self.int()
        self.int()   # R version that wrote it
        self.int()   # minimal reader version
        if version == 3:
            n = self.int()
            self._take(n)   # native encoding name
        elif version != 2:
            raise RDataError(f"unsupported serialization version {version}")

    # ---------------------------------------------------------------- items
    def charsxp(self, levels: int) -> Optional[str]:
        n = self.int()
        if n == -1:
            return None
        raw = bytes(self._take(n))
        if levels & LATIN1_MASK:
            return raw.decode("latin-1")
        return raw.decode("utf-8", errors="replace")

    def attributes(self, has_attr: bool) -> Dict[str, Any]:
        if not has_attr:
            return {}
        a = self.item()
        if isinstance(a, RPairList):
            return {k: v for k, v in a.pairs if k is not None}
        return {}

    def item(self) -> Any:
        if self.depth >= MAX_DEPTH:
            raise RDataError(f"items nested deeper than {MAX_DEPTH} levels")
        self.depth += 1
        try:
            return self._item()
        finally:
            self.depth -= 1

    def _item(self) -> Any:
        flags = self.int()
        t = flags & 0xFF
        levels = flags >> 12
        has_attr = bool(flags & (1 << 9))
        has_tag = bool(flags & (1 << 10))
        if t == NILVALUE_SXP or t == NILSXP:
            return None
        if t in (EMPTYENV_SXP, BASEENV_SXP, GLOBALENV_SXP, UNBOUNDVALUE_SXP, MISSINGARG_SXP,
                 BASENAMESPACE_SXP):
            return RSpecial({EMPTYENV_SXP: "emptyenv", BASEENV_SXP: "baseenv",
                             GLOBALENV_SXP: "globalenv", UNBOUNDVALUE_SXP: "unbound",
                             MISSINGARG_SXP: "missing", BASENAMESPACE_SXP: "base"}[t])
        if t == REFSXP:
            idx = flags >> 8
            if idx == 0:
                idx = self.int()
            if not 1 <= idx <= len(self.refs):
                raise RDataError(f"bad reference index {idx}")
            return self.refs[idx - 1]
        if t in (PERSISTSXP, PACKAGESXP, NAMESPACESXP):
            s = self._string_vec()
            v = RSpecial(f"{ {PERSISTSXP: 'persist', PACKAGESXP: 'package', NAMESPACESXP: 'namespace'}[t] }:{':'.join(x or '' for x in s)}")
            self.refs.append(v)
            return v
        if t == SYMSXP:
            name = self.item()
            sym = RSymbol(name if isinstance(name, str) else str(name))
            self.refs.append(sym)
            return sym
        if t == ENVSXP:
            self._code("environment")
            env = REnvironment()
            env.locked = bool(self.int())
            self.refs.append(env)
            self.item()                   # enclosure (not followed: data only)
            frame = self.item()
            hashtab = self.item()
            attr = self.item()
            for src in (frame,):
                if isinstance(src, RPairList):
                    env.frame.update(src.as_dict())
            if isinstance(hashtab, RList):
                for bucket in hashtab.items:
                    if isinstance(bucket, RPairList):
                        env.frame.update(bucket.as_dict())
            if isinstance(attr, RPairList):
                env.attrs = attr.as_dict()
            return env
        if t in (LISTSXP, LANGSXP, CLOSXP, PROMSXP, DOTSXP, ATTRLANGSXP, ATTRLISTSXP):
            if t in (CLOSXP, PROMSXP):
                self._code("function / promise")
            return self._pairlist(t, flags)
        if t == ALTREP_SXP:
            return self._altrep()
        if t == BCREPDEF:
            raise RDataError("byte-code repeat definition outside byte code")
        if t in (CLASSREFSXP, GENERICREFSXP):
            raise RDataError("unsupported reference type in the stream")
        # ---------------------------------------------------------- vector-like
        if t == CHARSXP:
            return self.charsxp(levels)
        if t == EXTPTRSXP:
            v = RLanguage("externalptr")
            self.refs.append(v)
            self.item()
            self.item()
        elif t == WEAKREFSXP:
            v = RLanguage("weakref")
            self.refs.append(v)
        elif t in (SPECIALSXP, BUILTINSXP):
            n = self.int()
            v = RLanguage("builtin:" + bytes(self._take(n)).decode("latin-1"))
        elif t in (LGLSXP, INTSXP):
            n = self.length()
            arr = np.frombuffer(bytes(self._take(4 * n)), dtype=">i4").astype(np.int32)
            v = RVector(arr, t)
        elif t == REALSXP:
            n = self.length()
            v = RVector(np.frombuffer(bytes(self._take(8 * n)), dtype=">f8").astype(np.float64), t)
        elif t == CPLXSXP:
            n = self.length()
            d = np.frombuffer(bytes(self._take(16 * n)), dtype=">f8").astype(np.float64)
            v = RVector(d[0::2] + 1j * d[1::2], t)
        elif t == STRSXP:
            n = self.length()
            out = []
            for _ in range(n):
                f = self.int()
                if (f & 0xFF) != CHARSXP:
                    raise RDataError("character vector element is not a CHARSXP")
                out.append(self.charsxp(f >> 12))
            v = RVector(out, t)
        elif t in (VECSXP, EXPRSXP):
            n = self.length()
            v = RList([self.item() for _ in range(n)])
        elif t == RAWSXP:
            n = self.length()
            v = RVector(np.frombuffer(bytes(self._take(n)), dtype=np.uint8).copy(), t)
        elif t == S4SXP:
            v = RS4()
        elif t == BCODESXP:
            self._code("byte code")
            reps: List[Any] = [None] * self.int()
            self._bc1(reps)
            v = RLanguage("bytecode")
        else:
            raise RDataError(f"unknown SEXP type {t}")
        v.attrs = self.attributes(has_attr)
        return v

    # byte code is consumed structurally (R serialize.c ReadBC / ReadBCConsts / ReadBCLang) and
    # discarded: only its length matters here
    def _bc1(self, reps: List[Any]) -> None:
        self.item()                      # the instruction vector
        for _ in range(self.int()):      # constant pool
            t = self.int()
            if t == BCODESXP:
                self._bc1(reps)
            elif t in (LANGSXP, LISTSXP, BCREPDEF, BCREPREF, ATTRLANGSXP, ATTRLISTSXP):
                self._bclang(t, reps)
            else:
                self.item()

    def _bclang(self, t: int, reps: List[Any]) -> None:
        if t == BCREPREF:
            self.int()
            return
        if t in (BCREPDEF, LANGSXP, LISTSXP, ATTRLANGSXP, ATTRLISTSXP):
            if t == BCREPDEF:
                self.int()               # position in reps
                t = self.int()
            if t in (ATTRLANGSXP, ATTRLISTSXP):
                self.item()              # attributes
            self.item()                  # tag
            self._bclang(self.int(), reps)   # car
            self._bclang(self.int(), reps)   # cdr
            return
        self.item()

    def _string_vec(self) -> List[Optional[str]]:
        if self.int() != 0:
            raise RDataError("bad string vector header")
        n = self.int()
        out = []
        for _ in range(n):
            f = self.int()
            out.append(self.charsxp(f >> 12))
        return out

    def _pairlist(self, t: int, flags: int):
        """Pairlist-shaped nodes, read iteratively along the CDR chain."""
        pairs: List[Tuple[Optional[str], Any]] = []
        first_attr: Dict[str, Any] = {}
        kind = {LISTSXP: "pairlist", ATTRLISTSXP: "pairlist", LANGSXP: "call",
                ATTRLANGSXP: "call", CLOSXP: "closure", PROMSXP: "promise", DOTSXP: "dots"}[t]
        first = True
        while True:
            has_attr = bool(flags & (1 << 9)) or t in (ATTRLANGSXP, ATTRLISTSXP)
            has_tag = bool(flags & (1 << 10))
            attr = self.attributes(has_attr)
            if first:
                first_attr = attr
            tag = self.item() if has_tag else None
            car = self.item()
            pairs.append((tag.name if isinstance(tag, RSymbol) else
                          (tag if isinstance(tag, str) else None), car))
            first = False
            # CDR: continue the chain without recursion while it is the same pairlist kind
            nf = self.int()
            nt = nf & 0xFF
            if nt in (LISTSXP, ATTRLISTSXP):   # (a call's arguments are a pairlist too)
                flags, t = nf, nt
                continue
            if nt in (NILVALUE_SXP, NILSXP):
                break
            self.p -= 4
            self.item()    # a non-pairlist CDR (language objects): consumed, not kept
            break
        if kind == "pairlist":
            return RPairList(pairs, first_attr)
        return RLanguage(kind, first_attr)

    def _altrep(self):
        info = self.item()
        state = self.item()
        attr = self.item()
        cls = None
        if isinstance(info, RPairList) and info.pairs and isinstance(info.pairs[0][1], RSymbol):
            cls = info.pairs[0][1].name
        v = _expand_altrep(cls, state)
        if v is None:
            raise RDataError(f"unsupported ALTREP class {cls!r}")
        if isinstance(attr, RPairList):
            v.attrs = attr.as_dict()
        return v


def _expand_altrep(cls: Optional[str], state) -> Optional[RObj]:
    if cls in ("compact_intseq", "compact_realseq") and isinstance(state, RVector):
        if len(state.values) < 3:
            raise RDataError(f"{cls} state has {len(state.values)} values, needs 3")
        n = state.values[0]
        if not np.isfinite(n) or not 0 <= n <= MAX_EXPANDED_ELEMENTS:
            raise RDataError(f"{cls} of length {n}: outside [0, {MAX_EXPANDED_ELEMENTS}]")
        n = int(n)
    if cls == "compact_intseq" and isinstance(state, RVector):
        start, step = (int(x) for x in state.values[1:3])
        return RVector((start + step * np.arange(n, dtype=np.int64)).astype(np.int32), INTSXP)
    if cls == "compact_realseq" and isinstance(state, RVector):
        start, step = state.values[1:3]
        return RVector(start + step * np.arange(n, dtype=np.float64), REALSXP)
    if cls == "deferred_string" and isinstance(state, RPairList) and state.pairs:
        src = state.pairs[0][1]
        if isinstance(src, RVector):
            vals = src.values
            if src.rtype == REALSXP:
                out = [None if np.isnan(x) else _r_num_str(x) for x in vals]
            else:
                out = [None if x == NA_INTEGER else str(int(x)) for x in vals]
            return RVector(out, STRSXP)
    if cls and cls.startswith("wrap_"):
        inner = None
        if isinstance(state, RList) and state.items:
            inner = state.items[0]
        elif isinstance(state, RPairList) and state.pairs:
            inner = state.pairs[0][1]
        return inner if isinstance(inner, RObj) else None
    return None


def _r_num_str(x: float) -> str:
    """as.character of a double the way R prints it (15 significant digits)."""
    if float(x).is_integer() and abs(x) < 1e15:
        return str(int(x))
    return f"{x:.15g}"


# ----------------------------------------------------------------------------- public API
def _deep(fn):
    """Run a parse on a thread with a stack sized for MAX_DEPTH item levels (up to ~4 Python
    frames each), so the depth counter -- not the C stack -- is what bounds a crafted stream."""
    import sys
    import threading
    out: Dict[str, Any] = {}

    def run():
        old = sys.getrecursionlimit()
        sys.setrecursionlimit(max(old, 4 * MAX_DEPTH + 500))
        try:
            out["v"] = fn()
        except BaseException as e:   # re-raised on the caller's thread
            out["e"] = e
        finally:
            sys.setrecursionlimit(old)

    # the parse thread's stack, sized from the depth bound: ~4 interpreter frames per nesting
    # level at a few KB each, with headroom (64 MB at MAX_DEPTH 8192). stack_size() is
    # process-wide, so it is set and restored under a lock: a thread another thread starts
    # meanwhile never inherits it by accident
    size = max(32 << 20, 4 * MAX_DEPTH * 2048)
    with _STACK_LOCK:
        prev = threading.stack_size()
        try:
            threading.stack_size(size)
            t = threading.Thread(target=run, name="rdata-parse")
            t.start()
        except (RuntimeError, ValueError, MemoryError) as e:
            raise RDataError(f"cannot start the parse thread with a {size >> 20} MB stack: {e}")
        finally:
            threading.stack_size(prev)
    t.join()
    if "e" in out:
        raise out["e"]
    return out["v"]


def read_rds(path: str, strict: bool = False) -> Any:
    """One object from a ``saveRDS`` file."""
    with open(path, "rb") as fh:
        buf = _decompress(fh.read())
    r = _Reader(buf, strict)
    r.header()
    return _deep(r.item)


def read_rdata(path: str, strict: bool = False) -> Dict[str, Any]:
    """Every object of a ``save()`` file (``.rda`` / ``.RData``), by variable name."""
    with open(path, "rb") as fh:
        buf = _decompress(fh.read())
    if buf[:5] not in (b"RDX2\n", b"RDX3\n"):
        raise RDataError("not an R save() file (missing RDX2/RDX3 magic)")
    r = _Reader(buf[5:], strict)
    r.header()
    top = _deep(r.item)
    if not isinstance(top, RPairList):
        raise RDataError("save() stream does not hold a pairlist of variables")
    return {k: v for k, v in top.pairs if k is not None}


# ----------------------------------------------------------------------------- helpers
def names(x) -> Optional[List[str]]:
    a = getattr(x, "attrs", {}).get("names")
    return list(a.values) if isinstance(a, RVector) else None


def is_na(v: RVector) -> np.ndarray:
    if v.rtype in (LGLSXP, INTSXP):
        return v.values == NA_INTEGER
    if v.rtype == REALSXP:
        return np.isnan(v.values)
    if v.rtype == STRSXP:
        return np.array([s is None for s in v.values])
    return np.zeros(len(v), dtype=bool)


def as_array(v: RVector) -> np.ndarray:
    """Numeric vector / matrix / array as numpy (column-major dims honoured, NA -> nan)."""
    if not isinstance(v, RVector):
        raise TypeError(f"not an atomic vector: {v!r}")
    if v.rtype == STRSXP:
        arr = np.array(v.values, dtype=object)
    elif v.rtype in (LGLSXP, INTSXP):
        arr = v.values.astype(np.float64)
        arr[v.values == NA_INTEGER] = np.nan
    else:
        arr = v.values
    dim = v.attrs.get("dim")
    if isinstance(dim, RVector):
        arr = arr.reshape([int(d) for d in dim.values], order="F")
    return arr


def dimnames(v: RObj) -> Optional[List[Optional[List[str]]]]:
    dn = v.attrs.get("dimnames")
    if isinstance(dn, RList):
        return [list(d.values) if isinstance(d, RVector) else None for d in dn.items]
    return None


def factor_labels(v: RVector) -> List[Optional[str]]:
    lev = v.attrs.get("levels")
    if not isinstance(lev, RVector):
        raise TypeError("not a factor")
    L = lev.values
    return [None if c == NA_INTEGER else L[c - 1] for c in v.values]


def _column(v):
    if isinstance(v, RVector):
        if "levels" in v.attrs:
            return factor_labels(v)
        if v.rtype == STRSXP:
            return list(v.values)
        if v.rtype == LGLSXP:
            out = v.values.astype(object)
            out[v.values == NA_INTEGER] = None
            return [None if x is None else bool(x) for x in out]
        return as_array(v)
    if isinstance(v, RS4) and "listData" in v.attrs:   # nested DataFrame column
        return None
    return None


def row_names(v: RObj) -> Optional[List[str]]:
    rn = v.attrs.get("row.names")
    if isinstance(rn, RVector):
        if rn.rtype == STRSXP:
            return list(rn.values)
        vals = rn.values
        if len(vals) == 2 and vals[0] == NA_INTEGER:   # compact form c(NA, -n)
            return [str(i + 1) for i in range(abs(int(vals[1])))]
        return [str(int(x)) for x in vals]
    return None


def as_frame(v: RObj):
    """data.frame (RList with class data.frame) or S4Vectors DataFrame (RS4 with listData) as a
    pandas DataFrame."""
    import pandas as pd
    if isinstance(v, RS4):
        ld = v.attrs.get("listData")
        rn = v.attrs.get("rownames")
        nrows = v.attrs.get("nrows")
        cols = {}
        if isinstance(ld, RList):
            for k, c in zip(names(ld) or [], ld.items):
                col = _column(c)
                if col is not None:
                    cols[k] = col
        index = list(rn.values) if isinstance(rn, RVector) else None
        df = pd.DataFrame(cols, index=index)
        if not cols and isinstance(nrows, RVector) and index is None:
            df = pd.DataFrame(index=range(int(nrows.values[0])))
        return df
    if isinstance(v, RList):
        cols = {}
        for k, c in zip(names(v) or [], v.items):
            col = _column(c)
            if col is not None:
                cols[k] = col
        return pd.DataFrame(cols, index=row_names(v))
    raise TypeError(f"cannot convert {v!r} to a data frame")


def walk_types(x, depth: int = 0, max_depth: int = 6, out: Optional[list] = None) -> list:
    """(depth, description) lines of an object tree (inspection / debugging)."""
    out = [] if out is None else out
    pad = "  " * depth
    if depth > max_depth:
        return out
    if isinstance(x, RS4):
        out.append(f"{pad}S4 {x.rclass}")
        for k, v in x.attrs.items():
            if k == "class":
                continue
            out.append(f"{pad} @{k}:")
            walk_types(v, depth + 1, max_depth, out)
    elif isinstance(x, RList):
        out.append(f"{pad}list[{len(x)}] names={(names(x) or [])[:6]} class={x.rclass}")
        for v in x.items[:6]:
            walk_types(v, depth + 1, max_depth, out)
    elif isinstance(x, RVector):
        dim = x.attrs.get("dim")
        out.append(f"{pad}vec type={x.rtype} n={len(x)} dim={list(dim.values) if isinstance(dim, RVector) else None} "
                   f"class={x.rclass}")
    elif isinstance(x, REnvironment):
        out.append(f"{pad}env {list(x.frame)[:8]}")
        for v in list(x.frame.values())[:6]:
            walk_types(v, depth + 1, max_depth, out)
    else:
        out.append(f"{pad}{x!r}"[:120])
    return out


# ----------------------------------------------------------------------------- Bioconductor
def _assay_list(se: RS4) -> "RList":
    """The assays of a SummarizedExperiment: a SimpleList held directly (``SimpleAssays``) or in
    the reference-class environment of ``ShallowSimpleListAssays`` (field ``data``, stored as
    ``.->data`` behind the active binding)."""
    a = se.attrs.get("assays")
    cur = a
    for _ in range(4):
        if isinstance(cur, RS4) and "listData" in cur.attrs:
            return cur.attrs["listData"]
        if isinstance(cur, RS4) and "data" in cur.attrs:
            cur = cur.attrs["data"]
            continue
        if isinstance(cur, RS4) and ".xData" in cur.attrs:
            env = cur.attrs[".xData"]
            cur = env.frame.get(".->data", env.frame.get("data")) if isinstance(env, REnvironment) \
                else None
            continue
        break
    raise RDataError("could not locate the assay list of the SummarizedExperiment")


def summarized_experiment(se: RS4) -> Dict[str, Any]:
    """Decode a (Ranged)SummarizedExperiment into plain parts:
    {assays: {name: np.ndarray [genes, samples]}, genes, samples, row_data (DataFrame: the
    rowRanges' mcols, e.g. the DE statistics, plus seqnames / start / end / strand), col_data
    (DataFrame), metadata (dict of str)}."""
    import pandas as pd
    if not isinstance(se, RS4) or not any("SummarizedExperiment" in c for c in se.rclass):
        raise RDataError(f"not a SummarizedExperiment: {se!r}")
    al = _assay_list(se)
    assays, genes, samples = {}, None, None
    for i, (nm, m) in enumerate(zip(names(al) or [None] * len(al), al.items)):
        arr = as_array(m)
        dn = dimnames(m)
        if dn:
            genes = genes or dn[0]
            samples = samples or dn[1]
        assays[nm or f"assay{i + 1}"] = arr
    col = as_frame(se.attrs["colData"]) if "colData" in se.attrs else pd.DataFrame()
    rd = pd.DataFrame()
    rr = se.attrs.get("rowRanges")
    if isinstance(rr, RS4):
        em = rr.attrs.get("elementMetadata")
        if isinstance(em, RS4):
            rd = as_frame(em)
        rg = rr.attrs.get("ranges")
        if isinstance(rg, RS4):
            start = rg.attrs["start"].values
            rd["start"] = start
            rd["end"] = start + rg.attrs["width"].values - 1
            nm = rg.attrs.get("NAMES")
            if genes is None and isinstance(nm, RVector):
                genes = list(nm.values)
        for slot, col_name in (("seqnames", "seqnames"), ("strand", "strand")):
            rle = rr.attrs.get(slot)
            if isinstance(rle, RS4) and "values" in rle.attrs:
                vals = factor_labels(rle.attrs["values"])
                rd[col_name] = np.repeat(np.array(vals, dtype=object),
                                         rle.attrs["lengths"].values.astype(np.int64))
    elif "elementMetadata" in se.attrs:
        rd = as_frame(se.attrs["elementMetadata"])
    if genes is not None and len(rd) == len(genes):
        rd.index = genes
    if samples is None and len(col):
        samples = list(col.index)
    meta = {}
    md = se.attrs.get("metadata")
    if isinstance(md, RList):
        for k, v in zip(names(md) or [], md.items):
            if isinstance(v, RVector) and v.rtype == STRSXP and len(v) == 1:
                meta[k] = v.values[0]
    return {"assays": assays, "genes": genes, "samples": samples, "row_data": rd,
            "col_data": col, "metadata": meta}
