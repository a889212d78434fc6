"""Crafted R serialization streams: the data-only reader refuses them with RDataError instead
of allocating without bound or exhausting the stack (select/rdata.py limits)."""
import struct

import numpy as np
import pytest

from consensusml_amd.select import rdata as R


def _i(v):
    return struct.pack(">i", v)


def _stream(body: bytes) -> bytes:
    return b"X\n" + _i(2) + _i(0x040000) + _i(0x020300) + body


def _write(tmp_path, body):
    p = tmp_path / "x.rds"
    p.write_bytes(_stream(body))
    return str(p)


def _charsxp(s: str) -> bytes:
    b = s.encode()
    return _i(9) + _i(len(b)) + b


def _altrep(cls: str, vals) -> bytes:
    info = _i(2) + _i(1) + _charsxp(cls) + _i(254)     # pairlist (SYMSXP cls), nil CDR
    state = _i(14) + _i(len(vals)) + b"".join(struct.pack(">d", v) for v in vals)
    return _i(238) + info + state + _i(254)


def test_compact_intseq_expands(tmp_path):
    v = R.read_rds(_write(tmp_path, _altrep("compact_intseq", [5, 3, 2])))
    assert v.values.tolist() == [3, 5, 7, 9, 11]


def test_compact_seq_length_capped(tmp_path):
    for cls in ("compact_intseq", "compact_realseq"):
        with pytest.raises(R.RDataError):
            R.read_rds(_write(tmp_path, _altrep(cls, [1e12, 1, 1])))
        with pytest.raises(R.RDataError):
            R.read_rds(_write(tmp_path, _altrep(cls, [-5, 1, 1])))
        with pytest.raises(R.RDataError):
            R.read_rds(_write(tmp_path, _altrep(cls, [float("nan"), 1, 1])))


def test_deep_nesting_refused(tmp_path):
    depth = R.MAX_DEPTH + 10
    body = (_i(19) + _i(1)) * depth + _i(254)          # list(list(list(... NULL)))
    with pytest.raises(R.RDataError):
        R.read_rds(_write(tmp_path, body))


def test_moderate_nesting_reads(tmp_path):
    body = (_i(19) + _i(1)) * 100 + _i(254)
    v = R.read_rds(_write(tmp_path, body))
    for _ in range(99):
        v = v.items[0]
    assert isinstance(v, R.RList) and v.items == [None]
