"""Native host runtime (csrc/runtime) — CPU tests."""
import os
import time
import zlib

import numpy as np
import pytest
import torch

from consensusml_amd import runtime as rt
from consensusml_amd.parallel.flat import ALIGN


def test_plan_buckets_matches_python_flatmodel():
    from consensusml_amd.parallel.flat import FlatModel
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(37, 53), torch.nn.ReLU(), torch.nn.Linear(53, 11),
                            torch.nn.Linear(11, 300))
    for world in (1, 2, 3, 8):
        fm = FlatModel(m, world, bucket_mb=0.01, param_dtype=torch.float32)
        numels = [fm.params[i].numel() for i in range(len(fm.params))][::-1]
        plan = rt.plan_buckets(numels, world, ALIGN, max(int(0.01 * 1024 * 1024 / 4), ALIGN))
        assert plan.total == fm.total
        assert plan.shard_total == fm.shard_total
        assert list(plan.offsets) == [b.offset for b in fm.buckets]
        rev = list(range(len(fm.params)))[::-1]
        assert [plan.param_offsets[k] for k in range(len(rev))] == [fm.param_offset[i] for i in rev]


def test_record_loader_epoch_shuffle_and_shares(tmp_path):
    n, d = 103, 5
    feats = np.arange(n * d, dtype=np.float32).reshape(n, d)
    labels = np.arange(n)
    path = str(tmp_path / "rec.bin")
    rb = rt.write_records(path, feats, labels)
    assert rb == d * 4 + 8
    seen = []
    for rank in range(2):
        L = rt.DeviceLoader(path, (d,), torch.float32, batch=10, device=torch.device("cpu"),
                            rank=rank, world=2, seed=7, threads=3, slots=3)
        assert len(L) == 5          # 51 records per rank, drop_last
        ys = []
        for _ in range(len(L)):
            x, y, ep = L.next()
            assert ep == 0
            torch.testing.assert_close(x[:, 0], (y * d).float())
            ys += y.tolist()
        # second epoch reshuffles
        x, y, ep = L.next()
        assert ep == 1
        L.close()
        assert len(set(ys)) == 50
        seen.append(set(ys))
    assert not (seen[0] & seen[1])   # disjoint rank shares


def test_record_loader_deterministic(tmp_path):
    path = str(tmp_path / "r.bin")
    rt.write_records(path, np.random.rand(64, 3).astype(np.float32), np.arange(64))
    a = rt.native().RecordLoader(path, 20, 8, 0, 1, 3, 2, True)
    b = rt.native().RecordLoader(path, 20, 8, 0, 1, 3, 2, True)
    assert a.batch_indices(0, 1) == b.batch_indices(0, 1)
    assert a.batch_indices(0, 1) != a.batch_indices(1, 1)


def test_watchdog_fires(tmp_path):
    rep = str(tmp_path / "wd.jsonl")
    with rt.Watchdog(0.3, rep) as wd:
        wd.beat(1)
        time.sleep(0.1)
        assert not wd.fired
        time.sleep(0.6)
        assert wd.fired
    assert "watchdog" in open(rep).read()


def test_crc_and_atomic_write(tmp_path):
    p = str(tmp_path / "f.bin")
    data = os.urandom(3 << 20)
    rt.write_file_atomic(p, data)
    assert open(p, "rb").read() == data
    assert rt.crc32_file(p) == zlib.crc32(data)


def test_write_csv(tmp_path):
    p = str(tmp_path / "t.csv")
    rt.write_csv(p, ["g1", "g2"], [("sym", ["A", "B"]), ("x", [1.5, float("nan")])])
    assert open(p).read() == '"","sym","x"\n"g1","A",1.5\n"g2","B",NA\n'
