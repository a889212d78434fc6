"""PerfPolicy (consensusml_amd/perf.py): defaults, the library() reference configuration, scoped
switching, validation and the round-2 CML_* environment overrides (CPU only)."""
import json

import pytest

from consensusml_amd import perf


def test_defaults_match_from_env_without_overrides(monkeypatch):
    for k in list(__import__("os").environ):
        if k.startswith("CML_"):
            monkeypatch.delenv(k, raising=False)
    assert perf.PerfPolicy.from_env() == perf.PerfPolicy()
    json.dumps(perf.PerfPolicy().to_dict())          # recorded in bench JSON / checkpoints


def test_library_turns_every_switch_off():
    lib = perf.PerfPolicy.library().validate()
    d = lib.to_dict()
    assert all(v is False for v in d.values() if isinstance(v, bool))
    assert lib.conv1x1_gemm == "miopen" and lib.conv1x1g == "regstage"


def test_env_overrides(monkeypatch):
    monkeypatch.setenv("CML_STEM_POOL_GATHER", "0")
    monkeypatch.setenv("CML_CAT_BNSUMS_MAXC", "64")
    p = perf.PerfPolicy.from_env()
    assert p.stem_pool_gather is False and p.cat_bnsums_maxc == 64
    assert p.replace(stem_pool_gather=True).stem_pool_gather is True


def test_use_policy_is_scoped():
    before = perf.policy()
    with perf.use_policy(before.replace(recompute_tail=not before.recompute_tail)) as p:
        assert perf.policy() is p and p.recompute_tail != before.recompute_tail
    assert perf.policy() == before


@pytest.mark.parametrize("kw", [{"conv1x1_gemm": "cudnn"}, {"conv1x1g": "fast"},
                                {"wgrad1x1_set": "some"}])
def test_validate_rejects_unknown_modes(kw):
    with pytest.raises(ValueError):
        perf.PerfPolicy().replace(**kw).validate()


def test_env_switches_recorded(monkeypatch):
    from consensusml_amd import perf
    monkeypatch.setenv("CML_CONV3P", "0")
    monkeypatch.setenv("CML_BENCH_SELF_LAUNCHED", "1")
    sw = perf.env_switches()
    assert sw.get("CML_CONV3P") == "0"
    assert "CML_BENCH_SELF_LAUNCHED" not in sw
