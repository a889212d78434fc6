"""C01 GDC acquisition without network: fake opener for paging / downloads, and the reference's own
manifest rebuilt from its ID-map CSV (`Manifest_Data/*.csv`, plain CSV)."""
import hashlib
import json
import os

import pandas as pd
import pytest

from consensusml_amd.select import gdc

REF = "/root/reference/Manifest_Data"
ENT = ["entity_id", "case_id", "entity_submitter_id", "entity_type"]


def _hits_from_idmap(df):
    hits = []
    for r in df.to_dict("records"):
        h = {k: v for k, v in r.items() if k not in ENT and k != "project.project_id"}
        h["cases"] = [{"project": {"project_id": r["project.project_id"]}}]
        h["associated_entities"] = [{k: r[k] for k in ENT}]
        hits.append(h)
    return hits


def _pager(hits, page):
    calls = []

    def opener(url, body):
        q = json.loads(body)
        calls.append(q)
        chunk = hits[q["from"]:q["from"] + q["size"]]
        return json.dumps({"data": {"hits": chunk, "pagination": {"total": len(hits)}}}).encode()
    return opener, calls


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference manifests not present")
def test_manifest_matches_reference():
    idm = pd.read_csv(os.path.join(REF, "GCD_TARGET_Data_Manifest_AML_NBL_WT_RT.csv"))
    ref = pd.read_csv(os.path.join(REF, "TARGET_Manifest_RNAseq_Counts.csv"))
    hits = _hits_from_idmap(idm)
    # one suspect file mapped to two samples must be dropped
    bad = dict(hits[0], file_id="dup", associated_entities=hits[0]["associated_entities"] * 2)
    opener, calls = _pager(hits + [bad], 100)
    got_hits = gdc.fetch_all(gdc.files_filter(), opener=opener, page_size=100)
    assert len(calls) == 5 and len(got_hits) == 475
    m = gdc.id_map(got_hits)
    assert len(m) == 474 and (m["project.project_id"].value_counts()["TARGET-AML"] == 187)
    man = gdc.manifest(m)
    pd.testing.assert_frame_equal(man.reset_index(drop=True), ref, check_dtype=False)


def test_filter_and_download(tmp_path):
    f = gdc.files_filter(["TARGET-AML"])
    assert f["content"][1]["content"]["value"] == "HTSeq - Counts"
    blobs = {"a": b"ENSG1\t5\nENSG2\t7\n", "b": b"ENSG1\t1\nENSG2\t0\n"}
    m = pd.DataFrame({"id": ["a", "b"], "filename": ["a.htseq.counts", "b.htseq.counts"],
                      "md5": [hashlib.md5(blobs[k]).hexdigest() for k in "ab"], "size": [1, 1],
                      "state": ["released"] * 2})
    fetched = []

    def opener(url, body):
        fetched.append(url)
        return blobs[url.rsplit("/", 1)[1]]
    paths = gdc.download(m, str(tmp_path), opener=opener)
    assert [open(p, "rb").read() for p in paths] == [blobs["a"], blobs["b"]]
    gdc.download(m, str(tmp_path), opener=opener)          # cached: no refetch
    assert len(fetched) == 2
    m.loc[0, "md5"] = "0" * 32
    os.remove(paths[0])
    with pytest.raises(IOError):
        gdc.download(m, str(tmp_path), opener=opener)
    gdc.write_manifest(m, str(tmp_path / "man.txt"))
    assert open(tmp_path / "man.txt").readline().startswith("id\tfilename")
