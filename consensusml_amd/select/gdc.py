"""GDC data acquisition (C01, `JSmith_code/GDC_Data_Download.Rmd:173-390`).

The reference uses the GenomicDataCommons R package: a ``files()`` query filtered to
``type == 'gene_expression'``, ``analysis.workflow_type == 'HTSeq - Counts'`` and the six TARGET
projects, ``results_all()`` with the ``associated_entities`` fields, removal of the files mapped
to two samples (`GDC:208-223`), an ID map CSV (`Manifest_Data/GCD_TARGET_Data_Manifest_AML_NBL_WT_RT.csv`),
a download manifest (`Manifest_Data/TARGET_Manifest_RNAseq_Counts.csv`), ``gdcdata()`` downloads
and ``gdc_clinical()``. Here the same steps talk to the GDC REST API directly:

  ``files_filter``        the GDC ``filters`` JSON of that query
  ``fetch_all``           paged POST /files (``size``/``from``), through an injectable ``opener``
  ``id_map``              flat file x entity table; files with != 1 associated entity dropped
  ``manifest``            gdc-client manifest (id, filename, md5, size, state)
  ``download``            GET /data/<id> per file with md5 verification and atomic writes
  ``clinical``            POST /cases with the demographic / diagnoses expansions, flattened

There is no network in CI: the tests drive ``fetch_all`` / ``download`` with a fake opener and
rebuild the reference's manifest CSV from its ID-map CSV (exact match, 474 files).
"""
from __future__ import annotations

import hashlib
import json
import os
import urllib.request
from typing import Callable, Dict, Iterable, List, Optional, Sequence

import pandas as pd

API = "https://api.gdc.cancer.gov"
TARGET_PROJECTS = ("TARGET-AML", "TARGET-NBL", "TARGET-WT", "TARGET-CCSK", "TARGET-OS", "TARGET-RT")
FILE_FIELDS = ("file_id", "file_name", "submitter_id", "data_type", "data_format", "data_category",
               "type", "experimental_strategy", "file_size", "md5sum", "access", "state",
               "created_datetime", "updated_datetime", "cases.project.project_id",
               "associated_entities.entity_id", "associated_entities.case_id",
               "associated_entities.entity_submitter_id", "associated_entities.entity_type",
               "analysis.analysis_type", "analysis.workflow_type", "analysis.workflow_version")

# opener(url, body_bytes_or_None) -> response bytes
Opener = Callable[[str, Optional[bytes]], bytes]


def _urlopen(url: str, body: Optional[bytes]) -> bytes:
    req = urllib.request.Request(url, data=body,
                                 headers={"Content-Type": "application/json"} if body else {})
    with urllib.request.urlopen(req, timeout=120) as r:
        return r.read()


def files_filter(projects: Sequence[str] = TARGET_PROJECTS, workflow: str = "HTSeq - Counts",
                 file_type: str = "gene_expression") -> Dict:
    def eq(field, value):
        return {"op": "=", "content": {"field": field, "value": value}}
    return {"op": "and", "content": [
        eq("files.type", file_type),
        eq("files.analysis.workflow_type", workflow),
        {"op": "in", "content": {"field": "cases.project.project_id", "value": list(projects)}},
    ]}


def fetch_all(filters: Dict, endpoint: str = "files", fields: Sequence[str] = FILE_FIELDS,
              page_size: int = 500, opener: Opener = _urlopen, api: str = API,
              expand: Sequence[str] = ()) -> List[Dict]:
    """All hits of a query (``results_all``), paging with from/size."""
    hits: List[Dict] = []
    start = 0
    while True:
        body = {"filters": filters, "fields": ",".join(fields), "format": "JSON",
                "size": page_size, "from": start}
        if expand:
            body["expand"] = ",".join(expand)
        data = json.loads(opener(f"{api}/{endpoint}", json.dumps(body).encode()))["data"]
        hits.extend(data["hits"])
        total = data["pagination"]["total"]
        start += len(data["hits"])
        if start >= total or not data["hits"]:
            return hits


def id_map(hits: Iterable[Dict], drop_multi: bool = True) -> pd.DataFrame:
    """One row per (file, associated entity); files whose ``associated_entities`` has more than
    one row are suspect and dropped (`GDC:208`, `GDC:219-223`)."""
    rows = []
    for h in hits:
        ents = h.get("associated_entities") or []
        if drop_multi and len(ents) != 1:
            continue
        base = {k: v for k, v in h.items() if not isinstance(v, (list, dict))}
        cases = h.get("cases") or []
        if cases:
            base["project.project_id"] = cases[0].get("project", {}).get("project_id")
        for e in ents:
            rows.append({**base, **e})
    return pd.DataFrame(rows)


def manifest(idmap: pd.DataFrame) -> pd.DataFrame:
    """gdc-client manifest (``manifest()``): id, filename, md5, size, state — one row per file."""
    m = idmap.drop_duplicates("file_id")
    return pd.DataFrame({"id": m["file_id"].values, "filename": m["file_name"].values,
                         "md5": m["md5sum"].values, "size": m["file_size"].values,
                         "state": m["state"].values})


def write_manifest(m: pd.DataFrame, path: str) -> None:
    """Tab-separated, unquoted (`GDC:251`)."""
    m.to_csv(path, sep="\t", index=False)


def md5_file(path: str, chunk: int = 1 << 20) -> str:
    h = hashlib.md5()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(chunk), b""):
            h.update(b)
    return h.hexdigest()


def download(m: pd.DataFrame, out_dir: str, opener: Opener = _urlopen, api: str = API,
             verify: bool = True) -> List[str]:
    """``gdcdata()``: fetch every manifest row to ``out_dir/<id>/<filename>`` (skipping files
    already present with the right md5), verifying md5 and writing atomically."""
    paths = []
    for r in m.itertuples(index=False):
        d = os.path.join(out_dir, r.id)
        os.makedirs(d, exist_ok=True)
        p = os.path.join(d, r.filename)
        if not (os.path.exists(p) and (not verify or md5_file(p) == r.md5)):
            data = opener(f"{api}/data/{r.id}", None)
            if verify and hashlib.md5(data).hexdigest() != r.md5:
                raise IOError(f"md5 mismatch for {r.id} ({r.filename})")
            tmp = p + ".part"
            with open(tmp, "wb") as f:
                f.write(data)
            os.replace(tmp, p)
        paths.append(p)
    return paths


def clinical(case_ids: Sequence[str], opener: Opener = _urlopen, api: str = API) -> pd.DataFrame:
    """``gdc_clinical()``: demographic + diagnoses of the given cases, one row per case."""
    flt = {"op": "in", "content": {"field": "case_id", "value": list(case_ids)}}
    hits = fetch_all(flt, "cases", fields=("case_id", "submitter_id", "project.project_id"),
                     opener=opener, api=api, expand=("demographic", "diagnoses"))
    rows = []
    for h in hits:
        row = {"case_id": h.get("case_id"), "submitter_id": h.get("submitter_id")}
        for k, v in (h.get("demographic") or {}).items():
            row[f"demographic.{k}"] = v
        diags = h.get("diagnoses") or []
        if diags:
            for k, v in diags[0].items():
                row[f"diagnoses.{k}"] = v
        rows.append(row)
    return pd.DataFrame(rows)
