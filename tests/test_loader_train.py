"""Training from record files through the native C++ loader (csrc/runtime) — CPU."""
import torch

from consensusml_amd import TrainConfig
from consensusml_amd.parallel.dist import DistInfo
from consensusml_amd.trainer.trainer import ConsensusTrainer, write_synthetic_records


def test_train_from_native_loader(tmp_path):
    cfg = TrainConfig()
    cfg.dtype = "fp32"
    cfg.virtual_workers = 3
    cfg.agg.rule = "median"
    cfg.model.extra = {"classes": 2}
    cfg.batch_per_worker = 32
    path = str(tmp_path / "mlp.rec")
    rb = write_synthetic_records(cfg, path, 2000)
    assert rb == cfg.model.in_features * 4 + 8
    cfg.data_path = path
    tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, torch.device("cpu"), "none"))
    r = tr.fit(30, log_every=0)
    tr.close()
    assert r["history"][-1] < 0.3 < r["history"][0]
