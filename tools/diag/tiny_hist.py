"""Loss history of the resnet_tiny Krum engine test under the fusion toggles (diagnostic)."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_engine_gpu import _cfg, _info  # noqa: E402
from consensusml_amd.trainer.trainer import ConsensusTrainer  # noqa: E402

cfg = _cfg("krum", "sharded", V=4, f=1, model="resnet_tiny", opt="sgd", lr=0.05)
cfg.model.num_classes = 10
cfg.model.image_size = 32
cfg.batch_per_worker = 4
tr = ConsensusTrainer(cfg, info=_info(torch.device("cuda")))
r = tr.fit(12, log_every=0)
print([round(h, 3) for h in r["history"]])
