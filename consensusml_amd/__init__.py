"""consensusml_amd — an MI355X-native consensus engine (robust data-parallel training and
ConsensusML-style feature-selection consensus) on PyTorch-ROCm + hand-written HIP/CDNA4 kernels
+ RCCL over xGMI. See README.md and SURVEY.md."""
from .config import (AggConfig, FaultConfig, ModelConfig, OptimConfig, TopologyConfig,
                     TrainConfig)

__version__ = "0.1.0"

__all__ = ["AggConfig", "FaultConfig", "ModelConfig", "OptimConfig", "TopologyConfig",
           "TrainConfig", "__version__"]


def __getattr__(name):   # lazy heavy imports
    if name == "ConsensusTrainer":
        from .trainer.trainer import ConsensusTrainer
        return ConsensusTrainer
    if name == "ConsensusEngine":
        from .parallel.engine import ConsensusEngine
        return ConsensusEngine
    raise AttributeError(name)
