from .stage import OptimConfig, Stage, StageParams
from .trainer import Trainer, default_distribution

__all__ = ["OptimConfig", "Stage", "StageParams", "Trainer", "default_distribution"]
