from .comm import DistPipe, LoopbackPipe
from .groups import Mesh, build_mesh, init_distributed
from .pipeline import GradSync, PipelineExecutor, schedule_ops

__all__ = ["DistPipe", "LoopbackPipe", "Mesh", "build_mesh", "init_distributed", "GradSync",
           "PipelineExecutor", "schedule_ops"]
